// Minimal ggml type shim for the drop-in whisper.h boundary.
//
// The reference's public header includes "ggml.h" / "ggml-cpu.h" (reference
// include/whisper.h:4-5) only for a few typedefs. This engine contains no ggml; this
// file supplies exactly those types so callers written against the reference header
// (examples/cli, the Swift SDK bridge) compile unchanged:
//   enum ggml_log_level    - reference ggml/include/ggml.h:622
//   ggml_abort_callback    - reference ggml/include/ggml.h:694
//   ggml_log_callback      - reference ggml/include/ggml.h:2651
#pragma once

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ggml_log_level {
    GGML_LOG_LEVEL_NONE  = 0,
    GGML_LOG_LEVEL_DEBUG = 1,
    GGML_LOG_LEVEL_INFO  = 2,
    GGML_LOG_LEVEL_WARN  = 3,
    GGML_LOG_LEVEL_ERROR = 4,
    GGML_LOG_LEVEL_CONT  = 5,
};

// return true to abort the current computation
typedef bool (*ggml_abort_callback)(void * data);

typedef void (*ggml_log_callback)(enum ggml_log_level level, const char * text, void * user_data);

#ifdef __cplusplus
}
#endif
