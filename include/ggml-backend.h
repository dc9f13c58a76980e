// Shim for the one ggml-backend entry point callers of the reference invoke
// unconditionally: examples/cli/cli.cpp:929 calls ggml_backend_load_all()
// (reference ggml/include/ggml-backend.h:246). This engine has a single built-in
// MI355X backend, so the call is a no-op exported by libwhisper.so.
#pragma once
#include "ggml.h"

#ifdef __cplusplus
extern "C" {
#endif

void ggml_backend_load_all(void);

#ifdef __cplusplus
}
#endif
