// Shim: the reference whisper.h includes "ggml-cpu.h" (reference include/whisper.h:5).
// The reference's ggml-cpu.h includes ggml-backend.h (reference ggml/include/ggml-cpu.h:4),
// and callers such as examples/cli/cli.cpp:929 and examples/bench/bench.cpp:168 rely on
// that to see ggml_backend_load_all(); so does this one. See ggml.h in this directory.
#pragma once
#include "ggml.h"
#include "ggml-backend.h"
