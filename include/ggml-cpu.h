// Empty shim: the reference whisper.h includes "ggml-cpu.h" (reference
// include/whisper.h:5) but uses nothing from it. See ggml.h in this directory.
#pragma once
#include "ggml.h"
