#!/bin/bash
# The CPU tests of the libraries' host code (tokenizer, model / GGUF header parsing, GBNF grammar,
# aligner, RTTM, DTW, k-quant expansion, VAD segment rules, ABI structs) against the ASan + UBSan
# build (make sanitize): the reference's WHISPER_SANITIZE_ADDRESS / _UNDEFINED CI jobs
# (ref .github/workflows/build.yml:435-464) restated for the host side of this library.
# Python itself is not instrumented, so the ASan runtime is preloaded; leak checking is off (the
# interpreter and the HIP runtime keep allocations until exit); any ASan or UBSan report aborts
# the process (halt_on_error / -fno-sanitize-recover) and fails the run.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
[ -f "$RT" ] || { echo "no ASan runtime"; exit 1; }
[ -f "$ROOT/open-whisper-kit_amd/lib/san/libwhisper.so" ] || { echo "run make sanitize first"; exit 1; }
export OWK_LIB=$ROOT/open-whisper-kit_amd/lib/san/libwhisper.so
export OWK_SF_LIB=$ROOT/open-whisper-kit_amd/lib/san/libsortformer.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0:alloc_dealloc_mismatch=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
cd "$ROOT"
LD_PRELOAD=$RT python -m pytest -x -q -p no:cacheprovider -m "not gpu" "$@" \
    tests/test_tokenize.py tests/test_grammar.py tests/test_diarize_align.py tests/test_dtw_cpu.py \
    tests/test_abi.py tests/test_kquant.py tests/test_vad.py tests/test_sortformer.py tests/test_sanitize_host.py
