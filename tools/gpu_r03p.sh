#!/bin/bash
# suites not rerun since r03k: callers, configs[4], VAD, SortFormer, quantized
set -o pipefail
bash tools/gpu_tests.sh r03p "tests/test_callers.py tests/test_gpu_c4.py tests/test_vad.py tests/test_q5.py tests/test_kquant.py" 0
