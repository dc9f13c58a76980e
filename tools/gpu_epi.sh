#!/bin/bash
# large-tile epilogue change: kernel cross-checks, GEMM timings, full-depth parity, bench
set -o pipefail
TAG=${1:-epi}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k gemm256 -m gpu -v -s --timeout 120 --timeout-method thread > gpurun_out/$TAG/epi.log 2>&1 || { grep -E "max\||FAIL|Error" gpurun_out/$TAG/epi.log | head -30; exit 1; }
grep -E "max\|" gpurun_out/$TAG/epi.log
timeout -k 10 300 python -u tools/gemm_big_check.py > gpurun_out/$TAG/gemm.jsonl 2> gpurun_out/$TAG/gemm.err || { tail -5 gpurun_out/$TAG/gemm.err; exit 1; }
grep '"kernel": "256"' gpurun_out/$TAG/gemm.jsonl
bash tools/gpu_tests.sh $TAG "${2:-tests/test_gpu_large.py tests/test_gpu_parity.py tests/test_gpu_nofa.py tests/test_gpu_extra.py tests/test_sortformer.py}" 1
