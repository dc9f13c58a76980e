#!/bin/bash
# NT column tiles per block for the logits GEMM: parity under NT=4, then turbo A/Bs
set -o pipefail
T=r03n
mkdir -p gpurun_out/$T
export OWK_MODEL_CACHE=/tmp/owk_models
OWK_ROWS_NT=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "dispatch or greedy or fixed or beam" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/$T/pytest.log | head -20; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash tools/gpu_ab.sh ab_nt4 OWK_ROWS_NT=0 OWK_ROWS_NT=4 --steps 2 --warmup 1 --model large-v3-turbo || exit $?
bash tools/gpu_ab.sh ab_nt2 OWK_ROWS_NT=0 OWK_ROWS_NT=2 --steps 2 --warmup 1 --model large-v3-turbo || exit $?
