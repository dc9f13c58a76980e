#!/bin/bash
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
OWK_ROWS_NT_PARTIAL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "dispatch or greedy or fixed or beam" -m gpu -q --timeout 300 --timeout-method thread > /tmp/nt5.log 2>&1 || { grep -E "^E |FAILED|passed|failed" /tmp/nt5.log | head -20; exit 1; }
tail -1 /tmp/nt5.log
bash tools/gpu_ab.sh ab_ntpart OWK_ROWS_NT_PARTIAL=0 OWK_ROWS_NT_PARTIAL=1 --steps 2 --warmup 1 || exit $?
