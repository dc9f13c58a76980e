#!/bin/bash
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "dispatch or greedy or fixed or beam" -m gpu -q --timeout 300 --timeout-method thread > /tmp/nt2.log 2>&1 || { grep -E "^E |FAILED|passed|failed" /tmp/nt2.log | head -20; exit 1; }
tail -1 /tmp/nt2.log
OWK_ROWS_NT=1 timeout -k 10 120 python tools/rows_nt_sweep.py || exit 1
OWK_ROWS_NT=2 OWK_ROWS_NT_MIN_N=1 timeout -k 10 120 python tools/rows_nt_sweep.py || exit 1
