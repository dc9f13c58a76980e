#!/bin/bash
set -o pipefail
T=gpurun_out/r03s3; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v -s -k "cross" --timeout 120 --timeout-method thread > $T/kern.log 2>&1; rc=$?
grep -E "attn_cross|passed|failed" $T/kern.log | tail -14
[ $rc -ne 0 ] && { grep -E "^E " $T/kern.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 2 --warmup 1 > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 1; }
cat $T/bench.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4.py tests/test_sortformer_q.py tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -v -s --timeout 400 --timeout-method thread > $T/par.log 2>&1; rc=$?
grep -E "\[c4\]|\[sfq\].*RTTM|passed|failed" $T/par.log | tail -30
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $T/par.log | head -20; exit $rc; }
echo ok
