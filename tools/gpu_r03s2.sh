#!/bin/bash
set -o pipefail
T=gpurun_out/r03s2; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 120 ./tools/lab_gemv p > $T/lab_pf.txt 2>&1 || { echo "lab failed"; tail $T/lab_pf.txt; exit 1; }
cat $T/lab_pf.txt
timeout -k 10 600 python -u -m pytest tests/test_sortformer_q.py tests/test_sortformer.py -m gpu -v -s --timeout 300 --timeout-method thread > $T/sfq.log 2>&1; rc=$?
grep -E "\[sfq\]|passed|failed" $T/sfq.log | tail -40
[ $rc -ne 0 ] && { grep -E "^E " $T/sfq.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 1; }
tail -3 $T/smoke.log
