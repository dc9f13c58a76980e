#!/bin/bash
# final tree: full GPU suite + smoke + driver-default bench
set -o pipefail
T=gpurun_out/r03o; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > $T/pytest.log 2>&1; rc=$?
tail -3 $T/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $T/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 1; }
tail -3 $T/smoke.log
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -5 $T/bench.err; exit 1; }
cut -c1-300 $T/bench.json
