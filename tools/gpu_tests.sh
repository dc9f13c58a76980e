#!/bin/bash
# GPU test pass for selected test files/expressions; outputs under gpurun_out/$TAG
#   tools/gpu_tests.sh TAG "<pytest args>" [BENCH=0|1]
set -o pipefail
TAG=${1:-tests}
ARGS=${2:-tests}
BENCH=${3:-0}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
eval timeout -k 10 1000 python -u -m pytest $ARGS -m gpu -v -s --timeout 400 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/$TAG/pytest.log | tail -3
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "^E |FAILED|Error" gpurun_out/$TAG/pytest.log | head -30; exit $rc; fi
if [ "$BENCH" = "1" ]; then
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
  cat gpurun_out/$TAG/bench.json
fi
