#!/bin/bash
# the driver's round-end checks: full GPU suite, smoke(), then bench + rocprofv3 kernel stats
set -o pipefail
TAG=${1:-full}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/$TAG/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -4 gpurun_out/$TAG/smoke.log
if [ "${2:-bench}" = "bench" ]; then bash tools/gpu_round.sh $TAG none; fi
