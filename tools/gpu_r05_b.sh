#!/bin/bash
# Round 5: the small-model parity suites with the every-step decision check and the cli_default injection
set -o pipefail
TAG=${1:-r05b}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
    tests/test_gpu_parity.py tests/test_gpu_nofa.py > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
grep -E "\[decisions\]|\[parity\].*parted|passed|failed|Error" gpurun_out/$TAG/pytest.log | tail -60
exit $rc
