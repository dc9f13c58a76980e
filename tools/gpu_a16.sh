#!/bin/bash
set -o pipefail
TAG=${1:-a16}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 700 python -u -m pytest tests/test_q5.py tests/test_gpu_large.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/$TAG/q5.log 2>&1; prc=$?
grep -E "A16 max|passed|failed" gpurun_out/$TAG/q5.log | tail -20; grep -E "^E |FAILED" gpurun_out/$TAG/q5.log | head -10
timeout -k 10 400 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/q5.json 2> gpurun_out/$TAG/q5.err || { tail -5 gpurun_out/$TAG/q5.err; exit 1; }
head -c 300 gpurun_out/$TAG/q5.json; echo; grep "\[bench\]" gpurun_out/$TAG/q5.err | head -9
exit $prc
