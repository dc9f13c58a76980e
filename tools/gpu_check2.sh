#!/bin/bash
set -o pipefail
TAG=${1:-chk}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_extra.py -k "fixed_work or audio_ctx" -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; rc=$?
grep -E "\[parity\]|passed|failed|Error" gpurun_out/$TAG/pytest.log | tail -25
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json; grep "\[bench\]" gpurun_out/$TAG/bench.err | head -8
timeout -k 10 600 python -u tools/pipeline_bench.py --minutes 10 --no-cpu --mode sequential > gpurun_out/$TAG/pipeline.json 2> gpurun_out/$TAG/pipeline.err || { tail -20 gpurun_out/$TAG/pipeline.err; exit 1; }
cat gpurun_out/$TAG/pipeline.json
exit $rc
