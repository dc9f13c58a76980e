#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pipe
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 900 python -u tools/pipeline_bench.py --minutes 10 ${PIPE_ARGS} > gpurun_out/pipe/pipeline.json 2> gpurun_out/pipe/pipeline.err || { echo "pipeline failed"; tail -30 gpurun_out/pipe/pipeline.err; exit 1; }
cat gpurun_out/pipe/pipeline.json; grep "\[prof\]" gpurun_out/pipe/pipeline.err | head -20 || true
