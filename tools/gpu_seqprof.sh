#!/bin/bash
# configs[4] sequential whisper_full with per-class HIP-event timing (eager launches)
set -o pipefail
mkdir -p gpurun_out/seqprof
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 600 python -u tools/pipeline_bench.py --minutes ${1:-2} --mode sequential --prof --no-cpu > gpurun_out/seqprof/pipeline.json 2> gpurun_out/seqprof/pipeline.err || { tail -20 gpurun_out/seqprof/pipeline.err; exit 1; }
cat gpurun_out/seqprof/pipeline.json; grep "\[prof\]" gpurun_out/seqprof/pipeline.err
