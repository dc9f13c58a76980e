#!/bin/bash
# round-end record: full GPU suite + smoke + F16 bench with rocprofv3 stats, then the other configs
set -o pipefail
TAG=${1:-final}
bash tools/gpu_full.sh $TAG || exit $?
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python bench.py --model large-v3-turbo --steps 2 --warmup 1 > gpurun_out/$TAG/turbo.json 2> gpurun_out/$TAG/turbo.err || { tail -5 gpurun_out/$TAG/turbo.err; exit 1; }
head -c 200 gpurun_out/$TAG/turbo.json; echo
timeout -k 10 400 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/q5.json 2> gpurun_out/$TAG/q5.err || { tail -5 gpurun_out/$TAG/q5.err; exit 1; }
head -c 200 gpurun_out/$TAG/q5.json; echo
timeout -k 10 600 python -u tools/pipeline_bench.py --minutes 10 --no-cpu > gpurun_out/$TAG/pipeline.json 2> gpurun_out/$TAG/pipeline.err || { tail -20 gpurun_out/$TAG/pipeline.err; exit 1; }
head -c 600 gpurun_out/$TAG/pipeline.json; echo
