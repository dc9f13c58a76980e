#!/bin/bash
# round-3 final, part 2: driver-default F16 bench + rocprofv3 kernel stats, turbo, Q5_0, configs[4]
set -o pipefail
T=r03f2
bash tools/gpu_round.sh $T none || exit $?
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python bench.py --model large-v3-turbo --steps 2 --warmup 1 > gpurun_out/$T/turbo.json 2> gpurun_out/$T/turbo.err || { tail -5 gpurun_out/$T/turbo.err; exit 1; }
head -c 300 gpurun_out/$T/turbo.json; echo
timeout -k 10 400 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$T/q5.json 2> gpurun_out/$T/q5.err || { tail -5 gpurun_out/$T/q5.err; exit 1; }
head -c 300 gpurun_out/$T/q5.json; echo
