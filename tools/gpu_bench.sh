#!/bin/bash
# bench + rocprofv3 kernel summary on the GPU box (outputs under gpurun_out/)
set -o pipefail
TAG=${1:-r1}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.err || exit $?
