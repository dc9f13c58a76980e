#!/bin/bash
# rocprofv3 kernel stats of one bench step of another model: tools/gpu_modelprof.sh TAG MODEL
set -o pipefail
TAG=${1:-mprof}
MODEL=${2:-large-v3-q5_0}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model $MODEL --steps 1 --warmup 1 --no-cpu-baseline --no-prof \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/$TAG/prof > gpurun_out/$TAG/kernel_stats.txt
rm -f gpurun_out/$TAG/prof/*kernel_trace.csv
head -30 gpurun_out/$TAG/kernel_stats.txt
