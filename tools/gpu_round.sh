#!/bin/bash
# GPU tests (pytest args) -> bench -> rocprofv3 kernel stats of one bench step; outputs under gpurun_out/$TAG
set -o pipefail
TAG=${1:-round}
ARGS=${2:-tests}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
if [ "$ARGS" != "none" ]; then
  bash tools/gpu_tests.sh $TAG "$ARGS" 0 || exit $?
fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
grep "\[bench\]" gpurun_out/$TAG/bench.err | head -20
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-prof \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/$TAG/prof > gpurun_out/$TAG/kernel_stats.txt
rm -f gpurun_out/$TAG/prof/*kernel_trace.csv
head -25 gpurun_out/$TAG/kernel_stats.txt
