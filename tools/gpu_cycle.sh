#!/bin/bash
# parity tests then bench (+ optional rocprof) in one GPU call; outputs under gpurun_out/$TAG
set -o pipefail
TAG=${1:-cycle}
PROF=${2:-0}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed $?"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
if [ "$PROF" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline \
      > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.err || exit $?
  cd $GRAFT_REPO_ROOT
  python3 tools/prof_summary.py gpurun_out/$TAG/prof > gpurun_out/$TAG/kernel_stats.txt
  rm -f gpurun_out/$TAG/prof/*kernel_trace.csv   # keep the stats, drop the per-dispatch trace
fi
