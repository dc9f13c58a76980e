#!/bin/bash
# VAD bench + rocprof kernel stats in one GPU call; outputs under gpurun_out/$TAG
set -o pipefail
TAG=${1:-vad}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python tools/vad_bench.py > gpurun_out/$TAG/vad_bench.json 2> gpurun_out/$TAG/vad_bench.err || { echo "vad bench failed"; tail -20 gpurun_out/$TAG/vad_bench.err; exit 1; }
cat gpurun_out/$TAG/vad_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/vad_bench.py --iters 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/$TAG/prof > gpurun_out/$TAG/kernel_stats.txt
rm -f gpurun_out/$TAG/prof/*kernel_trace.csv
grep -i vad gpurun_out/$TAG/kernel_stats.txt || true
