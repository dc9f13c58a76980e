#!/bin/bash
# Q5_0 bench kernel stats; one SortFormer 2 s stream (wall + kernel stats)
set -o pipefail
T=r03g
mkdir -p gpurun_out/$T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python tools/sf_stream_one.py > gpurun_out/$T/sf_stream.json 2> gpurun_out/$T/sf_stream.err || { tail -5 gpurun_out/$T/sf_stream.err; exit 1; }
cat gpurun_out/$T/sf_stream.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/sfprof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sf_stream_one.py --minutes 2 > $GRAFT_REPO_ROOT/gpurun_out/$T/sfprof.json 2> $GRAFT_REPO_ROOT/gpurun_out/$T/sfprof.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/$T/sfprof > gpurun_out/$T/sf_kernel_stats.txt
rm -f gpurun_out/$T/sfprof/*kernel_trace.csv
head -25 gpurun_out/$T/sf_kernel_stats.txt
bash tools/gpu_modelprof.sh r03q5p large-v3-q5_0
