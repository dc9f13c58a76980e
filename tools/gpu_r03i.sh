#!/bin/bash
# SortFormer 2 s stream: kernel stats + idle-gap breakdown of the kernel trace (after warm-up)
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python -u -m pytest tests/test_sortformer.py tests/test_sortformer_q.py -m gpu -q -x --timeout 200 --timeout-method thread > /tmp/sft.log 2>&1 || { tail -20 /tmp/sft.log; exit 1; }
tail -2 /tmp/sft.log
T=r03i3
mkdir -p gpurun_out/$T
export OWK_MODEL_CACHE=/tmp/owk_models
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/sfprof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sf_stream_one.py --minutes 2 > $GRAFT_REPO_ROOT/gpurun_out/$T/sfprof.json 2> $GRAFT_REPO_ROOT/gpurun_out/$T/sfprof.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/$T/sfprof > gpurun_out/$T/sf_kernel_stats.txt
python3 tools/trace_gaps.py gpurun_out/$T/sfprof --skip 0 > gpurun_out/$T/gaps.txt
rm -f gpurun_out/$T/sfprof/*kernel_trace.csv
cat gpurun_out/$T/sfprof.json gpurun_out/$T/gaps.txt
head -16 gpurun_out/$T/sf_kernel_stats.txt
