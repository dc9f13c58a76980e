#!/bin/bash
# configs[4] sequential (2 min of audio): rocprofv3 kernel trace + stats, GPU busy vs wall (on the box)
set -o pipefail
TAG=${1:-seq_trace}
MIN=${2:-2}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0  # rocprofiler-sdk walks captured graph packets otherwise (profiles/r05_rocprof_graph_segv.txt)
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/seqtr -o run -- \
    python tools/pipeline_bench.py --minutes $MIN --no-cpu --mode sequential --serial > gpurun_out/$TAG/seq.json 2> gpurun_out/$TAG/seq.err \
    || { echo "trace failed"; tail -5 gpurun_out/$TAG/seq.err; exit 1; }
python tools/trace_gaps.py /tmp/seqtr ${GAPS_ARGS:---skip 20} | tee gpurun_out/$TAG/gaps.txt || exit 1
python tools/prof_summary.py /tmp/seqtr > gpurun_out/$TAG/kernel_stats.txt && head -30 gpurun_out/$TAG/kernel_stats.txt
