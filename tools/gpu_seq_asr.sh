#!/bin/bash
# configs[4] transcription leg: wall per token with / without DTW and flash_attn, then a kernel trace
set -o pipefail
TAG=${1:-seq_asr}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/seq_asr.py --minutes 2 | tee gpurun_out/$TAG/dtw.json || exit 1
timeout -k 10 200 python -u tools/seq_asr.py --minutes 2 --no-dtw | tee gpurun_out/$TAG/nodtw.json || exit 1
timeout -k 10 200 python -u tools/seq_asr.py --minutes 2 --no-dtw --fa | tee gpurun_out/$TAG/fa.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/seqtr -o run -- \
    python tools/seq_asr.py --minutes 2 > gpurun_out/$TAG/trace_run.json 2> gpurun_out/$TAG/trace_run.err || { echo "trace failed"; grep -v "^    @" gpurun_out/$TAG/trace_run.err | tail -5; exit 1; }
python tools/trace_gaps.py /tmp/seqtr --skip 25 | tee gpurun_out/$TAG/gaps.txt
python tools/prof_summary.py /tmp/seqtr > gpurun_out/$TAG/kernel_stats.txt && head -30 gpurun_out/$TAG/kernel_stats.txt
