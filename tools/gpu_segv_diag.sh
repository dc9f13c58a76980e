#!/bin/bash
# Reproduce the rocprofv3 --kernel-trace crash on graph replays of the flash_attn = false decode
# passes (configs[4] sequential, 2 min of audio) with the library's symbolizing SIGSEGV handler
# (OWK_BACKTRACE=1: library+offset per frame, the maps around the fault address).
set -o pipefail
TAG=${1:-segv}
MIN=${2:-2}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
export TMPDIR=/tmp
export OWK_BACKTRACE=1
# PKTCAP=0: HIP submits a replayed graph node by node instead of as one captured AQL packet batch
[ -n "$PKTCAP" ] && export DEBUG_CLR_GRAPH_PACKET_CAPTURE=$PKTCAP
python -c "import sys; sys.path.insert(0, 'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('large-v3', cache_dir='/tmp/owk_models')" \
    || exit 1
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/seqtr -o run -- \
    python $GRAFT_REPO_ROOT/tools/pipeline_bench.py --minutes $MIN --no-cpu --mode sequential --serial \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.err
rc=$?
cd $GRAFT_REPO_ROOT
echo "rocprofv3 exit $rc"
grep -v "^W20\|^I20" gpurun_out/$TAG/seq.err | tail -80
if [ $rc -eq 0 ]; then
    python tools/prof_summary.py /tmp/seqtr > gpurun_out/$TAG/kernel_stats.txt && head -30 gpurun_out/$TAG/kernel_stats.txt
fi
exit 0
