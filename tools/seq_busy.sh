# configs[4] transcription leg (tools/seq_asr.py, 2 min, greedy without fallback): the kernels' busy time
# inside the timed run (rocprofv3 kernel trace, its final seconds) against the unprofiled wall of the same run
set -o pipefail
O=gpurun_out/${1:-r06w}
mkdir -p $O
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python3 -u tools/seq_asr.py --minutes 2 > $O/seq_plain.txt 2>&1 || exit 1
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/seqb -o run -- \
    python3 -u tools/seq_asr.py --minutes 2 > $O/seq_prof.txt 2>&1 || exit 1
W=$(python3 -c "import json; print([json.loads(l) for l in open('$O/seq_prof.txt') if l.startswith('{')][-1]['wall_s'])")
python3 tools/trace_gaps.py /tmp/seqb --last $W > $O/seq_busy.txt || exit 1
cat $O/seq_plain.txt $O/seq_prof.txt $O/seq_busy.txt
