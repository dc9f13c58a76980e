#!/bin/bash
# rocprofv3 kernel stats of the Q5_0 large-v3 bench
set -o pipefail
mkdir -p gpurun_out/q5p
export OWK_MODEL_CACHE=/tmp/owk_models
export PYTHONPATH=$PWD/open-whisper-kit_amd/python:$PYTHONPATH
timeout -k 10 600 python -u -c "
import threading, time, owk_synth as S
done = []
def hb():
    t = time.time()
    while not done:
        time.sleep(20); print('quantizing', int(time.time() - t), 's', flush=True)
threading.Thread(target=hb, daemon=True).start()
print(S.ensure_model('large-v3-q5_0'), flush=True); done.append(1)
" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/q5p/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model large-v3-q5_0 --steps 1 --warmup 1 --no-cpu-baseline --no-prof \
    > $GRAFT_REPO_ROOT/gpurun_out/q5p/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/q5p/bench.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/q5p/prof > gpurun_out/q5p/kernel_stats.txt
rm -f gpurun_out/q5p/prof/*kernel_trace.csv
head -24 gpurun_out/q5p/kernel_stats.txt
