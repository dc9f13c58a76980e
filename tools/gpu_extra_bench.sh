#!/bin/bash
# extra measurements: SortFormer diarization RTF (GPU vs reference CPU) and the Q5_0 large-v3 bench
set -o pipefail
mkdir -p gpurun_out/extra
export OWK_MODEL_CACHE=/tmp/owk_models
export PYTHONPATH=$PWD/open-whisper-kit_amd/python:$PYTHONPATH
timeout -k 10 600 python -u tools/sf_bench.py --minutes 10 --cpu-seconds 60 > gpurun_out/extra/sf_bench.json 2> gpurun_out/extra/sf_bench.err || { echo "sf_bench failed"; tail -20 gpurun_out/extra/sf_bench.err; exit 1; }
cat gpurun_out/extra/sf_bench.json
# Q5_0 large-v3 model (quantized on the box from the synthetic F16 file), with a heartbeat
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
timeout -k 10 600 python -u bench.py --model large-v3-q5_0 --steps 1 --warmup 1 > gpurun_out/extra/q5_bench.json 2> gpurun_out/extra/q5_bench.err || { echo "q5 bench failed"; tail -20 gpurun_out/extra/q5_bench.err; exit 1; }
cat gpurun_out/extra/q5_bench.json
grep "\[bench\]" gpurun_out/extra/q5_bench.err | head -12
