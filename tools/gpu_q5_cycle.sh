#!/bin/bash
# Q5_0: GEMM restatement check, Q5 parity tests, Q5 large-v3 bench
set -o pipefail
mkdir -p gpurun_out/q5c
export OWK_MODEL_CACHE=/tmp/owk_models
export PYTHONPATH=$PWD/open-whisper-kit_amd/python:$PYTHONPATH
timeout -k 10 300 python -u tools/q5_gemm_check.py || exit 1
timeout -k 10 600 python -u -m pytest tests/test_q5.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/q5c/pytest.log 2>&1 || { tail -30 gpurun_out/q5c/pytest.log; exit 1; }
tail -2 gpurun_out/q5c/pytest.log
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
timeout -k 10 600 python -u bench.py --model large-v3-q5_0 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/q5c/q5_bench.json 2> gpurun_out/q5c/q5_bench.err || { echo "q5 bench failed"; tail -20 gpurun_out/q5c/q5_bench.err; exit 1; }
cut -c1-200 gpurun_out/q5c/q5_bench.json
grep "\[bench\]" gpurun_out/q5c/q5_bench.err | head -12
