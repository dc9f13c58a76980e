#!/bin/bash
# encoder attention change: encoder/full-depth parity, F16 + turbo benches
set -o pipefail
TAG=${1:-attn}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_q5.py tests/test_gpu_extra.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1; prc=$?
tail -2 gpurun_out/$TAG/parity.log; grep -E "^E |FAILED" gpurun_out/$TAG/parity.log | head -10
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
head -c 300 gpurun_out/$TAG/bench.json; echo; grep "\[bench\]" gpurun_out/$TAG/bench.err | grep -E "attn_encoder|gemm_enc"
timeout -k 10 400 python bench.py --model large-v3-turbo --steps 2 --warmup 1 > gpurun_out/$TAG/turbo.json 2> gpurun_out/$TAG/turbo.err || { tail -5 gpurun_out/$TAG/turbo.err; exit 1; }
head -c 300 gpurun_out/$TAG/turbo.json; echo; grep "\[bench\]" gpurun_out/$TAG/turbo.err | head -8
exit $prc
