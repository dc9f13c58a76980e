#!/bin/bash
# wave-per-row resid_layernorm: A/B bench (OWK_RLN_WAVE=0 / 1) and decode parity
set -o pipefail
TAG=${1:-rln}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
for v in 1 0; do
  OWK_RLN_WAVE=$v timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench$v.json 2> gpurun_out/$TAG/bench$v.err || { tail -5 gpurun_out/$TAG/bench$v.err; exit 1; }
  echo "RLN_WAVE=$v: $(head -c 200 gpurun_out/$TAG/bench$v.json | grep -o '"value": [0-9.]*')"; grep "\[bench\]" gpurun_out/$TAG/bench$v.err | grep layernorm
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_q5.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1; prc=$?
tail -1 gpurun_out/$TAG/parity.log; grep -E "^E |FAILED" gpurun_out/$TAG/parity.log | head
exit $prc
