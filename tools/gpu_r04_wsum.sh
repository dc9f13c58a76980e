#!/bin/bash
# decode-row GEMMs with batched wave-order reductions: decode parity / bit-identity suites, F16 + Q5 bench
set -o pipefail
TAG=${1:-wsum}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py tests/test_gpu_parity.py tests/test_q5.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/k.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/k.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/$TAG/k.log | head -10; exit $rc; }
for m in large-v3 large-v3-q5_0; do
  timeout -k 10 300 python bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/b_$m.json 2> gpurun_out/$TAG/b_$m.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$TAG/b_$m.json')); print('$m RTF', d['value'], 'ms/step', d['ms_per_step'])"
  grep -E "\] (gemm_dec|gemm_logits) " gpurun_out/$TAG/b_$m.err
done
