#!/bin/bash
# fused resid_layernorm: bit identity, chain A/B, bench and configs[4] sequential timing
set -o pipefail
TAG=${1:-rln}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v -s -k "fused_rln or whole_k" --timeout 300 --timeout-method thread > gpurun_out/$TAG/k.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/$TAG/k.log | tail -1
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/$TAG/k.log | head -10; exit $rc; }
timeout -k 10 120 python -u tools/chain_ab.py --rows 32,8,1 > gpurun_out/$TAG/chain_ab.txt 2>&1 && cat gpurun_out/$TAG/chain_ab.txt &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
python -c "import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print('bench RTF', d['value'], 'ms/step', d['ms_per_step'])" &&
timeout -k 10 200 python -u tools/seq_asr.py --minutes 2
