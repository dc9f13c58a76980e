# A/B: self attention through the loader + math two-wave form (OWK_SELF2=1, temporary switch) vs one wave
set -o pipefail
mkdir -p gpurun_out/r06r
export OWK_MODEL_CACHE=/tmp/owk_models
for v in 0 1 0 1; do
  OWK_SELF2=$v timeout -k 10 400 python -u bench.py --model large-v3 --steps 4 --warmup 1 --no-cpu-baseline --verbose > gpurun_out/r06r/b_$v.json 2> gpurun_out/r06r/b_$v.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r06r/b_$v.json').read().strip().splitlines()[-1]); print('self2=$v', d['value'], d['ms_per_step'])" >> gpurun_out/r06r/ab.txt
  grep -E "attn_self" gpurun_out/r06r/b_$v.err | sed "s/^/self2=$v /" >> gpurun_out/r06r/ab.txt
done
OWK_SELF2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "greedy or fixed_work or token_ts" -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06r/parity_self2.txt 2>&1
