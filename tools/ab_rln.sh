set -o pipefail
mkdir -p gpurun_out/r06h
export OWK_MODEL_CACHE=/tmp/owk_models
for v in 0 1 0 1; do
  OWK_RLN_WAVE=$v timeout -k 10 300 python -u bench.py --model large-v3 --steps 4 --warmup 1 --no-cpu-baseline --verbose > gpurun_out/r06h/b_$v.json 2> gpurun_out/r06h/b_$v.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r06h/b_$v.json').read().strip().splitlines()[-1]); print('wave=$v', d['value'], d['ms_per_step'])" >> gpurun_out/r06h/ab.txt
  grep -E "layernorm|gemm_dec " gpurun_out/r06h/b_$v.err | sed "s/^/wave=$v /" >> gpurun_out/r06h/ab.txt
done
timeout -k 10 120 python -u tools/sm_split_time.py > gpurun_out/r06h/sm_split.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "softmax" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06h/sm_tests.txt 2>&1
