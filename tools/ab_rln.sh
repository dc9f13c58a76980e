# round-6 A/Bs (one box): one-wave resid_layernorm (OWK_RLN_WAVE, temporary switch), the Q5_0 decode-row
# kernel's direct activation-scale loads (OWK_LIB = the build before them), the key-split P.V ticket's
# release/acquire fences (timing + bit-identity)
set -o pipefail
mkdir -p gpurun_out/r06h
export OWK_MODEL_CACHE=/tmp/owk_models
BASE=open-whisper-kit_amd/lib_ab/libwhisper_base.so
run() {  # tag, env..., bench args
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --verbose $BENCH > gpurun_out/r06h/b_$tag.json 2> gpurun_out/r06h/b_$tag.err || return 1
  python -c "import json; d=json.loads(open('gpurun_out/r06h/b_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'])" >> gpurun_out/r06h/ab.txt
  grep -E "layernorm|gemm_dec " gpurun_out/r06h/b_$tag.err | sed "s/^/$tag /" >> gpurun_out/r06h/ab.txt
}
timeout -k 10 120 python -u tools/sm_split_time.py > gpurun_out/r06h/sm_split.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "softmax" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06h/sm_tests.txt 2>&1 || exit 1
BENCH="--model large-v3"
for i in 1 2; do
  run f16_w0_$i OWK_RLN_WAVE=0 || exit 1
  run f16_w1_$i OWK_RLN_WAVE=1 || exit 1
done
BENCH="--model large-v3-q5_0"
for i in 1 2; do
  run q5_base_$i OWK_LIB=$BASE || exit 1
  run q5_new_$i OWK_LIB=open-whisper-kit_amd/lib/libwhisper.so || exit 1
done
