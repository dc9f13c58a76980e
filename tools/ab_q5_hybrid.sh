# A/B: Q5_0 decode-row kernels with per-lane activation-scale loads everywhere but cross-Q (b) vs HEAD (a)
#   tools/ab_q5_hybrid.sh LIB_A LIB_B   (outputs gpurun_out/r06x2/)
set -o pipefail
O=gpurun_out/r06x2
bash tools/prof_ab_q5.sh $1 $2 r06x2 || exit 1
export OWK_MODEL_CACHE=/tmp/owk_models
for v in a b a b; do
  if [ $v = a ]; then L=$1; else L=$2; fi
  OWK_LIB=$L timeout -k 10 400 python3 -u bench.py --model large-v3-q5_0 --steps 4 --warmup 1 --no-cpu-baseline --no-prof > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json; d=[json.loads(l) for l in open('$O/bench_$v.json') if l.startswith('{')][-1]; print('$v', d['value'], d['ms_per_step'], (d.get('parity') or {}).get('tokens_equal'))" >> $O/bench.txt || exit 1
done
timeout -k 10 600 python3 -u -m pytest tests/test_q5.py tests/test_kquant.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/q5_tests.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_large.py -k "q5" -q -rP --timeout 500 --timeout-method thread -p no:cacheprovider > $O/large_q5_tests.txt 2>&1
