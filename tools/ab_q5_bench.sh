# unprofiled Q5_0 bench A/B of two library builds (a b a b) + the output digest of each (tools/q5_lib_diff.py)
#   tools/ab_q5_bench.sh LIB_A LIB_B TAG
set -o pipefail
O=gpurun_out/$3
mkdir -p $O
export OWK_MODEL_CACHE=/tmp/owk_models
for v in a b; do
  if [ $v = a ]; then L=$1; else L=$2; fi
  OWK_LIB=$L timeout -k 10 300 python3 -u tools/q5_lib_diff.py > $O/digest_$v.txt 2>&1 || exit 1
done
for v in a b a b; do
  if [ $v = a ]; then L=$1; else L=$2; fi
  OWK_LIB=$L timeout -k 10 400 python3 -u bench.py --model large-v3-q5_0 --steps 4 --warmup 1 --no-cpu-baseline --no-prof > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json; d=[json.loads(l) for l in open('$O/bench_$v.json') if l.startswith('{')][-1]; print('$v', d['value'], d['ms_per_step'])" >> $O/bench.txt || exit 1
done
cat $O/digest_a.txt $O/digest_b.txt $O/bench.txt
