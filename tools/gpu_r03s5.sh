#!/bin/bash
set -o pipefail
T=gpurun_out/r03s5; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 500 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > $T/bench_q5.json 2> $T/bench_q5.err || { tail -20 $T/bench_q5.err; exit 1; }
python -c "import json;d=json.load(open('$T/bench_q5.json'));print('Q5_0', d['value'], d['ms_per_step'])"
grep "\[bench\] alone" $T/bench_q5.err | head -4
timeout -k 10 600 python -u -m pytest tests/test_q5.py -m gpu -q -x --timeout 300 --timeout-method thread > $T/q5.log 2>&1; rc=$?
tail -3 $T/q5.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $T/q5.log | head; exit $rc; }
echo ok
