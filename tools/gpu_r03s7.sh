#!/bin/bash
set -o pipefail
T=gpurun_out/r03s7; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $T/bench_f16.json 2> $T/bench_f16.err || { tail -20 $T/bench_f16.err; exit 1; }
python -c "import json;d=json.load(open('$T/bench_f16.json'));print('F16', d['value'], d['ms_per_step'], d['parity'])"
grep "\[bench\]" $T/bench_f16.err | grep -E "gemm_enc|attn_enc|gemm_cross" | head -4
timeout -k 10 400 python bench.py --model large-v3-turbo --steps 2 --warmup 1 > $T/bench_turbo.json 2> $T/bench_turbo.err || { tail -20 $T/bench_turbo.err; exit 1; }
python -c "import json;d=json.load(open('$T/bench_turbo.json'));print('turbo', d['value'], d['ms_per_step'], d['parity'])"
grep "\[bench\]" $T/bench_turbo.err | head -8
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_nofa.py tests/test_sortformer.py -m gpu -q --timeout 400 --timeout-method thread > $T/par.log 2>&1; rc=$?
tail -3 $T/par.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $T/par.log | head -20; exit $rc; }
echo ok
