#!/bin/bash
# baseline benches on this tree: F16 (driver default) and large-v3 Q5_0
set -o pipefail
T=gpurun_out/r03s4; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $T/bench_f16.json 2> $T/bench_f16.err || { tail -20 $T/bench_f16.err; exit 1; }
python -c "import json;d=json.load(open('$T/bench_f16.json'));print('F16', d['value'], d['ms_per_step'])"
timeout -k 10 500 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > $T/bench_q5.json 2> $T/bench_q5.err || { tail -20 $T/bench_q5.err; exit 1; }
python -c "import json;d=json.load(open('$T/bench_q5.json'));print('Q5_0', d['value'], d['ms_per_step'])"
grep "\[bench\]" $T/bench_q5.err | head -12
