#!/bin/bash
# vectorized Q8 quantizer of the quantized encoder: quantized suites, then the Q5_0 bench + kernel stats
set -o pipefail
T=r03j
mkdir -p gpurun_out/$T
export OWK_MODEL_CACHE=/tmp/owk_models
bash tools/gpu_tests.sh $T "tests/test_q5.py tests/test_kquant.py tests/test_gpu_large.py -k 'q5 or Q5 or quant'" 0 || exit $?
timeout -k 10 400 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$T/q5.json 2> gpurun_out/$T/q5.err || { tail -5 gpurun_out/$T/q5.err; exit 1; }
head -c 400 gpurun_out/$T/q5.json; echo
bash tools/gpu_modelprof.sh ${T}p large-v3-q5_0
