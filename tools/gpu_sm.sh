#!/bin/bash
# soft_max (flash_attn = false) attention change: nofa/DTW/large parity, then the sequential profile
set -o pipefail
TAG=${1:-sm}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 700 python -u -m pytest tests/test_gpu_nofa.py tests/test_gpu_large.py tests/test_gpu_kernels.py tests/test_gpu_extra.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/parity.log 2>&1; prc=$?
tail -2 gpurun_out/$TAG/parity.log; grep -E "^E |FAILED" gpurun_out/$TAG/parity.log | head -10
[ $prc -eq 0 ] || exit $prc
timeout -k 10 600 python -u tools/pipeline_bench.py --minutes 2 --mode sequential --prof --no-cpu > gpurun_out/$TAG/seqprof.json 2> gpurun_out/$TAG/seqprof.err || { tail -20 gpurun_out/$TAG/seqprof.err; exit 1; }
cat gpurun_out/$TAG/seqprof.json; grep "\[prof\]" gpurun_out/$TAG/seqprof.err | head -5
timeout -k 10 900 python -u tools/pipeline_bench.py --minutes 10 > gpurun_out/$TAG/pipeline.json 2> gpurun_out/$TAG/pipeline.err || { tail -10 gpurun_out/$TAG/pipeline.err; exit 1; }
cat gpurun_out/$TAG/pipeline.json
