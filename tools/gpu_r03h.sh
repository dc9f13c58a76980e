#!/bin/bash
# 64x64 ring tile: kernel checks first (bit-identity, speed), then the suites it feeds, then the stream timing
set -o pipefail
T=r03h2
mkdir -p gpurun_out/$T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "mid or dispatch or epilogue" -m gpu -v -s --timeout 120 --timeout-method thread > gpurun_out/$T/kern.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/$T/kern.log | head -30; exit 1; }
grep -E "64x64 ring|passed|failed" gpurun_out/$T/kern.log
timeout -k 10 300 env OWK_GEMM_MID64_MIN=1 python tools/sf_stream_one.py > gpurun_out/$T/sf_stream64.json 2> gpurun_out/$T/sf_stream64.err && cat gpurun_out/$T/sf_stream64.json || exit 1
bash tools/gpu_tests.sh $T "tests/test_sortformer.py tests/test_sortformer_q.py tests/test_gpu_parity.py tests/test_vad.py" 0 || exit $?
timeout -k 10 300 python tools/sf_stream_one.py > gpurun_out/$T/sf_stream.json 2> gpurun_out/$T/sf_stream.err || { tail -5 gpurun_out/$T/sf_stream.err; exit 1; }
cat gpurun_out/$T/sf_stream.json
