#!/bin/bash
# large-tile GEMM changes: epilogue cross-checks + quantized q16 path vs the reference, then the
# full-depth parity tests, the F16 and Q5_0 benches and a rocprofv3 kernel summary of one F16 step
set -o pipefail
TAG=${1:-q16}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_q5.py -k "gemm256 or q16" -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/$TAG/unit.log 2>&1 || { grep -E "max|err|FAIL|Error" gpurun_out/$TAG/unit.log | head -30; exit 1; }
grep -E "max\||max rel" gpurun_out/$TAG/unit.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_extra.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1; prc=$?
grep -E "passed|failed" gpurun_out/$TAG/parity.log | tail -2; grep -E "^E |FAILED" gpurun_out/$TAG/parity.log | head -10
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json; grep "\[bench\]" gpurun_out/$TAG/bench.err | head -8
timeout -k 10 400 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/q5.json 2> gpurun_out/$TAG/q5.err || { tail -5 gpurun_out/$TAG/q5.err; exit 1; }
cat gpurun_out/$TAG/q5.json; grep "\[bench\]" gpurun_out/$TAG/q5.err | head -8
exit $prc
