#!/bin/bash
# decode attention change: kernel tests + key sweep, parity suites, F16 bench, configs[4] pipeline
set -o pipefail
TAG=${1:-dattn}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -s --timeout 120 --timeout-method thread > gpurun_out/$TAG/kernels.log 2>&1 || { tail -30 gpurun_out/$TAG/kernels.log; exit 1; }
tail -1 gpurun_out/$TAG/kernels.log
timeout -k 10 120 python -u tools/attn_sweep.py > gpurun_out/$TAG/attn.jsonl 2>&1 || { tail -5 gpurun_out/$TAG/attn.jsonl; exit 1; }
cat gpurun_out/$TAG/attn.jsonl
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_extra.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1; prc=$?
tail -2 gpurun_out/$TAG/parity.log; grep -E "^E |FAILED" gpurun_out/$TAG/parity.log | head -10
[ $prc -eq 0 ] || exit $prc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
head -c 300 gpurun_out/$TAG/bench.json; echo; grep "\[bench\]" gpurun_out/$TAG/bench.err | head -9
timeout -k 10 900 python -u tools/pipeline_bench.py --minutes 10 > gpurun_out/$TAG/pipeline.json 2> gpurun_out/$TAG/pipeline.err || { tail -10 gpurun_out/$TAG/pipeline.err; exit 1; }
cat gpurun_out/$TAG/pipeline.json
