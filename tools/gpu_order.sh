#!/bin/bash
set -o pipefail
TAG=${1:-order}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_q5.py -k "gemm256 or q16" -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/$TAG/unit.log 2>&1 || { grep -E "max|FAIL|Error" gpurun_out/$TAG/unit.log | head -30; exit 1; }
tail -1 gpurun_out/$TAG/unit.log
timeout -k 10 300 python -u tools/gemm_big_check.py > gpurun_out/$TAG/gemm.jsonl 2> gpurun_out/$TAG/gemm.err || { tail -5 gpurun_out/$TAG/gemm.err; exit 1; }
grep '"kernel": "256"' gpurun_out/$TAG/gemm.jsonl
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
head -c 250 gpurun_out/$TAG/bench.json; echo; grep "\[bench\]" gpurun_out/$TAG/bench.err | grep -E "gemm_enc|gemm_cross|attn_enc"
timeout -k 10 400 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/q5.json 2> gpurun_out/$TAG/q5.err || { tail -5 gpurun_out/$TAG/q5.err; exit 1; }
head -c 250 gpurun_out/$TAG/q5.json; echo; grep "\[bench\]" gpurun_out/$TAG/q5.err | grep -E "gemm_enc|gemm_cross"
