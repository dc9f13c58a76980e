#!/bin/bash
# large-GEMM check + timing, then the full-depth parity tests that run it, then the bench
set -o pipefail
TAG=${1:-gemm}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -u tools/gemm_big_check.py > gpurun_out/$TAG/gemm.jsonl 2> gpurun_out/$TAG/gemm.err || { echo "gemm check failed rc=$?"; tail -20 gpurun_out/$TAG/gemm.err; exit 1; }
cat gpurun_out/$TAG/gemm.jsonl
if grep -q '"ok": false' gpurun_out/$TAG/gemm.jsonl; then echo "GEMM MISMATCH"; exit 1; fi
bash tools/gpu_tests.sh $TAG "${2:-tests/test_gpu_large.py -k 'not q5 and not dtw'}" 1
