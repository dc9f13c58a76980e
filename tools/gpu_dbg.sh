#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/dbg
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -rf > gpurun_out/dbg/kern.log 2>&1; echo "kern exit $?" >> gpurun_out/dbg/kern.log
OWK_NO_GRAPH=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "test_encoder_and_prefill_logits or test_whisper_full" > gpurun_out/dbg/nograph.log 2>&1; echo "nograph exit $?" >> gpurun_out/dbg/nograph.log
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "test_encoder_and_prefill_logits" > gpurun_out/dbg/graph.log 2>&1; echo "graph exit $?" >> gpurun_out/dbg/graph.log
