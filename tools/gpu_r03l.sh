#!/bin/bash
# split-row logit processing: decode parity suites, then turbo A/B (one block per row vs split)
set -o pipefail
T=r03l
bash tools/gpu_tests.sh $T "tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_extra.py" 0 || exit $?
bash tools/gpu_ab.sh ablg3 OWK_LOGITS_SPLIT=0 OWK_LOGITS_SPLIT=1 --steps 2 --warmup 1 --model large-v3-turbo || exit $?
