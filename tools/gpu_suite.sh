#!/bin/bash
# The GPU suite on the current tree in two parts (A: everything but the full-depth large / configs[4]
# files, B: those), logs under gpurun_out/TAG
set -o pipefail
TAG=${1:-r05f}
PART=${2:-A}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
if [ "$PART" = A ]; then
  SEL="--ignore=tests/test_gpu_large.py --ignore=tests/test_gpu_c4.py"
else
  SEL="tests/test_gpu_large.py tests/test_gpu_c4.py"
  [ "$PART" = B ] || exit 2
fi
if [ "$PART" = A ]; then TARGET=tests; else TARGET=""; fi
timeout -k 10 1100 python -u -m pytest $TARGET $SEL -m gpu -q -rP --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$TAG/gpu_tests_$PART.txt 2>&1
rc=$?
tail -5 gpurun_out/$TAG/gpu_tests_$PART.txt
grep -E "FAILED|Error" gpurun_out/$TAG/gpu_tests_$PART.txt | head -20
exit $rc
