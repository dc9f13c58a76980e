#!/bin/bash
# Round 5: softmax attention loads issued together (bit-identical) -- kernel tests, the flash_attn = false /
# DTW / configs[4] suites, then configs[4] sequential 2 min under rocprofv3 (graphs on, packet capture off)
set -o pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py tests/test_sortformer.py tests/test_gpu_c4.py "tests/test_gpu_large.py::test_large_dtw" -s \
    > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/$TAG/pytest.log | tail -3
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/seqtr -o run -- \
    python $GRAFT_REPO_ROOT/tools/pipeline_bench.py --minutes 2 --no-cpu --mode sequential --serial \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.err || { echo "trace failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py /tmp/seqtr > gpurun_out/$TAG/kernel_stats.txt && head -16 gpurun_out/$TAG/kernel_stats.txt
cat gpurun_out/$TAG/seq.json
