#!/bin/bash
# Round 5: quantized decode-row GEMM scale reads hoisted -- quantized suites, then the Q5_0 bench under
# rocprofv3 --stats (one step) and a timed Q5_0 bench line
set -o pipefail
TAG=${1:-r05q}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_q5.py "tests/test_gpu_large.py::test_large_batch32" tests/test_kquant.py > gpurun_out/$TAG/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/gpu_profiles.sh $TAG large-v3-q5_0 || exit 1
timeout -k 10 600 python bench.py --model large-v3-q5_0 --no-cpu-baseline > gpurun_out/$TAG/bench_q5.json 2> gpurun_out/$TAG/bench_q5.err || { echo "q5 bench failed"; tail -5 gpurun_out/$TAG/bench_q5.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/$TAG/bench_q5.json')); r=d.get('roofline') or {}
print('q5 RTF', d['value'], 'ms/step', d['ms_per_step'], 'dom', r.get('kernel_class'), 'frac', r.get('frac'))"
