#!/bin/bash
# Round 5: quantized decode-row GEMM scale reads hoisted, XCD-aware encoder attention -- the large and
# quantized suites, then timed bench lines of large-v3 Q5_0 and F16 (no CPU leg)
set -o pipefail
TAG=${1:-r05q}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
    "tests/test_gpu_kernels.py::test_softmax_attention_split_bit_identical" tests/test_gpu_large.py tests/test_q5.py \
    tests/test_kquant.py > gpurun_out/$TAG/pytest.log 2>&1 \
    || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest.log | tail -20; exit 1; }
grep -E "passed|failed|\[decisions\]|parted|bit-identical; single" gpurun_out/$TAG/pytest.log | tail -24
for m in large-v3-q5_0 large-v3; do
  timeout -k 10 600 python bench.py --model $m --no-cpu-baseline > gpurun_out/$TAG/bench_$m.json 2> gpurun_out/$TAG/bench_$m.err \
      || { echo "$m bench failed"; tail -5 gpurun_out/$TAG/bench_$m.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/$TAG/bench_$m.json')); r=d.get('roofline') or {}
print('$m RTF', d['value'], 'ms/step', d['ms_per_step'], 'dom', r.get('kernel_class'), 'frac', r.get('frac'), 'phases', (r.get('phases') or {}).get('encoder_mfma'))"
  grep "\[bench\]" gpurun_out/$TAG/bench_$m.err | head -14
done
