#!/bin/bash
# Round 5: persistent decode chain -- bit-identity, stamps of one layer, configs[4] sequential 2 min A/B
set -o pipefail
TAG=${1:-r05d}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_chain.py > gpurun_out/$TAG/pytest.log 2>&1 \
    || { echo "pytest failed"; grep -E "FAILED|Error|assert|\[chain\]" gpurun_out/$TAG/pytest.log | tail -30; exit 1; }
grep -E "passed|failed|\[chain\]" gpurun_out/$TAG/pytest.log | tail -20
timeout -k 10 300 python -u tools/chain_trace.py --layer 10 > gpurun_out/$TAG/trace_l10.txt 2>&1 || { echo "trace failed"; tail -5 gpurun_out/$TAG/trace_l10.txt; exit 1; }
grep -v "^{" gpurun_out/$TAG/trace_l10.txt
for c in 1 0; do
  timeout -k 10 300 python -u tools/pipeline_bench.py --minutes 2 --no-cpu --mode sequential --serial --dec-chain $c \
      > gpurun_out/$TAG/seq_chain$c.json 2> gpurun_out/$TAG/seq_chain$c.err || { echo "seq $c failed"; tail -5 gpurun_out/$TAG/seq_chain$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$TAG/seq_chain$c.json'))['sequential']; print('chain $c seq 2 min RTF', d['value'], 'asr', d['asr_wall_s'], 'tokens', d['tokens'])"
done
