#!/bin/bash
# Round 5: the persistent decode chain (csrc/k_chain.hip) -- bit-identity against the launch chain, then
# configs[4] sequential 2 min with and without it, and its kernel trace (graphs on, packet capture off)
set -o pipefail
TAG=${1:-r05c}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_chain.py > gpurun_out/$TAG/pytest.log 2>&1 \
    || { echo "pytest failed"; grep -E "FAILED|Error|assert|\[chain\]" gpurun_out/$TAG/pytest.log | tail -30; exit 1; }
grep -E "passed|failed|\[chain\]" gpurun_out/$TAG/pytest.log | tail -20
for c in 1 0; do
  timeout -k 10 300 python -u tools/pipeline_bench.py --minutes 2 --no-cpu --mode sequential --serial --dec-chain $c \
      > gpurun_out/$TAG/seq_chain$c.json 2> gpurun_out/$TAG/seq_chain$c.err || { echo "seq $c failed"; tail -5 gpurun_out/$TAG/seq_chain$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$TAG/seq_chain$c.json')); print('chain $c seq 2 min', d['sequential'])"
done
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/seqtr -o run -- \
    python $GRAFT_REPO_ROOT/tools/pipeline_bench.py --minutes 2 --no-cpu --mode sequential --serial \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.err || { echo "trace failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py /tmp/seqtr > gpurun_out/$TAG/kernel_stats.txt && head -16 gpurun_out/$TAG/kernel_stats.txt
