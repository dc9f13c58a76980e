#!/bin/bash
# one rocprofv3 PMC pass over a 1-step bench with the counters given (comma list, one block's limits)
set -o pipefail
TAG=${1:-pmcsq}
CTRS=${2:-SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_VALU,SQ_WAIT_ANY}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc ${CTRS//,/ } --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/raw -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/bench.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py gpurun_out/$TAG/raw $CTRS > gpurun_out/$TAG/summary.txt
rm -rf gpurun_out/$TAG/raw
grep -A4 "^#" gpurun_out/$TAG/summary.txt | head -60
