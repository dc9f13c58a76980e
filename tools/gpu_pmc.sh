#!/bin/bash
# HBM traffic of the bench kernels: rocprofv3 PMC pass (FETCH_SIZE), counters in their own run
set -o pipefail
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/fetch -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/bench.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py gpurun_out/$TAG/fetch FETCH_SIZE > gpurun_out/$TAG/fetch_summary.txt
python3 tools/prof_summary.py gpurun_out/$TAG/fetch > gpurun_out/$TAG/fetch_kernel_stats.txt || true
head -5 gpurun_out/$TAG/fetch_summary.txt
rm -rf gpurun_out/$TAG/fetch   # per-dispatch CSVs are too large to copy back
