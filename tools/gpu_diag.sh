#!/bin/bash
# diagnostics: large-GEMM epilogue timings, counter list of this rocprofv3 (outputs under gpurun_out/$TAG)
set -o pipefail
TAG=${1:-diag}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -u tools/gemm_big_check.py > gpurun_out/$TAG/gemm.jsonl 2> gpurun_out/$TAG/gemm.err || { echo "gemm check failed rc=$?"; tail -20 gpurun_out/$TAG/gemm.err; exit 1; }
grep -v '"kernel": "128"' gpurun_out/$TAG/gemm.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/$TAG/counters.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
grep -o "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*\|SQ_BUSY[A-Z_]*\|GRBM_GUI_ACTIVE" gpurun_out/$TAG/counters.txt | sort -u | head -40
