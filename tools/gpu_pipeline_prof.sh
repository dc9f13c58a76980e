#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pipep
export OWK_MODEL_CACHE=/tmp/owk_models
python -u -c "import sys; sys.path.insert(0,'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('large-v3')" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pipep/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/pipeline_bench.py --minutes 5 --no-cpu \
    > $GRAFT_REPO_ROOT/gpurun_out/pipep/pipeline.json 2> $GRAFT_REPO_ROOT/gpurun_out/pipep/pipeline.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/pipep/prof > gpurun_out/pipep/kernel_stats.txt
rm -f gpurun_out/pipep/prof/*kernel_trace.csv
cat gpurun_out/pipep/pipeline.json
head -22 gpurun_out/pipep/kernel_stats.txt
