#!/bin/bash
# measurement refresh (outputs under gpurun_out/$TAG): large-v3-turbo and large-v3 Q5_0 bench lines,
# the configs[4] pipeline (sequential and chunked), rocprofv3 FETCH_SIZE and SQ MFMA counter passes
set -o pipefail
TAG=${1:-meas}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
run() { echo "== $1"; shift; "$@"; }
run turbo timeout -k 10 400 python bench.py --model large-v3-turbo --steps 2 --warmup 1 > gpurun_out/$TAG/turbo.json 2> gpurun_out/$TAG/turbo.err || { tail -5 gpurun_out/$TAG/turbo.err; exit 1; }
cat gpurun_out/$TAG/turbo.json
run q5 timeout -k 10 400 python bench.py --model large-v3-q5_0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/q5.json 2> gpurun_out/$TAG/q5.err || { tail -5 gpurun_out/$TAG/q5.err; exit 1; }
cat gpurun_out/$TAG/q5.json
run pipeline timeout -k 10 600 python -u tools/pipeline_bench.py --minutes 10 --no-cpu > gpurun_out/$TAG/pipeline.json 2> gpurun_out/$TAG/pipeline.err || { tail -20 gpurun_out/$TAG/pipeline.err; exit 1; }
cat gpurun_out/$TAG/pipeline.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run fetch timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/fetch -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $R/gpurun_out/$TAG/fetch_bench.json 2> $R/gpurun_out/$TAG/fetch_bench.err || exit 1
python3 $R/tools/pmc_summary.py $R/gpurun_out/$TAG/fetch FETCH_SIZE > $R/gpurun_out/$TAG/fetch_summary.txt
rm -rf $R/gpurun_out/$TAG/fetch
CTRS=SQ_WAVES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_F16,SQ_INSTS_VALU_MFMA_MOPS_I8,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,GRBM_GUI_ACTIVE
run sq timeout -k 10 600 rocprofv3 --pmc ${CTRS//,/ } --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/sq -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $R/gpurun_out/$TAG/sq_bench.json 2> $R/gpurun_out/$TAG/sq_bench.err || exit 1
python3 $R/tools/pmc_summary.py $R/gpurun_out/$TAG/sq $CTRS > $R/gpurun_out/$TAG/sq_summary.txt
python3 $R/tools/prof_summary.py $R/gpurun_out/$TAG/sq > $R/gpurun_out/$TAG/sq_kernel_stats.txt || true
rm -rf $R/gpurun_out/$TAG/sq
head -8 $R/gpurun_out/$TAG/fetch_summary.txt
