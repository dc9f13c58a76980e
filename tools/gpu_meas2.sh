#!/bin/bash
# measurement refresh on the current build: SortFormer offline + streaming benches with rocprofv3 kernel
# stats, FETCH_SIZE and SQ (MFMA) counter passes over one large-v3 bench step
set -o pipefail
TAG=${1:-meas2}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
echo "== sortformer"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/sfprof -o run -- \
    python3 $R/tools/sf_bench.py --minutes 10 --cpu-seconds 0 --reps 2 > $R/gpurun_out/$TAG/sf.json 2> $R/gpurun_out/$TAG/sf.err || { tail -5 $R/gpurun_out/$TAG/sf.err; exit 1; }
python3 $R/tools/prof_summary.py $R/gpurun_out/$TAG/sfprof > $R/gpurun_out/$TAG/sf_kernel_stats.txt; rm -f $R/gpurun_out/$TAG/sfprof/*kernel_trace.csv
head -c 400 $R/gpurun_out/$TAG/sf.json; echo; head -12 $R/gpurun_out/$TAG/sf_kernel_stats.txt
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/sfsprof -o run -- \
    python3 $R/tools/sf_stream_bench.py --streams 32 --seconds 30 > $R/gpurun_out/$TAG/sfs.json 2> $R/gpurun_out/$TAG/sfs.err || { tail -5 $R/gpurun_out/$TAG/sfs.err; exit 1; }
python3 $R/tools/prof_summary.py $R/gpurun_out/$TAG/sfsprof > $R/gpurun_out/$TAG/sfs_kernel_stats.txt; rm -f $R/gpurun_out/$TAG/sfsprof/*kernel_trace.csv
head -c 400 $R/gpurun_out/$TAG/sfs.json; echo
echo "== fetch"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/fetch -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $R/gpurun_out/$TAG/fetch_bench.json 2> $R/gpurun_out/$TAG/fetch_bench.err || exit 1
python3 $R/tools/pmc_summary.py $R/gpurun_out/$TAG/fetch FETCH_SIZE > $R/gpurun_out/$TAG/fetch_summary.txt
rm -rf $R/gpurun_out/$TAG/fetch
echo "== sq"
CTRS=SQ_WAVES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_F16,SQ_INSTS_VALU_MFMA_MOPS_I8,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,GRBM_GUI_ACTIVE
timeout -k 10 600 rocprofv3 --pmc ${CTRS//,/ } --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/sq -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $R/gpurun_out/$TAG/sq_bench.json 2> $R/gpurun_out/$TAG/sq_bench.err || exit 1
python3 $R/tools/pmc_summary.py $R/gpurun_out/$TAG/sq $CTRS > $R/gpurun_out/$TAG/sq_summary.txt
rm -rf $R/gpurun_out/$TAG/sq
cd $R && python3 tools/mfma_util.py gpurun_out/$TAG/sq_summary.txt | head -12
