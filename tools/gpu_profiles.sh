#!/bin/bash
# Profiles bench.py's roofline cross-checks read (bench.py PROFILES), for each bench model on this tree:
#   rocprofv3 --kernel-trace --stats of one bench step  -> profiles/r05_<m>_kernel_stats.txt (copied by hand)
#   rocprofv3 --pmc FETCH_SIZE of one bench step        -> profiles/r05_<m>_pmc_fetch_summary.txt
# (counters in a run of their own, MI355X_MICROARCH.md). Outputs under gpurun_out/$TAG/<model>.
#   tools/gpu_profiles.sh TAG [models...]
set -o pipefail
TAG=${1:-prof}
shift
MODELS=${@:-large-v3 large-v3-turbo large-v3-q5_0}
export OWK_MODEL_CACHE=/tmp/owk_models
R=$GRAFT_REPO_ROOT
for M in $MODELS; do
  O=$R/gpurun_out/$TAG/$M
  mkdir -p $O
  # model file first (not under the profiler)
  (cd $R && timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('$M')") || exit $?
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
      python3 $R/bench.py --model $M --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $O/prof_bench.json 2> $O/prof_bench.err || exit $?
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- \
      python3 $R/bench.py --model $M --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_bench.json 2> $O/pmc_bench.err || exit $?
  cd $R
  python3 tools/prof_summary.py $O/prof > $O/kernel_stats.txt || exit $?
  python3 tools/pmc_summary.py $O/fetch FETCH_SIZE > $O/fetch_summary.txt || exit $?
  rm -rf $O/fetch $O/prof/*kernel_trace.csv
  echo "== $M"; head -12 $O/kernel_stats.txt
done
