#!/bin/bash
# A/B of decode-path variants on the GPU: optional pytest args, then one bench line per
# "NAME:ENV=VAL[,ENV=VAL]" variant (no CPU baseline), then rocprofv3 kernel stats of the default.
#   bash tools/gpu_ab.sh TAG "pytest args|none" "default:" "xattn1:OWK_XATTN=1" ...
set -o pipefail
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
if [ "$ARGS" != "none" ]; then
  bash tools/gpu_tests.sh $TAG "$ARGS" 0 || exit $?
fi
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  ( IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done
    timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      > gpurun_out/$TAG/bench_$name.json 2> gpurun_out/$TAG/bench_$name.err ) || { echo "bench $name failed"; tail -20 gpurun_out/$TAG/bench_$name.err; exit 1; }
  echo "$name: $(python3 tools/bench_line.py gpurun_out/$TAG/bench_$name.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_bench.err || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py gpurun_out/$TAG/prof > gpurun_out/$TAG/kernel_stats.txt
rm -f gpurun_out/$TAG/prof/*kernel_trace.csv
head -22 gpurun_out/$TAG/kernel_stats.txt
