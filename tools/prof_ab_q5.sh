# rocprofv3 kernel stats + per-layer cross-attention durations of one Q5_0 bench step, for two library
# builds:  tools/prof_ab_q5.sh LIB_A LIB_B [TAG]   (paths relative to the repo; outputs gpurun_out/TAG/{a,b}_*, TAG r06i)
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
R=$GRAFT_REPO_ROOT
T=${3:-r06i}
mkdir -p $R/gpurun_out/$T
(cd $R && timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('large-v3-q5_0')") || exit 1
cd /tmp && export TMPDIR=/tmp
for v in a b; do
  if [ $v = a ]; then export OWK_LIB=$R/$1; else export OWK_LIB=$R/$2; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/$v -o run -- \
      python3 $R/bench.py --model large-v3-q5_0 --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $R/gpurun_out/$T/$v.json 2> $R/gpurun_out/$T/$v.err || exit 1
  (cd $R && python3 tools/prof_summary.py gpurun_out/$T/$v > gpurun_out/$T/${v}_stats.txt) || exit 1
  (cd $R && python3 tools/attn_by_layer.py gpurun_out/$T/$v > gpurun_out/$T/${v}_bylayer.txt) || exit 1
  rm -f $R/gpurun_out/$T/$v/*kernel_trace.csv
done
