# rocprofv3 kernel stats of one Q5_0 bench step with the current library and with OWK_LIB's A/B build
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06i
(cd $R && timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('large-v3-q5_0')") || exit 1
(cd $R && timeout -k 10 120 python3 tools/sm_split_time.py > gpurun_out/r06i/sm_split.txt 2>&1) || exit 1
cd /tmp && export TMPDIR=/tmp
for v in new base; do
  if [ $v = base ]; then export OWK_LIB=$R/open-whisper-kit_amd/lib_ab/libwhisper_base.so; else unset OWK_LIB; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06i/$v -o run -- \
      python3 $R/bench.py --model large-v3-q5_0 --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $R/gpurun_out/r06i/$v.json 2> $R/gpurun_out/r06i/$v.err || exit 1
  (cd $R && python3 tools/prof_summary.py gpurun_out/r06i/$v > gpurun_out/r06i/${v}_stats.txt) || exit 1
  rm -f $R/gpurun_out/r06i/$v/*kernel_trace.csv
done
