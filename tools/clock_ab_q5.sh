# effective clock of the Q5_0 bench's kernels with the current library and with the pre-change build
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06j
(cd $R && timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('large-v3-q5_0')") || exit 1
cd /tmp && export TMPDIR=/tmp
for v in new base; do
  if [ $v = base ]; then export OWK_LIB=$R/open-whisper-kit_amd/lib_ab/libwhisper_base.so; else unset OWK_LIB; fi
  timeout -s KILL 300 rocprofv3 --pmc GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/r06j/$v -o run -- \
      python3 $R/bench.py --model large-v3-q5_0 --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $R/gpurun_out/r06j/$v.json 2> $R/gpurun_out/r06j/$v.err || exit 1
  (cd $R && python3 tools/clock_summary.py gpurun_out/r06j/$v > gpurun_out/r06j/${v}_clock.txt) || exit 1
  rm -rf $R/gpurun_out/r06j/$v
done
