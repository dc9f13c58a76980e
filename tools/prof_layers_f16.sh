# per-layer cross-attention durations of one F16 bench step (rocprofv3 kernel trace)
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06w
(cd $R && timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('large-v3')") || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r06w/f16 -o run -- \
    python3 $R/bench.py --model large-v3 --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $R/gpurun_out/r06w/f16.json 2> $R/gpurun_out/r06w/f16.err || exit 1
(cd $R && python3 tools/attn_by_layer.py gpurun_out/r06w/f16 > gpurun_out/r06w/f16_bylayer.txt) || exit 1
rm -f $R/gpurun_out/r06w/f16/*kernel_trace.csv
