set -o pipefail
mkdir -p gpurun_out/r04h
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 600 python -u -m pytest tests/test_gpu_nofa.py tests/test_gpu_c4.py tests/test_gpu_kernels.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04h/pytest.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04h/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r04h/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/chain_ab.py > gpurun_out/r04h/chain_ab.txt 2>&1 && cat gpurun_out/r04h/chain_ab.txt &&
timeout -k 10 300 python -u tools/pipeline_bench.py --minutes 10 --no-cpu --mode sequential --whole-k-rows 0 > gpurun_out/r04h/seq_wk0.json 2> gpurun_out/r04h/seq_wk0.err && tail -c 600 gpurun_out/r04h/seq_wk0.json &&
timeout -k 10 300 python -u tools/pipeline_bench.py --minutes 10 --no-cpu --mode sequential > gpurun_out/r04h/seq.json 2> gpurun_out/r04h/seq.err && tail -c 600 gpurun_out/r04h/seq.json
