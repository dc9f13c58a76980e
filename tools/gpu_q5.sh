export OWK_MODEL_CACHE=/tmp/owk_models
mkdir -p gpurun_out/q5
timeout -k 10 600 python -u -m pytest tests/test_q5.py -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/q5/pytest.log 2>&1; rc=$?; tail -40 gpurun_out/q5/pytest.log; exit $rc
