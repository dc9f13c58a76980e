set -o pipefail
export PYTHONPATH=open-whisper-kit_amd/python
OWK_INJ_DUMP=gpurun_out/inj timeout -k 10 1000 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf > gpurun_out/r5_pytest.log 2>&1
echo "pytest exit $?" >> gpurun_out/r5_pytest.log
