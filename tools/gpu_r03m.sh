#!/bin/bash
# 16x25 mel DFT: mel / parity suites, smoke, then turbo bench with its reference token check
set -o pipefail
T=r03m3
mkdir -p gpurun_out/$T
export OWK_MODEL_CACHE=/tmp/owk_models
bash tools/gpu_tests.sh $T "tests/test_gpu_parity.py tests/test_gpu_large.py -k 'mel or large_batch32 or greedy or tokens'" 0 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -3 gpurun_out/$T/smoke.log
timeout -k 10 500 python bench.py --model large-v3-turbo --steps 2 --warmup 1 > gpurun_out/$T/turbo.json 2> gpurun_out/$T/turbo.err || { tail -5 gpurun_out/$T/turbo.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$T/turbo.json'));print(d['value'], d['ms_per_step'], d.get('parity'))"
grep -E "\] mel " gpurun_out/$T/turbo.err
