#!/bin/bash
# parity tests, then the bench with an env knob on/off: bash tools/gpu_ab.sh TAG VAR
set -o pipefail
TAG=${1:-ab}; VAR=${2:-OWK_DEC_LNP}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
for V in 1 0; do
  env $VAR=$V timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/b$V.json 2> gpurun_out/$TAG/b$V.err || { echo "bench $V failed"; tail -20 gpurun_out/$TAG/b$V.err; exit 1; }
  echo "$VAR=$V $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' gpurun_out/$TAG/b$V.json)"
  grep "\[bench\]" gpurun_out/$TAG/b$V.err | head -8
done
