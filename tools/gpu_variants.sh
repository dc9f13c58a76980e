#!/bin/bash
# turbo F16 and Q5_0 headline benches (bench.py contract, N = 1)
set -o pipefail
TAG=${1:-variants}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
for m in large-v3-turbo large-v3-q5_0; do
  timeout -k 10 500 python bench.py --model $m --steps 2 --warmup 1 > gpurun_out/$TAG/$m.json 2> gpurun_out/$TAG/$m.err || { tail -5 gpurun_out/$TAG/$m.err; exit 1; }
  head -c 200 gpurun_out/$TAG/$m.json; echo; grep -o '"parity": {[^}]*}' gpurun_out/$TAG/$m.json || true
done
