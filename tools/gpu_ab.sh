#!/bin/bash
# interleaved A/B of bench.py under two environment settings on one box:  tools/gpu_ab.sh TAG "ENV_A" "ENV_B" [bench args]
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
T=gpurun_out/$TAG; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
for r in 1 2; do
  for v in A B; do
    E=$A; [ $v = B ] && E=$B
    env $E timeout -k 10 400 python bench.py --no-cpu-baseline --no-prof "$@" > $T/$v$r.json 2> $T/$v$r.err || { tail -5 $T/$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('$T/$v$r.json'));print('$v$r [$E]', d['value'], d['ms_per_step'])"
  done
done
