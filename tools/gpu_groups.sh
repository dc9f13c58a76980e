#!/bin/bash
# RTF vs number of concurrent clip groups (OWK_STREAM_GROUPS) for the default bench workload
set -o pipefail
mkdir -p gpurun_out/groups
export OWK_MODEL_CACHE=/tmp/owk_models
for G in ${GROUPS_LIST:-1 2 4}; do
  OWK_STREAM_GROUPS=$G timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-prof \
      > gpurun_out/groups/g$G.json 2> gpurun_out/groups/g$G.err || { echo "G=$G failed"; tail -20 gpurun_out/groups/g$G.err; exit 1; }
  echo "G=$G $(cat gpurun_out/groups/g$G.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
done
