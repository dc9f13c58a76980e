#!/bin/bash
# Closing measurements of a round on the final tree, in two calls:
#   tools/gpu_closing.sh TAG prof   rocprofv3 --kernel-trace --stats + the PMC FETCH_SIZE pass of each bench model
#                                     (gpurun_out/TAG/<model>/; copied to profiles/r<NN>_* for bench.py PROFILES)
#   tools/gpu_closing.sh TAG bench  the three bench lines WITH the reference CPU leg and the clip-0 token check,
#                                     configs[4] at 10 min (both modes)
set -o pipefail
TAG=${1:-r05z}
PART=${2:-prof}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
if [ "$PART" = prof ]; then
  bash tools/gpu_profiles.sh $TAG large-v3 large-v3-turbo large-v3-q5_0
  exit $?
fi
[ "$PART" = bench ] || exit 2
for m in large-v3 large-v3-turbo large-v3-q5_0; do
  timeout -k 10 900 python bench.py --model $m > gpurun_out/$TAG/bench_$m.json 2> gpurun_out/$TAG/bench_$m.err \
      || { echo "$m bench failed"; tail -5 gpurun_out/$TAG/bench_$m.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/$TAG/bench_$m.json')); r=d.get('roofline') or {}
print('$m RTF', d['value'], 'ms/step', d['ms_per_step'], 'dom', r.get('kernel_class'), 'frac', r.get('frac'),
      'ev/rocprof', r.get('events_vs_rocprof'), 'rocprof dom', r.get('rocprof_dominant_class'),
      'parity', (d.get('parity') or {}).get('tokens_equal'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 600 python -u tools/pipeline_bench.py --minutes 10 --no-cpu > gpurun_out/$TAG/pipeline.json 2> gpurun_out/$TAG/pipeline.err \
    || { echo "pipeline failed"; tail -5 gpurun_out/$TAG/pipeline.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/$TAG/pipeline.json'))
print('configs[4] chunked', d['chunked']['value'], 'sequential', d['sequential']['value'], 'asr_wall', d['sequential']['asr_wall_s'])"
