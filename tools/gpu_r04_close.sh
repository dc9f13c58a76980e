#!/bin/bash
# round-4 closing measurements on the committed profiles: the three bench lines, then configs[4]
# (10 min, both modes)
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models

timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench_f16.json 2> gpurun_out/$TAG/bench_f16.err || { echo "f16 bench failed"; tail -5 gpurun_out/$TAG/bench_f16.err; exit 1; }
timeout -k 10 600 python bench.py --model large-v3-turbo --no-cpu-baseline > gpurun_out/$TAG/bench_turbo.json 2> gpurun_out/$TAG/bench_turbo.err || { echo "turbo bench failed"; exit 1; }
timeout -k 10 600 python bench.py --model large-v3-q5_0 --no-cpu-baseline > gpurun_out/$TAG/bench_q5.json 2> gpurun_out/$TAG/bench_q5.err || { echo "q5 bench failed"; exit 1; }
for m in f16 turbo q5; do python -c "
import json,sys; d=json.load(open('gpurun_out/$TAG/bench_$m.json')); r=d.get('roofline') or {}
print('$m', 'RTF', d['value'], 'ms/step', d['ms_per_step'], 'dom', r.get('kernel_class'), 'frac', r.get('frac'), 'ev/rocprof', r.get('events_vs_rocprof'), 'parity', (d.get('parity') or {}).get('tokens_equal'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
timeout -k 10 400 python -u tools/pipeline_bench.py --minutes 10 --no-cpu > gpurun_out/$TAG/pipeline.json 2> gpurun_out/$TAG/pipeline.err || { echo "pipeline failed"; tail -5 gpurun_out/$TAG/pipeline.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/$TAG/pipeline.json'))
print('configs[4] chunked', d['chunked']['value'], 'sequential', d['sequential']['value'], 'asr_wall', d['sequential']['asr_wall_s'], 'diarize_wall', d['sequential']['diarize_wall_s'])"
