#!/bin/bash
# Round-5 closing measurements on one box: rocprofv3 --kernel-trace --stats and the PMC FETCH_SIZE pass of
# each bench model (copied into profiles/r05_* so the bench lines cross-check against this tree), the three
# bench lines WITH the reference CPU leg and the clip-0 token check, configs[4] (10 min, both modes) and its
# sequential kernel trace with graphs on (packet capture off: profiles/r05_rocprof_graph_segv.txt).
#   tools/gpu_r05_final.sh TAG
set -o pipefail
TAG=${1:-r05f}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models
bash tools/gpu_profiles.sh $TAG large-v3 large-v3-turbo large-v3-q5_0 || exit 1
cp gpurun_out/$TAG/large-v3/kernel_stats.txt profiles/r05_bench_kernel_stats.txt
cp gpurun_out/$TAG/large-v3/fetch_summary.txt profiles/r05_pmc_fetch_summary.txt
cp gpurun_out/$TAG/large-v3-turbo/kernel_stats.txt profiles/r05_turbo_kernel_stats.txt
cp gpurun_out/$TAG/large-v3-turbo/fetch_summary.txt profiles/r05_turbo_pmc_fetch_summary.txt
cp gpurun_out/$TAG/large-v3-q5_0/kernel_stats.txt profiles/r05_q5_kernel_stats.txt
cp gpurun_out/$TAG/large-v3-q5_0/fetch_summary.txt profiles/r05_q5_pmc_fetch_summary.txt
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
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/seqtr -o run -- \
    python $GRAFT_REPO_ROOT/tools/pipeline_bench.py --minutes 2 --no-cpu --mode sequential --serial \
    > $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/seq.err || { echo "trace failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py /tmp/seqtr > gpurun_out/$TAG/c4seq_kernel_stats.txt && head -14 gpurun_out/$TAG/c4seq_kernel_stats.txt
