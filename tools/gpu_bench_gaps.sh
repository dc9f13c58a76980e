#!/bin/bash
# GPU busy vs wall over the bench's steps (rocprofv3 kernel trace, analysed on the box)
set -o pipefail
TAG=${1:-gaps}
mkdir -p gpurun_out/$TAG
export OWK_MODEL_CACHE=/tmp/owk_models TMPDIR=/tmp
python3 -c "import sys; sys.path.insert(0,'open-whisper-kit_amd/python'); import owk_synth as S; S.ensure_model('large-v3')" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/bg -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err || { echo trace failed; exit 1; }
python - <<'PY'
import csv, glob
path = glob.glob('/tmp/bg/**/*kernel_trace.csv', recursive=True)[0]
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in csv.DictReader(open(path)))
# the timed steps: the last 3 of the 4 k_mel_norm-started steps
starts = [s for s, e, n in ev if 'k_mel_norm' in n]
print('steps (mel launches):', len(starts))
t0 = starts[-3]
ev = [x for x in ev if x[0] >= t0]
import collections
busy, end, gaps, prev = 0, ev[0][0], {}, ''
around = collections.Counter()
for s, e, n in ev:
    if s > end:
        g = (s - end) / 1e3
        k = '<5us' if g < 5 else '5-20us' if g < 20 else '20-100us' if g < 100 else '>=100us'
        gaps.setdefault(k, [0, 0.0]); gaps[k][0] += 1; gaps[k][1] += g
        if g >= 20: around[(k, prev[:40], n[:40])] += 1
    busy += max(0, e - max(s, end)); end = max(end, e); prev = n
span = end - ev[0][0]
print(f'3 steps: span {span/1e6:.1f} ms, kernels busy {busy/1e6:.1f} ms ({100*busy/span:.1f} %)')
for k, (n, t) in sorted(gaps.items()): print(f'gaps {k:>9}: {n:7d} totalling {t/1e3:8.2f} ms')
for (k, a, b), c in around.most_common(8): print(f'{c:6d} x {k}: after {a} -> before {b}')
PY
