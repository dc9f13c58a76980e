#!/usr/bin/env python3
"""Per-dispatch durations of the cross-attention kernel from a rocprofv3 kernel trace, averaged by decoder layer
(dispatch index mod n_layers) and by the kernel launched just before it.  python tools/attn_by_layer.py <dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

NAME = "_ZN3owk11k_attn_stepILb0ELb1ELi2E"
d = sys.argv[1]
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = []
with open(kt) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
att = [(i, s, e) for i, (s, e, n) in enumerate(rows) if n.startswith(NAME)]
by_layer = defaultdict(list)
by_prev = defaultdict(list)
gaps = []
for j, (i, s, e) in enumerate(att):
    by_layer[j % 32].append((e - s) / 1e3)
    prev = rows[i - 1]
    by_prev[prev[2][:60]].append((e - s) / 1e3)
    gaps.append((s - prev[1]) / 1e3)
print("layer: mean us")
print(" ".join(f"{k}:{sum(v) / len(v):.1f}" for k, v in sorted(by_layer.items())))
for k, v in by_prev.items():
    print(f"after {k}: n={len(v)} mean {sum(v) / len(v):.2f} us")
gaps.sort()
print(f"gap from the previous kernel's end: median {gaps[len(gaps) // 2]:.2f} us, p10 {gaps[len(gaps) // 10]:.2f}, "
      f"p90 {gaps[9 * len(gaps) // 10]:.2f}")
durs = sorted((e - s) / 1e3 for _, s, e in att)
print(f"durations: p10 {durs[len(durs) // 10]:.1f} median {durs[len(durs) // 2]:.1f} p90 {durs[9 * len(durs) // 10]:.1f}")
