#!/usr/bin/env python3
"""Kernel concurrency in a rocprofv3 --kernel-trace CSV: sum of kernel durations vs the union of busy
intervals (overlap > 1 means kernels ran concurrently), per queue / stream id, over the dispatches after
the first `--skip` seconds.

    python tools/trace_overlap.py gpurun_out/<tag>/prof [--skip 0]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=float, default=0.0)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    ev, per_q = [], collections.Counter()
    with open(path) as f:
        rd = csv.DictReader(f)
        cols = rd.fieldnames
        qcol = next((c for c in ("Queue_Id", "Stream_Id") if c in cols), None)
        for r in rd:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            if qcol:
                per_q[r[qcol]] += 1
    ev.sort()
    t0 = ev[0][0] + int(a.skip * 1e9)
    ev = [e for e in ev if e[0] >= t0]
    total = sum(e - s for s, e in ev)
    union, cur_s, cur_e = 0, ev[0][0], ev[0][1]
    for s, e in ev[1:]:
        if s > cur_e:
            union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    span = ev[-1][1] - ev[0][0]
    print(f"kernels {len(ev)}  sum {total / 1e6:.1f} ms  busy union {union / 1e6:.1f} ms  span {span / 1e6:.1f} ms  "
          f"concurrency {total / max(union, 1):.3f}")
    print("dispatches per", qcol, dict(per_q.most_common(8)))


if __name__ == "__main__":
    main()
