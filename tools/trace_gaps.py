#!/usr/bin/env python3
"""GPU busy time vs wall span of a rocprofv3 --kernel-trace CSV: the idle gaps between kernels,
bucketed (dispatch-sized < 10 us, 10-100 us, >= 100 us = host work / syncs), over the dispatches
after the first `--skip` seconds of the trace (or in its final `--last` seconds).

    python tools/trace_gaps.py gpurun_out/<tag>/prof [--skip 0]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=float, default=0.0)
    ap.add_argument("--last", type=float, default=0.0, help="only the dispatches of the trace's final N seconds")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    t0 = ev[0][0] + int(a.skip * 1e9)
    if a.last > 0:
        t0 = max(t0, max(e for _, e, _ in ev) - int(a.last * 1e9))
    ev = [e for e in ev if e[0] >= t0]
    busy, gaps, end = 0, {"<10us": [0, 0], "10-100us": [0, 0], ">=100us": [0, 0]}, ev[0][0]
    for s, e, _ in ev:
        if s > end:
            g = (s - end) / 1e3
            k = "<10us" if g < 10 else "10-100us" if g < 100 else ">=100us"
            gaps[k][0] += 1
            gaps[k][1] += g
        busy += max(0, e - max(s, end))
        end = max(end, e)
    span = (end - ev[0][0]) / 1e3
    print(f"# {path}: {len(ev)} dispatches after {a.skip} s")
    print(f"span {span / 1e3:.2f} ms, kernels busy {busy / 1e6:.2f} ms ({100 * busy / 1e3 / span:.1f} %)")
    for k, (n, t) in gaps.items():
        print(f"gaps {k:>9}: {n:7d} totalling {t / 1e3:9.2f} ms")


if __name__ == "__main__":
    main()
