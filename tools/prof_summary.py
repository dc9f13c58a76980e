#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max us, %) of a rocprofv3 --kernel-trace run.

Reads the rocpd SQLite output (<dir>/*_results.db) or kernel_stats.csv, prints a table.
    python tools/prof_summary.py gpurun_out/r1a/prof > profiles/archive/r01_bench_kernel_stats.txt
"""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
         "from kernels group by name order by sum(end-start) desc")
    try:
        return [(r[0], r[1], r[2] / 1e3, r[3] / 1e3, r[4] / 1e3, r[5] / 1e3) for r in c.execute(q)]
    except sqlite3.OperationalError:
        return [(r[0], r[1], r[2], r[3], None, None) for r in
                c.execute("select name, total_calls, total_duration, average from top_kernels")]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    return out


def main(d):
    dbs = glob.glob(os.path.join(d, "**", "*_results.db"), recursive=True)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    tot = sum(r[2] for r in rows)
    print(f"# source: {(csvs or dbs)[0]}")
    print(f"{'calls':>8} {'total_us':>12} {'avg_us':>10} {'min_us':>9} {'max_us':>9} {'pct':>6}  kernel")
    for name, n, t, a, mn, mx in rows:
        f = lambda v: f"{v:9.2f}" if v is not None else f"{'-':>9}"
        print(f"{n:8d} {t:12.1f} {a:10.3f} {f(mn)} {f(mx)} {100 * t / tot:6.2f}  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
