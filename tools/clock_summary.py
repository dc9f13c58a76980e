#!/usr/bin/env python3
"""Effective GFX clock per kernel from a rocprofv3 --pmc GRBM_COUNT --kernel-trace run: GRBM_COUNT
(cycles, summed over the XCDs) / the dispatch's duration, averaged per kernel name (the top ones by
time). A power-managed clock drop shows as a lower ratio for the same kernel.
    python tools/clock_summary.py <dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        print("no counter_collection.csv under", d)
        return
    cyc = {}
    with open(cc[0]) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") == "GRBM_COUNT":
                cyc[r["Dispatch_Id"]] = (r.get("Kernel_Name", "?"), float(r["Counter_Value"]))
    dur = {}
    if kt:
        with open(kt[0]) as f:
            for r in csv.DictReader(f):
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot_t, tot_c, n = defaultdict(float), defaultdict(float), defaultdict(int)
    for k, (name, c) in cyc.items():
        if k in dur and dur[k] > 0:
            tot_t[name] += dur[k]
            tot_c[name] += c
            n[name] += 1
    print(f"# GRBM_COUNT / duration per kernel (MHz x XCDs), source {os.path.basename(cc[0])}")
    for name in sorted(tot_t, key=lambda x: -tot_t[x])[:12]:
        print(f"{n[name]:8d} {tot_t[name] / n[name]:9.2f} us {tot_c[name] / tot_t[name]:9.1f}  {name[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])
