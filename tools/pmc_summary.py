#!/usr/bin/env python3
"""Per-kernel mean of a rocprofv3 --pmc counter (e.g. FETCH_SIZE) from run_counter_collection.csv.

Writes a small table (kernel, dispatches, mean counter value per dispatch) so the multi-MB
per-dispatch CSV need not leave the GPU box:
    python tools/pmc_summary.py <dir> FETCH_SIZE > summary.txt
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        print("no counter_collection.csv under", d)
        return
    tot = defaultdict(float)
    cnt = defaultdict(int)
    with open(files[0]) as f:
        rd = csv.DictReader(f)
        for r in rd:
            if r.get("Counter_Name") != counter:
                continue
            k = r.get("Kernel_Name", "?")
            tot[k] += float(r["Counter_Value"])
            cnt[k] += 1
    print(f"# {counter} per dispatch (rocprofv3 units), source {os.path.basename(files[0])}")
    print(f"{'dispatches':>10} {'mean':>16} {'total':>18}  kernel")
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"{cnt[k]:10d} {tot[k] / cnt[k]:16.1f} {tot[k]:18.1f}  {k}")


if __name__ == "__main__":
    for c in (sys.argv[2] if len(sys.argv) > 2 else "FETCH_SIZE").split(","):
        main(sys.argv[1], c)
