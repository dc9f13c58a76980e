#!/usr/bin/env python3
"""MFMA utilisation per kernel from a rocprofv3 SQ counter pass (tools/gpu_measure.sh -> sq_summary.txt).

    python tools/mfma_util.py gpurun_out/<tag>/sq_summary.txt > profiles/<round>_mfma_util.txt

util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles): SQ_VALU_MFMA_BUSY_CYCLES sums the SIMD
cycles of every MFMA issued (16 per v_mfma_f32_16x16x32_f16, MI355X_MICROARCH.md), and
GRBM_GUI_ACTIVE counts the dispatch's busy cycles summed over the 8 XCDs. TFLOP/s from
SQ_INSTS_VALU_MFMA_MOPS_F16 / _I8 (512 FLOP / OPS per unit) over the same cycles at 2.4 GHz.
"""
import collections
import re
import sys

SIMDS, XCDS, CLK = 256 * 4, 8, 2.4e9


def main(path):
    cur, data = None, collections.defaultdict(dict)
    for line in open(path):
        if line.startswith("# "):
            cur = line.split()[1]
            continue
        p = line.split(None, 3)
        if len(p) == 4 and p[0].isdigit():
            data[p[3].strip()][cur] = (int(p[0]), float(p[1]))
    print(f"# MFMA utilisation per kernel (source {path}); cycles per dispatch = GRBM_GUI_ACTIVE / {XCDS}")
    print(f"{'dispatches':>10} {'us/disp':>9} {'mfma_util':>9} {'TFLOP/s':>9} {'TOPS_i8':>9}  kernel")
    rows = []
    for k, v in data.items():
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", (0, 0.0))[1]
        gui = v.get("GRBM_GUI_ACTIVE", (0, 0.0))[1]
        if busy <= 0 or gui <= 0:
            continue
        n = v.get("GRBM_GUI_ACTIVE")[0]
        cyc = gui / XCDS
        f16 = v.get("SQ_INSTS_VALU_MFMA_MOPS_F16", (0, 0.0))[1] * 512
        i8 = v.get("SQ_INSTS_VALU_MFMA_MOPS_I8", (0, 0.0))[1] * 512
        rows.append((busy * n, n, cyc / CLK * 1e6, busy / (SIMDS * cyc), f16 / (cyc / CLK) / 1e12, i8 / (cyc / CLK) / 1e12, k))
    for _, n, us, u, tf, ti, k in sorted(rows, reverse=True):
        print(f"{n:10d} {us:9.1f} {u:9.3f} {tf:9.1f} {ti:9.1f}  {k[:150]}")


if __name__ == "__main__":
    main(sys.argv[1])
