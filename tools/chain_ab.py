"""Per-layer device time of the decoder's matmul + LayerNorm chain (no attention), large-v3 shapes,
one captured hipGraph, per chain form (owk_debug_decode_chain2 variants, whisper_api.cpp).

    python tools/chain_ab.py [--rows 32,16,8,4,1] [--variants 0,5,1]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open-whisper-kit_amd", "python"))
import owk  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", default="32,16,8,4,1")
ap.add_argument("--variants", default=None, help="default: 0,1 at > 16 rows, 0,5,1 otherwise")
ap.add_argument("--iters", type=int, default=40)
a = ap.parse_args()
L = owk.load()
f = L.owk_debug_decode_chain2
f.restype = C.c_double
f.argtypes = [C.c_int] * 5
for R in (int(x) for x in a.rows.split(",")):
    vs = [int(x) for x in a.variants.split(",")] if a.variants else ((0, 1, 0, 1) if R > 16 else (0, 5, 1, 0, 5))
    for v in vs:
        print(f"R={R} variant {v}: {f(0, R, 8, a.iters, v):.2f} us per layer", flush=True)
