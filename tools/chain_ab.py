"""Per-layer device time of the decoder's matmul + LayerNorm chain (no attention), large-v3 shapes,
one captured hipGraph, per chain form (owk_debug_decode_chain2 variants, whisper_api.cpp)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open-whisper-kit_amd", "python"))
import owk  # noqa: E402

L = owk.load()
f = L.owk_debug_decode_chain2
f.restype = C.c_double
f.argtypes = [C.c_int] * 5
for R in (32, 16, 8, 4, 1):
    for v in ((0, 1, 0, 1) if R > 16 else (0, 5, 1, 0, 5)):
        print(f"R={R} variant {v}: {f(0, R, 8, 40, v):.2f} us per layer", flush=True)
