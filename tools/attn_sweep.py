"""Device time of the one_chunk decode attention kernel (k_attn_step, cross instantiation) against
the key count: 32 rows x 20 heads, T = 64 .. 1536 keys (owk_debug_attn_cross, random q/k/v)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk  # noqa: E402

L = owk.load()
L.owk_debug_attn_cross.restype = C.c_double
u16 = C.POINTER(C.c_uint16)
L.owk_debug_attn_cross.argtypes = [C.c_int] * 6 + [C.c_float, u16, u16, u16, u16, C.c_int]
for R in (32, 1):
    for T in (64, 128, 192, 256, 384, 512, 1024, 1500):
        us = min(L.owk_debug_attn_cross(0, 1, R, 20, T, 0, 0.35, None, None, None, None, 50) for _ in range(3))
        print(json.dumps({"rows": R, "keys": T, "us": round(us, 2), "us_per_chunk": round(us / ((T + 63) // 64), 2),
                          "GBps": round(2 * 2 * R * 20 * T * 64 / us / 1e3, 1)}), flush=True)
