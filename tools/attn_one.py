"""One shape of the one_chunk cross attention (owk_debug_attn_cross, random q/k/v over rotated K/V
copies) for counter runs: python tools/attn_one.py ROWS KEYS [ITERS]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open-whisper-kit_amd", "python"))
import owk  # noqa: E402

L = owk.load()
L.owk_debug_attn_cross.restype = C.c_double
u16 = C.POINTER(C.c_uint16)
L.owk_debug_attn_cross.argtypes = [C.c_int] * 6 + [C.c_float, u16, u16, u16, u16, C.c_int]
R, T = int(sys.argv[1]), int(sys.argv[2])
it = int(sys.argv[3]) if len(sys.argv) > 3 else 20
which = int(os.environ.get("OWK_ATTN_WHICH", "1"))
print(f"rows {R} keys {T} which {which}: {L.owk_debug_attn_cross(0, which, R, 20, T, 0, 0.35, None, None, None, None, it):.2f} us")
