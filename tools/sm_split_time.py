"""Key-split soft_max attention (k_sm_split_scores + k_sm_split_pv) device time per launch pair at 1-2 rows,
20 heads (owk_debug_attn_softmax split = 1), for the record of a change to its in-launch hand-off."""
import ctypes as C
import os

L = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "open-whisper-kit_amd/lib/libwhisper.so"))
L.owk_debug_attn_softmax.restype = C.c_double
L.owk_debug_attn_softmax.argtypes = [C.c_int] * 5 + [C.c_void_p, C.c_void_p, C.c_int]
for R in (1, 2):
    for T in (448, 1500):
        us = min(L.owk_debug_attn_softmax(0, 1, R, 20, T, None, None, 50) for _ in range(5))
        print({"rows": R, "keys": T, "keysplit_us": round(us, 2)}, flush=True)
