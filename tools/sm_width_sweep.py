"""soft_max decoder attention at one row (configs[4]'s self attention: 20 heads, up to n_text_ctx keys):
device time of the single-block kernel at 256 / 1024 threads and of the key-split form, by key count
(owk_debug_attn_softmax)."""
import ctypes as C
import os

L = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "open-whisper-kit_amd/lib/libwhisper.so"))
L.owk_debug_attn_softmax.restype = C.c_double
L.owk_debug_attn_softmax.argtypes = [C.c_int] * 5 + [C.c_void_p, C.c_void_p, C.c_int]
for R in (1, 2):
    for T in (64, 128, 200, 256, 320, 384, 448):
        row = {}
        for split, name in ((0, "engine"), (256, "nt256"), (512, "nt512"), (1024, "nt1024"), (1, "keysplit")):
            row[name] = round(min(L.owk_debug_attn_softmax(0, split, R, 20, T, None, None, 50) for _ in range(3)), 2)
        print({"rows": R, "keys": T, **row}, flush=True)
