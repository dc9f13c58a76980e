"""GPU check of the Q5_0 x Q8_0 GEMM against a numpy restatement of ggml's x86 path."""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "open-whisper-kit_amd", "python"))
import owk, owk_synth as S
L = owk.load()
L.owk_debug_gemm_q5.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_float), C.c_void_p, C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
rng = np.random.default_rng(0)

def q8_ref(a):  # x86 quantize_row_q8_0
    b = a.reshape(a.shape[0], -1, 32)
    am = np.abs(b).max(-1)
    d = (am / np.float32(127)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(am != 0, np.float32(127) / am, np.float32(0)).astype(np.float32)
    q = np.rint((b * idv[..., None]).astype(np.float32)).astype(np.int8)
    return q.reshape(a.shape), d.astype(np.float16).astype(np.float32)

def q5_vals(blocks, N, K):
    bl = np.frombuffer(blocks, np.uint8).reshape(N, K // 32, 22)
    d = bl[..., 0:2].copy().view("<f2")[..., 0].astype(np.float32)
    qh = bl[..., 2:6].copy().view("<u4")[..., 0]
    qs = bl[..., 6:22]
    lo = np.concatenate([qs & 15, qs >> 4], axis=-1).astype(np.int32)
    hb = ((qh[..., None] >> np.arange(32)) & 1).astype(np.int32)
    return (lo | (hb << 4)) - 16, d

for M, N, K in ((8, 384, 384), (32, 1280, 5120), (24, 3840, 1280), (17, 5120, 1280), (40, 1536, 384), (300, 384, 1536), (1500, 1152, 384)):
    a = (rng.standard_normal((M, K)) * 0.7).astype(np.float32)
    wf = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    blocks = S.q5_0_blocks(wf)
    out = np.zeros((M, N), np.float32)
    q = np.zeros((M, K), np.int8); dq = np.zeros((M, K // 32), np.float32)
    assert L.owk_debug_gemm_q5(0, M, N, K, a.ctypes.data_as(C.POINTER(C.c_float)), blocks, out.ctypes.data_as(C.POINTER(C.c_float)),
                               q.ctypes.data, dq.ctypes.data) == 0
    qr, dr = q8_ref(a)
    wq, wd = q5_vals(blocks, N, K)
    isum = np.einsum("mbk,nbk->mnb", qr.reshape(M, -1, 32).astype(np.int64), wq.astype(np.int64))
    ref = (isum.astype(np.float64) * (dr[:, None, :].astype(np.float64) * wd[None, :, :].astype(np.float64))).sum(-1)
    print(M, N, K, "q8 equal", np.array_equal(q, qr), "d equal", np.array_equal(dq.astype(np.float16).astype(np.float32), dr),
          "gemm max rel", float(np.abs(out - ref).max() / np.abs(ref).max()))
