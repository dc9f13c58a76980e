"""Where the Q4_1 tiled GEMM (M > 64) departs from the numpy restatement of ggml's q4_1 x q8_1 path."""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "open-whisper-kit_amd", "python"))
import owk, owk_synth as S
L = owk.load()
L.owk_debug_gemm_quant.argtypes = [C.c_int] * 5 + [C.POINTER(C.c_float), C.c_void_p, C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
f16 = lambda x: x.astype(np.float16).astype(np.float32)
for M, N, K in ((300, 384, 1536), (65, 384, 384), (128, 128, 64)):
    rng = np.random.default_rng(M * 7 + N + K)
    a = (rng.standard_normal((M, K)) * 0.7).astype(np.float32)
    wf = (rng.standard_normal((N, K)) / np.sqrt(K) + 0.02).astype(np.float32)
    blocks = S.q4_1_blocks(wf)
    out = np.zeros((M, N), np.float32)
    q8 = np.zeros((M, K), np.int8); dq = np.zeros((M, K // 32), np.float32)
    assert L.owk_debug_gemm_quant(0, 3, M, N, K, a.ctypes.data_as(C.POINTER(C.c_float)), blocks,
                                  out.ctypes.data_as(C.POINTER(C.c_float)), q8.ctypes.data, dq.ctypes.data) == 0
    bl = np.frombuffer(blocks, np.uint8).reshape(N, K // 32, 20)
    d = bl[..., 0:2].copy().view("<f2")[..., 0].astype(np.float64)
    m = bl[..., 2:4].copy().view("<f2")[..., 0].astype(np.float64)
    qs = bl[..., 4:20]
    q = np.concatenate([qs & 15, qs >> 4], axis=-1).astype(np.int64)
    qa = q8.reshape(M, -1, 32).astype(np.int64)
    sa = f16((dq * qa.sum(-1).astype(np.float32)).astype(np.float32)).astype(np.float64)
    isum = np.einsum("mbk,nbk->mnb", qa, q)
    part_d = (isum * f16(dq).astype(np.float64)[:, None, :] * d[None]).sum(-1)
    part_m = (m[None] * sa[:, None, :]).sum(-1)
    err = out - (part_d + part_m)
    rel = np.abs(err) / np.abs(part_d + part_m).max()
    r, c = np.unravel_index(np.argmax(rel), rel.shape)
    print(M, N, K, "max rel", rel.max(), "at", r, c, "rows with rel>1e-6:", np.unique(np.nonzero(rel > 1e-6)[0])[:20],
          "cols:", np.unique(np.nonzero(rel > 1e-6)[1])[:20], "err/m-part", err[r, c], part_m[r, c], part_d[r, c])
    # per-block suspicion: which (row, block) s-term offsets explain the error of row r
    print("   err row r (first 8 cols):", err[r, :8])
