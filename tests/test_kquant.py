"""K-quant models (Q2_K .. Q6_K, ftype 10-14; whisper-quantize q2_k .. q6_k, ref
examples/common-ggml.cpp:12-16, block formats ref ggml/src/ggml-common.h, ggml-quants.c:703-1877).

CPU (libwhisper.so host code, no device) against the reference's own ggml functions from
oracle/_ref/libwhisper_ref.so, on blocks made by the reference quantizer (quantize_row_q*_K_ref):
  * the token-embedding row dequantization equals dequantize_row_q*_K bit for bit;
  * the virtual-block expansion the GEMMs run on (kquant.h) reproduces ggml_vec_dot_q*_K_q8_K: every
    virtual block's integer dot (exact) times its scale, summed, equals the reference's dot up to f32
    summation order, against activation rows quantized by the reference's quantize_row_q8_K_ref.
GPU: the model path (Q8_K quantizer + gemm_q16 over the virtual K) against ggml_mul_mat at decode
and encoder shapes; the Q8_K activation rows bit-exact against quantize_row_q8_K_ref.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import owk

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# kind -> (kernels.h QFmt, GGML_TYPE, block bytes per 256, virtual K per 256)
KQ = {"q2_k": (5, 10, 84, 288), "q3_k": (6, 11, 110, 256), "q4_k": (7, 12, 144, 288), "q5_k": (8, 13, 176, 288),
      "q6_k": (9, 14, 210, 512)}
Q8K_BYTES = 4 + 256 + 32  # block_q8_K: float d, int8 qs[256], int16 bsums[16]


@pytest.fixture(scope="module")
def refl():
    import ref_oracle as R

    if not R.available():
        pytest.skip("reference oracle not built")
    L = R.lib()
    L.ggml_cpu_init()  # the f16 conversion tables of ggml-base / ggml-cpu
    for k in KQ:
        n = k[:2] + "_K"
        getattr(L, f"quantize_row_{n}_ref").argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        getattr(L, f"dequantize_row_{n}").argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        getattr(L, f"ggml_vec_dot_{n}_q8_K").argtypes = [C.c_int, C.POINTER(C.c_float), C.c_size_t, C.c_void_p,
                                                          C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
    L.quantize_row_q8_K_ref.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    return L


def ref_blocks(L, kind, w):
    """rows of w (f32 [N][K]) quantized by the reference's quantize_row_q*_K_ref"""
    N, K = w.shape
    bb = KQ[kind][2]
    out = np.zeros(N * K // 256 * bb, np.uint8)
    f = getattr(L, f"quantize_row_{kind[:2]}_K_ref")
    for n in range(N):
        row = np.ascontiguousarray(w[n])
        f(row.ctypes.data, out[n * K // 256 * bb:].ctypes.data, K)
    return out


def ref_q8k(L, a):
    """quantize_row_q8_K_ref of one f32 row -> (d [K/256], qs [K], bsums [K/16], raw bytes)"""
    K = a.shape[0]
    raw = np.zeros(K // 256 * Q8K_BYTES, np.uint8)
    L.quantize_row_q8_K_ref(np.ascontiguousarray(a).ctypes.data, raw.ctypes.data, K)
    blk = raw.reshape(-1, Q8K_BYTES)
    d = blk[:, :4].copy().view(np.float32).ravel()
    qs = blk[:, 4:260].copy().view(np.int8).ravel()
    bs = blk[:, 260:].copy().view(np.int16).ravel()
    return d, qs, bs, raw


def weights(rng, N, K):
    # per-row offsets and a few large entries: non-trivial mins and sub-block scales
    w = rng.standard_normal((N, K)).astype(np.float32) / np.sqrt(K)
    w += rng.uniform(-0.05, 0.05, (N, 1)).astype(np.float32)
    w[:, ::97] *= 4
    return w.astype(np.float32)


def ours(kind, blocks, N, K, expand=True, deq=True):
    Lw = owk.load()
    Lw.owk_debug_kquant.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    kx = K // 256 * KQ[kind][3]
    wi = np.zeros((N, kx), np.uint16) if expand else None
    dwt = np.zeros((kx // 32, N), np.float32) if expand else None
    y = np.zeros((N, K), np.float32) if deq else None
    ptr = lambda x: None if x is None else x.ctypes.data
    assert Lw.owk_debug_kquant(KQ[kind][0], N, K, blocks.ctypes.data, ptr(wi), ptr(dwt), ptr(y)) == 0
    return (wi.view(np.float16).astype(np.float64) if expand else None), dwt, y


@pytest.mark.parametrize("kind", list(KQ))
def test_dequant_row_bit_exact(refl, kind):
    rng = np.random.default_rng(KQ[kind][0])
    N, K = 24, 1280
    w = weights(rng, N, K)
    blocks = ref_blocks(refl, kind, w)
    _, _, y = ours(kind, blocks, N, K, expand=False)
    ref = np.zeros((N, K), np.float32)
    rb = K // 256 * KQ[kind][2]
    f = getattr(refl, f"dequantize_row_{kind[:2]}_K")
    for n in range(N):
        f(blocks[n * rb:].ctypes.data, ref[n].ctypes.data, K)
    assert np.array_equal(y.view(np.uint32), ref.view(np.uint32)), \
        (kind, int((y != ref).sum()), float(np.abs(y - ref).max()))
    # sanity: the format reconstructs the weights to its resolution
    assert np.abs(ref - w).max() < 0.5 * np.abs(w).max()


def virtual_act(kind, qs, bs):
    """the activation side of one row in the layout of kquant.h (k_quantize_q8k_f16)"""
    nsb = qs.size // 256
    lay = {"q3_k": 1, "q6_k": 2}.get(kind, 0)
    out = []
    for sb in range(nsb):
        q = qs[sb * 256:(sb + 1) * 256].astype(np.int64)
        if lay == 0:
            out += [q, bs[sb * 16:(sb + 1) * 16].astype(np.int64), np.zeros(16, np.int64)]
        elif lay == 1:
            out.append(q)
        else:
            for j in range(16):
                out += [q[16 * j:16 * j + 16], np.zeros(16, np.int64)]
    return np.concatenate(out)


@pytest.mark.parametrize("kind", list(KQ))
def test_expansion_reproduces_vec_dot(refl, kind):
    """sum_b dot_b(virtual W row, virtual Q8_K row) * dw_b * d_a == ggml_vec_dot_q*_K_q8_K"""
    rng = np.random.default_rng(100 + KQ[kind][0])
    N, K = 16, 1536
    w = weights(rng, N, K)
    blocks = ref_blocks(refl, kind, w)
    wi, dwt, _ = ours(kind, blocks, N, K, deq=False)
    assert np.all(wi == np.round(wi)) and np.abs(wi).max() <= 2048, "virtual weights must be exact f16 integers"
    rb = K // 256 * KQ[kind][2]
    vdot = getattr(refl, f"ggml_vec_dot_{kind[:2]}_K_q8_K")
    worst = 0.0
    for trial in range(4):
        a = (rng.standard_normal(K) * (0.3 + trial)).astype(np.float32)
        d, qs, bs, raw = ref_q8k(refl, a)
        va = virtual_act(kind, qs, bs)
        per = KQ[kind][3] // 32
        da = np.repeat(d.astype(np.float64), per)
        for n in range(N):
            dots = (wi[n].astype(np.int64).reshape(-1, 32) * va.reshape(-1, 32)).sum(axis=1)
            assert np.all(np.abs(dots) < 2 ** 24), "a virtual block dot must stay exact in f32"
            terms = dots * dwt[:, n].astype(np.float64) * da
            got = float(terms.sum())
            s = C.c_float()
            vdot(K, C.byref(s), 0, blocks[n * rb:].ctypes.data, 0, raw.ctypes.data, 0, 1)
            scale = float(np.abs(terms).sum()) + 1e-30
            if abs(got - s.value) / scale > 1e-6:
                print(trial, n, got, s.value, scale, float(np.abs(terms).sum()))
            worst = max(worst, abs(got - s.value) / scale)
    print(f"[kquant] {kind}: virtual-block dot vs ggml_vec_dot max |diff| / sum|terms| = {worst:.2e}")
    assert worst < 1e-6, (kind, worst)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", list(KQ))
@pytest.mark.parametrize("M,N,K", [(1, 512, 512), (17, 1280, 1280), (32, 5120, 1280), (32, 1280, 5120),
                                   (300, 512, 2048), (2100, 1296, 1280)])
def test_kquant_gemm_vs_reference(refl, kind, M, N, K):
    """the model's K-quant linear (Q8_K rows + gemm_q16 over the virtual K) against ggml_mul_mat on
    the same blocks and f32 activations (ref_mul_mat: quantize_row_q8_K + vec_dot); the Q8_K rows
    bit-exact against quantize_row_q8_K_ref"""
    import ref_oracle as R

    L = owk.load()
    L.owk_debug_gemm_quant.argtypes = [C.c_int] * 5 + [C.POINTER(C.c_float), C.c_void_p, C.POINTER(C.c_float),
                                                       C.c_void_p, C.c_void_p]
    fmt, wtype, bb, per = KQ[kind]
    rng = np.random.default_rng(M * 7 + N + K + fmt)
    a = (rng.standard_normal((M, K)) * 0.7).astype(np.float32)
    wf = weights(rng, N, K)
    blocks = ref_blocks(refl, kind, wf)
    kx = K // 256 * per
    out = np.zeros((M, N), np.float32)
    qv = np.zeros((M, kx), np.int8)
    dv = np.zeros((M, K // 256), np.float32)
    assert L.owk_debug_gemm_quant(0, fmt, M, N, K, a.ctypes.data_as(C.POINTER(C.c_float)), blocks.ctypes.data,
                                  out.ctypes.data_as(C.POINTER(C.c_float)), qv.ctypes.data, dv.ctypes.data) == 0
    for r in range(0, M, max(1, M // 7)):
        d, qs, bs, _ = ref_q8k(refl, a[r])
        assert np.array_equal(dv[r].view(np.uint32), d.view(np.uint32)), (kind, r)
        va = virtual_act(kind, qs, bs)
        keep = np.abs(va) <= 127  # bsums saturate in the int8 copy
        assert np.array_equal(qv[r][keep].astype(np.int64), va[keep]), (kind, r)
    RL = R.lib()
    RL.ref_mul_mat.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float), C.c_int,
                               C.POINTER(C.c_float), C.c_int]
    ref = np.zeros((M, N), np.float32)
    assert RL.ref_mul_mat(wtype, blocks.ctypes.data, N, K, a.ctypes.data_as(C.POINTER(C.c_float)), M,
                          ref.ctypes.data_as(C.POINTER(C.c_float)), 8) == 0
    err = np.abs(out - ref).max() / np.abs(ref).max()
    print(f"[kquant] {kind} M={M} N={N} K={K}: max rel err vs ggml_mul_mat {err:.2e}")
    assert err < 2e-6, (kind, M, N, K, err)
