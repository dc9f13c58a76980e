"""GPU kernel numerics vs a plain fp32 reference of the same op (numpy on the f16 inputs).

The GEMM dispatch covers the decode-row kernel (M <= 32, incl. split-K), the skinny
kernel (M <= 64) and the 128x128 tile kernel; f32 accumulation of exact f16 products,
so the only difference to the fp32 reference is summation order."""
import ctypes as C

import numpy as np
import pytest

import owk

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 5, 16, 17, 32, 33, 64, 65, 130])
@pytest.mark.parametrize("NK", [(384, 384), (1280, 5120), (5120, 1280), (51866, 384)])
def test_gemm_dispatch(M, NK):
    N, K = NK
    if N * K > 2e7 and M > 64:
        pytest.skip("large big-tile case covered by the parity tests")
    L = owk.load()
    rng = np.random.default_rng(M * 7 + N)
    a = (rng.standard_normal((M, K)) * 0.5).astype(np.float16)
    w = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    out = np.zeros((M, N), np.float32)
    u16 = C.POINTER(C.c_uint16)
    rc = L.owk_debug_gemm(0, M, N, K, a.view(np.uint16).ctypes.data_as(u16), w.view(np.uint16).ctypes.data_as(u16),
                          out.ctypes.data_as(C.POINTER(C.c_float)))
    assert rc == 0
    ref = a.astype(np.float32) @ w.astype(np.float32).T
    assert np.isfinite(out).all()
    np.testing.assert_allclose(out, ref, atol=2e-4 * np.sqrt(K), rtol=1e-4)


def _one_chunk_np(q, k, v, scale, n_zero_pad):
    """The reference's one_chunk recurrence (ggml-cpu/ops.cpp:8140-8233) for one (row, head):
    F16 V accumulator rounded after every key; f32 scores (sum order differs from the kernels,
    hence a tolerance)."""
    M, S = -np.inf, np.float32(0)
    acc = np.zeros(64, np.float16)
    s_all = (k.astype(np.float32) @ q.astype(np.float32)) * np.float32(scale)
    for j in range(len(k) + n_zero_pad):
        s = s_all[j] if j < len(k) else np.float32(0)
        vj = v[j].astype(np.float32) if j < len(k) else np.zeros(64, np.float32)
        ms, vs = np.float32(1), np.float32(1)
        if s > M:
            ms = np.float32(np.exp(np.float32(M - s))) if M > -np.inf else np.float32(0)
            M = s
            acc = (acc.astype(np.float32) * ms).astype(np.float16)
        else:
            vs = np.float32(np.exp(np.float32(s - M)))
        acc = (vj * vs + acc.astype(np.float32)).astype(np.float16)
        S = np.float32(S * ms + vs)
    return acc.astype(np.float32) / S if S != 0 else np.zeros(64, np.float32)


XSHAPES = [(3, 2, 1, 0), (3, 2, 63, 0), (2, 2, 64, 36), (2, 3, 65, 0), (4, 2, 200, 0), (2, 2, 257, 5), (2, 2, 768, 0),
           (32, 20, 1500, 0), (2, 2, 0, 0)]


def _cross_outputs(R, H, T, pad, which):
    L = owk.load()
    L.owk_debug_attn_cross.restype = C.c_double
    u16 = C.POINTER(C.c_uint16)
    L.owk_debug_attn_cross.argtypes = [C.c_int] * 6 + [C.c_float, u16, u16, u16, u16, C.c_int]
    rng = np.random.default_rng(T * 31 + R)
    q = rng.standard_normal((R, H * 64)).astype(np.float16)
    # keys with a slowly rising trend: new running maxima keep appearing deep into the sequence
    trend = np.linspace(0, 3, max(T, 1))[:T, None]
    k = (rng.standard_normal((R, H, T, 64)) * 0.7 + trend * 0.05).astype(np.float16)
    v = rng.standard_normal((R, H, T, 64)).astype(np.float16)
    scale = 64 ** -0.25
    outs = {}
    for w in which:
        o = np.zeros((R, H * 64), np.float16)
        rc = L.owk_debug_attn_cross(0, w, R, H, T, pad, scale, q.view(np.uint16).ctypes.data_as(u16),
                                    k.view(np.uint16).ctypes.data_as(u16), v.view(np.uint16).ctypes.data_as(u16),
                                    o.view(np.uint16).ctypes.data_as(u16), 0)
        assert rc == 0
        outs[w] = o.astype(np.float32)
    return q, k, v, scale, outs


@pytest.mark.parametrize("R,H,T,pad", XSHAPES)
def test_attn_cross_one_wave(R, H, T, pad):
    """k_attn_step (the cross-attention kernel: one wave per row and head, and the production form with a
    loader wave beside the math wave) against the numpy restatement of the reference's one_chunk
    recurrence; the two forms bit-identical"""
    q, k, v, scale, outs = _cross_outputs(R, H, T, pad, (1, 2))
    assert np.isfinite(outs[1]).all()
    assert np.array_equal(outs[1].view(np.uint32), outs[2].view(np.uint32))
    for r in range(min(R, 2)):
        for h in range(min(H, 2)):
            ref = _one_chunk_np(q[r, h * 64:(h + 1) * 64], k[r, h], v[r, h], scale, pad)
            np.testing.assert_allclose(outs[1][r, h * 64:(h + 1) * 64], ref, atol=2e-3, rtol=2e-2)


def test_attn_cross_speed():
    """Device time of the cross-attention kernel on the large-v3 decode shape (32 rows x 20 heads x
    1500 keys), printed for the record."""
    L = owk.load()
    L.owk_debug_attn_cross.restype = C.c_double
    u16 = C.POINTER(C.c_uint16)
    L.owk_debug_attn_cross.argtypes = [C.c_int] * 6 + [C.c_float, u16, u16, u16, u16, C.c_int]
    for w, name in ((1, "k_attn_step one wave"), (2, "k_attn_step loader + math waves")):
        for R in (32, 1):
            t = min(L.owk_debug_attn_cross(0, w, R, 20, 1500, 0, 0.35, None, None, None, None, 30) for _ in range(3))
            print(f"attn_cross {name} R={R}: {t:.1f} us ({R * 20 * 1500 * 64 * 2 * 2 / t / 1e3:.0f} GB/s)")
            assert t > 0


# kernels.h EPI_* codes and (N, d, T) per mode for the large-tile epilogue cross-check
_EPI_CASES = {
    "f16": (0, 1280, 0, 0), "gelu": (1, 5120, 0, 0), "resid": (2, 1280, 0, 0), "conv2": (3, 1280, 1280, 1500),
    "qkv_enc": (4, 3840, 1280, 1500), "kv_cross": (5, 2560, 1280, 1500), "f32": (7, 1024, 0, 0),
    "bias_f32": (9, 1024, 0, 0), "silu": (10, 1024, 0, 0), "half_resid": (11, 1024, 0, 0), "relu": (12, 1024, 0, 0),
    "sigmoid": (13, 1024, 0, 0), "f16_ragged": (0, 1288, 0, 0),
}


@pytest.mark.parametrize("kern", [0x800], ids=["8phase"])
@pytest.mark.parametrize("case", sorted(_EPI_CASES))
def test_gemm256_epilogue_matches_128(case, kern):
    """The 256x256 ring kernel computes C^T tiles and writes 8-column runs with 16-byte vector
    epilogues (k_gemm.hip epi_row8); the 128x128 kernel writes every element with epi_store.
    Same operands, bias, residual, positions and GELU table: every output must agree."""
    mode, N, d, T = _EPI_CASES[case]
    L = owk.load()
    L.owk_debug_gemm_epi_diff.restype = C.c_double
    L.owk_debug_gemm_epi_diff.argtypes = [C.c_int] * 7
    M = 3000 if T else 2304
    diff = L.owk_debug_gemm_epi_diff(0, mode | kern, M, N, 1280, d, T)
    print(f"{case} {kern:#x}: max|256 - 128| = {diff:.3g}")
    assert diff >= 0
    assert diff <= 1e-6, f"{case}: epilogues differ by {diff}"


@pytest.mark.parametrize("kern", [0x1000, 0x2000], ids=["mid64", "mid32"])
@pytest.mark.parametrize("case", sorted(_EPI_CASES))
def test_gemm_mid_matches_128(case, kern):
    """The 64x64 ring tile (k_gemm_mid: mid-size GEMMs, e.g. SortFormer chunk passes) runs the same
    MFMA sequence per output as the 128x128 tile: every epilogue output must be bit-identical.
    Ragged M (not a multiple of 64) and N (f16_ragged) exercise the edge tiles."""
    mode, N, d, T = _EPI_CASES[case]
    L = owk.load()
    L.owk_debug_gemm_epi_diff.restype = C.c_double
    L.owk_debug_gemm_epi_diff.argtypes = [C.c_int] * 7
    M = 1500 if T else 413
    diff = L.owk_debug_gemm_epi_diff(0, mode | kern, M, N, 512, d, T)
    print(f"{case} {kern:#x}: max|mid - 128| = {diff:.3g}")
    assert diff == 0, f"{case}: epilogues differ by {diff}"


def test_gemm_mid_speed():
    """Device time of the SortFormer chunk-pass GEMM shapes (M = 413 rows) through the 64x64 ring
    tile and the 128x128 tile, printed for the record; the ring tile must not be slower."""
    L = owk.load()
    L.owk_debug_gemm_bench.restype = C.c_double
    L.owk_debug_gemm_bench.argtypes = [C.c_int] * 6
    worse = []
    for mode, N, K in ((9, 1536, 512), (10, 2048, 512), (11, 512, 2048), (2, 512, 512), (9, 192, 512),
                       (12, 768, 192), (2, 192, 768)):
        t_mid = min(L.owk_debug_gemm_bench(0, mode | 0x1000 | 0x200, 413, N, K, 50) for _ in range(3))
        t_32 = min(L.owk_debug_gemm_bench(0, mode | 0x2000 | 0x200, 413, N, K, 50) for _ in range(3))
        t_big = min(L.owk_debug_gemm_bench(0, mode | 0x100 | 0x200, 413, N, K, 50) for _ in range(3))
        print(f"M=413 N={N} K={K} mode {mode}: 64x64 ring {t_mid:.2f} us, 32x32 ring {t_32:.2f} us, "
              f"128x128 {t_big:.2f} us")
        assert t_mid > 0 and t_32 > 0 and t_big > 0
        t_mid = min(t_mid, t_32)
        if t_mid > 1.1 * t_big:
            worse.append((N, K))
    assert not worse, worse


@pytest.mark.parametrize("M,N,K", [(1, 1280, 1280), (7, 3840, 1280), (16, 5120, 1280), (32, 1280, 1280),
                                   (32, 3840, 1280), (32, 5120, 1280), (5, 1536, 384), (32, 2048, 512)])
def test_gemm_rows_ln_matches_two_launch_form(M, N, K):
    """The decoder's LayerNorm-prologue GEMM (k_gemm_rows_ln: the waves of a block hold the row's k ranges,
    statistics combined in LDS) equals layernorm_f16 + the decode-row GEMM on the same rows: the
    LayerNorm statistics are the same double sums in another association, so the f16 rows (and the
    outputs) agree except where a sum lands on an f32 rounding boundary -- rare, at most 1 f16 ulp.
    With N <= 1280, also the whole-K residual epilogue (EPI_RESID_F32, the mlp.2 shape K = 4 N, J = 10)
    against split-K partials + resid_layernorm: f32 re-association only."""
    L = owk.load()
    f = L.owk_debug_gemm_rows_ln
    fp = C.POINTER(C.c_float)
    u16 = C.POINTER(C.c_uint16)
    f.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, fp, fp, fp, fp, u16, u16, u16, u16, fp, fp, fp]
    rng = np.random.default_rng(M * 1000 + N + K)
    x = (rng.standard_normal((M, K)) * 2 + 0.3).astype(np.float32)
    lnw = (1 + 0.1 * rng.standard_normal(K)).astype(np.float32)
    lnb = (0.05 * rng.standard_normal(K)).astype(np.float32)
    b = (0.02 * rng.standard_normal(N)).astype(np.float32)
    w = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    o1 = np.zeros((M, N), np.uint16)
    o2 = np.zeros((M, N), np.uint16)
    res_case = N <= 1280
    w2 = (rng.standard_normal((N, 4 * N)) / np.sqrt(4 * N)).astype(np.float16) if res_case else None
    resid = rng.standard_normal((M, N)).astype(np.float32) if res_case else None
    r1 = np.zeros((M, N), np.float32)
    r2 = np.zeros((M, N), np.float32)
    P = lambda a, t: a.ctypes.data_as(t) if a is not None else None  # noqa: E731
    assert f(0, M, N, K, P(x, fp), P(lnw, fp), P(lnb, fp), P(b, fp), P(w.view(np.uint16), u16), P(o1, u16), P(o2, u16),
             P(w2.view(np.uint16) if res_case else None, u16), P(resid, fp), P(r1, fp) if res_case else None,
             P(r2, fp) if res_case else None) == 0
    a, r = o1.view(np.float16).astype(np.float32), o2.view(np.float16).astype(np.float32)
    n_eq = int((o1 == o2).sum())
    ulp = np.abs(r) * 2.0 ** -10 + 2.0 ** -24
    print(f"M={M} N={N} K={K}: {n_eq}/{o1.size} outputs bit-identical, max|diff| {np.abs(a - r).max():.3g}")
    assert np.isfinite(a).all()
    assert np.all(np.abs(a - r) <= 2 * ulp)
    assert n_eq >= 0.999 * o1.size
    if res_case:
        d = np.abs(r1 - r2)
        print(f"  residual epilogue over the whole K vs split-K: max|diff| {d.max():.3g} "
              f"({int((r1 == r2).sum())}/{r1.size} identical)")
        assert d.max() <= 1e-4 * max(1.0, float(np.abs(r2).max()))


@pytest.mark.parametrize("model", ["tiny.en", "base.en", "tiny", "l3-mini"])
def test_whole_k_chain_bit_identical(model, model_path, clips):
    """The decoder's whole-K chain (gemm_rows_res + gemm_rows_lnx: one launch per residual matmul, the
    LayerNorm in the next matmul's prologue; off by default since it measured slower, enabled here
    through the test hook) reproduces the split-K + resid_layernorm
    chain bit for bit: a clip's logits and tokens must not depend on how many rows share its decode pass.
    Staged decode (prompt + teacher-forced steps) and whisper_full, with the chain forced each way."""
    import ctypes as C

    L = owk.load()
    owk.quiet()
    L.owk_debug_set_whole_k_rows.argtypes = [C.c_int]
    w = owk.Whisper(model_path(model))
    pcm = np.ascontiguousarray(clips["jfk"], np.float32)

    def run(limit):
        prev = L.owk_debug_set_whole_k_rows(limit)
        try:
            st = w.new_state()
            assert L.whisper_pcm_to_mel_with_state(w.ctx, st, owk.fptr(pcm), len(pcm), 1) == 0
            assert L.whisper_encode_with_state(w.ctx, st, 0, 1) == 0
            sot = L.whisper_token_sot(w.ctx)
            prompt = [sot] if w.n_vocab < 51865 else [sot, sot + 1, L.whisper_token_transcribe(w.ctx)]
            out = []
            toks = (C.c_int32 * len(prompt))(*prompt)
            assert L.whisper_decode_with_state(w.ctx, st, toks, len(prompt), 0, 1) == 0
            out.append(np.ctypeslib.as_array(L.whisper_get_logits_from_state(st), shape=(len(prompt) * w.n_vocab,))
                       [-w.n_vocab:].copy())
            n_past = len(prompt)
            for t in (440, 1029, 257, 11, 318):
                one = (C.c_int32 * 1)(t)
                assert L.whisper_decode_with_state(w.ctx, st, one, 1, n_past, 1) == 0
                out.append(np.ctypeslib.as_array(L.whisper_get_logits_from_state(st), shape=(w.n_vocab,)).copy())
                n_past += 1
            w.free_state(st)
            st = w.new_state()
            assert w.full(st, pcm, w.params(0, language="en", temperature_inc=0.0)) == 0
            segs = w.segments(st)
            w.free_state(st)
            return out, segs
        finally:
            L.owk_debug_set_whole_k_rows(prev)

    lg_split, seg_split = run(0)
    lg_whole, seg_whole = run(16)
    for i, (a, b) in enumerate(zip(lg_split, lg_whole)):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), \
            f"{model}: decode call {i}: logits differ (max {np.abs(a - b).max():.3g})"
    assert seg_split == seg_whole, f"{model}: whisper_full results differ between the chains"
    print(f"{model}: {len(lg_split)} decode calls and {sum(len(s['tokens']) for s in seg_split)} whisper_full tokens "
          f"bit-identical")



@pytest.mark.parametrize("R,T", [(1, 1500), (3, 1500), (2, 100), (1, 128), (1, 129), (5, 384), (32, 1500), (7, 2048),
                                 (1, 60), (1, 200)])
def test_softmax_attention_split_bit_identical(R, T):
    """The key-split soft_max attention (k_sm_split_scores + k_sm_split_pv: scores per 128-key chunk,
    P.V per block of 16 residue groups, in-launch combine by the last-arriving block) reproduces the
    single-block k_attn_softmax bit for bit -- outputs and DTW probability captures -- so the flash_attn =
    false results (and the DTW timestamps) do not depend on which form ran. Random q/K/V, 20 heads."""
    L = owk.load()
    f = L.owk_debug_attn_softmax
    f.restype = C.c_double
    f.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint16), C.POINTER(C.c_float), C.c_int]
    H = 20
    outs, caps = [], []
    # the split form twice (its arrival tickets must be reset between launches), then the single-block
    # kernel at both widths (outputs do not depend on the width)
    for split in (0, 1, 1, 256, 512, 1024):
        o = np.zeros(R * H * 64, np.uint16)
        cp = np.zeros(4 * T * R, np.float32)
        assert f(0, split, R, H, T, o.ctypes.data_as(C.POINTER(C.c_uint16)), cp.ctypes.data_as(C.POINTER(C.c_float)), 3) >= 0
        outs.append(o)
        caps.append(cp)
    assert np.abs(outs[0].view(np.float16).astype(np.float32)).max() > 0
    for i in (1, 2, 3, 4, 5):
        bad = np.nonzero(outs[0] != outs[i])[0]
        a16, b16 = outs[0].view(np.float16), outs[i].view(np.float16)
        assert bad.size == 0, (f"R={R} T={T}: split outputs differ ({bad.size} values): " +
                               ", ".join(f"[r{k // (H * 64)} h{k // 64 % H} d{k % 64}] {a16[k]} vs {b16[k]}" for k in bad[:8]))
        assert np.array_equal(caps[0].view(np.uint32), caps[i].view(np.uint32)), f"R={R} T={T}: captures differ"
    us = [f(0, s, R, H, T, None, None, 20) for s in (0, 1, 256, 1024)]
    print(f"R={R} T={T}: bit-identical; single-block {us[0]:.1f} us (256 threads {us[2]:.1f}, 1024 threads {us[3]:.1f}), "
          f"key-split {us[1]:.1f} us")
