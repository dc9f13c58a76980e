"""The persistent decode chain (csrc/k_chain.hip) against the launch chain it replaces.

Passes of <= 8 rows of an F16 model run each decoder layer's residual matmuls, LayerNorms, cross-Q,
mlp.0 and the next layer's Q/K/V as two persistent launches (stage hand-offs inside the launch). Every
output is meant to be the same MFMA chain, wave order and residual / LayerNorm arithmetic as the
k_gemm_rows + k_resid_layernorm launches, so whisper_full must give bit-identical results with the
chain on (the default) and off (owk_debug_set_dec_chain(0)): token ids, probabilities (p, plog, pt,
ptsum), segment bounds, energy and DTW token timestamps. Covered: one-row greedy steps, 5-row beam
search and best-of-5 sampling (two LayerNorm row groups per stage), flash_attn = false with DTW
capture, and full-depth large-v3 (configs[4]'s model and attention mode).
"""
import ctypes as C
import json
import os
import time

import numpy as np
import pytest

import owk

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _run(w, pcm, params, mode):
    L = w.L
    L.owk_debug_set_dec_chain.argtypes = [C.c_int]
    prev = L.owk_debug_set_dec_chain(mode)
    try:
        st = w.new_state()
        t0 = time.perf_counter()
        assert w.full(st, pcm, params) == 0
        dt = time.perf_counter() - t0
        segs = w.segments(st)
        w.free_state(st)
        return segs, dt
    finally:
        L.owk_debug_set_dec_chain(prev)


def _same(w, pcm, params, what):
    _run(w, pcm, params, 1)  # warm: graphs captured, chain buffers allocated
    on, t_on = _run(w, pcm, params, 1)
    off, t_off = _run(w, pcm, params, 0)
    n = sum(len(s["tokens"]) for s in off)
    assert n > 0, what
    for i, (a, b) in enumerate(zip(on, off)):
        assert a == b, f"{what}: segment {i} differs with the persistent chain\n{a}\n{b}"
    assert len(on) == len(off), what
    print(f"[chain] {what}: {n} tokens in {len(off)} segments bit-identical; whisper_full {t_on * 1e3:.0f} ms "
          f"with the chain, {t_off * 1e3:.0f} ms without")


@pytest.mark.parametrize("model", ["tiny.en", "base.en", "tiny", "l3-mini"])
def test_chain_greedy_bit_identical(model, model_path, clips):
    owk.quiet()
    w = owk.Whisper(model_path(model))
    try:
        for clip in ("jfk", "synth30"):
            p = w.params(0, language="en", temperature_inc=0.0, token_timestamps=True)
            _same(w, clips[clip], p, f"{model}/{clip}/greedy")
    finally:
        w.close()


@pytest.mark.parametrize("model", ["tiny.en", "l3-mini"])
def test_chain_beam_and_best_of_bit_identical(model, model_path, clips):
    owk.quiet()
    w = owk.Whisper(model_path(model))
    try:
        p = w.params(1, language="en", temperature_inc=0.0, beam_size=5)
        _same(w, clips["jfk"], p, f"{model}/jfk/beam5")
        p = w.params(0, language="en", temperature=0.4, temperature_inc=0.0, best_of=5)
        _same(w, clips["jfk"], p, f"{model}/jfk/best_of5_t0.4")
    finally:
        w.close()


@pytest.mark.parametrize("model", ["tiny.en", "l3-mini"])
def test_chain_nofa_dtw_bit_identical(model, model_path, clips):
    meta = json.load(open(os.path.join(GOLDEN, "nofa_golden.json")))
    preset, n_top = meta["dtw"][model]
    owk.quiet()
    w = owk.Whisper(model_path(model), flash_attn=False, dtw_preset=preset, dtw_n_top=n_top)
    try:
        for clip in ("jfk", "synth30"):
            p = w.params(0, language="en", temperature_inc=0.0, token_timestamps=True)
            _same(w, clips[clip], p, f"{model}/{clip}/nofa+dtw")
    finally:
        w.close()


def test_chain_large_v3_nofa_dtw_bit_identical(clips):
    """configs[4]'s decoder: full-depth large-v3, flash_attn = false, DTW (LARGE_V3 heads), one row per step"""
    import owk_synth as S

    meta = json.load(open(os.path.join(GOLDEN, "large_golden.json")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    path = S.ensure_model("large-v3", meta["seed"], cache)
    owk.quiet()
    w = owk.Whisper(path, flash_attn=False, dtw_preset=meta["dtw"]["large-v3"])
    try:
        p = w.params(0, language="en", temperature_inc=0.0, token_timestamps=True)
        _same(w, clips["jfk"], p, "large-v3/jfk/nofa+dtw")
        p = w.params(1, language="en", temperature_inc=0.0, beam_size=5)
        _same(w, clips["jfk"], p, "large-v3/jfk/nofa/beam5")
    finally:
        w.close()
