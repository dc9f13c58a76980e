"""Streaming-SortFormer parity: the MI355X libsortformer.so against the reference's golden
vectors (tests/golden/make_golden_sf.py ran the reference streaming-sortformer + ggml CPU
path on synthetic GGUF weights).

CPU tests: ABI exports of include/sortformer.h, the host-only entry points (RTTM, WAV
loading, presets), the deterministic GGUF writer, and that the library fails loudly
without a GPU. GPU tests: every stage of the staged API from the golden input of that
stage, whole-clip diarization (default and FIFO configs), RTTM text, and the streaming
API (feed/flush frame counts exact, probabilities within the reference's noise floor).

Tolerances. Stages: max|diff| <= 1e-3 (mel / pre-encoder / projection / head) or 2e-3
(the 17-layer conformer and 18-layer transformer stacks; measured 3-4e-4). End to end, the
synthetic deep stack amplifies ulp-level f32 differences through 35 layers and the
speaker-cache feedback: the reference itself moves by the recorded noise floor when its
input is perturbed by 1e-7 relative noise (sf_golden.json "noise_floor/*"); the GPU result
must stay within 2x that floor (max and mean).
"""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(ROOT, "open-whisper-kit_amd", "lib", "libsortformer.so")
STREAMS = {
    "2s_blocks8000": ("2s", [8000]),
    "low_ragged": ("low", [3200, 7000, 160, 12345, 999]),
    "5s_blocks16000": ("5s", [16000]),
}


@pytest.fixture(scope="module")
def sfg():
    meta = json.load(open(os.path.join(GOLDEN, "sf_golden.json")))
    arrays = np.load(os.path.join(GOLDEN, "sf_golden.npz"))
    return meta, arrays


@pytest.fixture(scope="module")
def test60():
    import owk_synth as S

    return S.read_wav_16k_mono(os.path.join(GOLDEN, "sf_test60.wav"))


@pytest.fixture(scope="module")
def sf_model(sfg):
    import sortformer_synth as SS

    meta, _ = sfg
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
    sha_file = path + ".sha256"
    if not (os.path.exists(path) and os.path.exists(sha_file) and open(sha_file).read().strip() == meta["sha256"]):
        sha = SS.write_model(path, meta["seed"])
        assert sha == meta["sha256"], "synthetic SortFormer GGUF differs from the fixture's"
        with open(sha_file, "w") as f:
            f.write(sha)
    return path


def header_functions():
    txt = open(os.path.join(ROOT, "include", "sortformer.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sortformer_\w+)\s*\(", txt)))


# ------------------------------------------------------------------ CPU
def test_exports_every_header_symbol():
    lib = C.CDLL(LIB)
    names = header_functions()
    assert len(names) == 19
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_header_matches_reference_layout():
    import sortformer as SF

    assert C.sizeof(SF.Params) == 9 * 4 and C.sizeof(SF.StreamParams) == 6 * 4
    L = SF.load(LIB)
    p = L.sortformer_default_params()
    assert (p.chunk_len, p.right_context, p.fifo_len, p.spkcache_len, p.spkcache_update_period, p.median_filter,
            p.n_threads, p.chunk_left_context) == (188, 1, 0, 188, 188, 11, 4, 1)
    assert abs(p.threshold - 0.5) < 1e-9
    want = {0: (6, 7, 1, 188, 188, 144), 1: (15, 10, 1, 100, 188, 144), 2: (30, 7, 1, 100, 188, 100),
            3: (55, 7, 1, 100, 188, 100)}
    for k, v in want.items():
        sp = L.sortformer_stream_preset_params(k)
        assert (sp.chunk_len, sp.right_context, sp.left_context, sp.fifo_len, sp.spkcache_len,
                sp.spkcache_update_period) == v


def test_rttm_matches_reference(sfg):
    import sortformer as SF

    meta, A = sfg
    for name in ("test60", "synth45"):
        got = SF.to_rttm(A[f"diarize/{name}"], 0.5, 11, f"/x/{name}.wav", lib=LIB)
        assert got == meta["results"][f"rttm/{name}"]
    # buffer too small -> -1 (ref sortformer.cpp:2659-2661); no frames -> -1
    assert SF.to_rttm(A["diarize/test60"], 0.5, 11, "a.wav", lib=LIB, buf_size=16) is None
    assert SF.to_rttm(np.zeros((0, 4), np.float32), lib=LIB) is None


def test_load_wav(test60):
    import sortformer as SF

    L = SF.load(LIB)
    p = C.POINTER(C.c_float)()
    n = L.sortformer_load_wav(os.path.join(GOLDEN, "sf_test60.wav").encode(), C.byref(p))
    assert n == len(test60)
    got = np.ctypeslib.as_array(p, shape=(n,)).copy()
    SF._libc.free(C.cast(p, C.c_void_p))
    assert np.array_equal(got, test60)
    assert L.sortformer_load_wav(os.path.join(GOLDEN, "golden.json").encode(), C.byref(p)) == -1


def test_gguf_writer_deterministic(sfg, sf_model):
    import hashlib

    meta, _ = sfg
    h = hashlib.sha256(open(sf_model, "rb").read()).hexdigest()
    assert h == meta["sha256"]


def test_fails_loudly_without_gpu(sf_model):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import sortformer as SF

    with pytest.raises(RuntimeError):
        SF.Sortformer(sf_model, lib=LIB)


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def sf(sf_model):
    import sortformer as SF

    s = SF.Sortformer(sf_model, lib=LIB)
    yield s
    s.close()


def close(got, want, tol):
    got = np.asarray(got, np.float64)
    assert got.shape == want.shape
    d = np.abs(got - want).max()
    assert d <= tol, f"max|diff| {d:.3e} > {tol:.1e}"


@pytest.mark.gpu
def test_stage_mel(sf, sfg, test60):
    meta, A = sfg
    mel, seq = sf.mel(test60[:16000 * 15])
    assert seq == meta["results"]["stage/seq_len"]
    close(mel, A["stage/mel"], 1e-3)


@pytest.mark.gpu
def test_stage_preenc(sf, sfg):
    meta, A = sfg
    close(sf.preenc(A["stage/mel"], meta["results"]["stage/seq_len"]), A["stage/preenc"], 1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("layer", [0, 16])
def test_stage_conformer(sf, sfg, layer):
    _, A = sfg
    close(sf.conformer(A["stage/preenc"], layer), A[f"stage/conf{layer}"], 2e-3)


@pytest.mark.gpu
def test_stage_projection(sf, sfg):
    _, A = sfg
    close(sf.projection(A["stage/conf16"]), A["stage/proj"], 1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("layer", [0, 17])
def test_stage_transformer(sf, sfg, layer):
    _, A = sfg
    close(sf.transformer(A["stage/proj"], layer), A[f"stage/trans{layer}"], 2e-3)


@pytest.mark.gpu
def test_stage_prediction(sf, sfg):
    _, A = sfg
    close(sf.prediction(A["stage/trans17"]), A["stage/pred"], 1e-3)


def within_floor(meta, key, got, want):
    fl = meta["results"]["noise_floor/" + key]
    got = np.asarray(got, np.float64)
    assert got.shape == want.shape, (got.shape, want.shape)
    d = np.abs(got - want)
    assert d.max() <= 2 * fl["max"] + 1e-4, f"{key}: max|diff| {d.max():.3e} vs floor {fl['max']:.3e}"
    assert d.mean() <= 2 * fl["mean"] + 1e-5, f"{key}: mean|diff| {d.mean():.3e} vs floor {fl['mean']:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["test60", "synth45"])
def test_diarize(sf, sfg, test60, name):
    import owk_synth as S
    import sortformer as SF

    meta, A = sfg
    x = test60 if name == "test60" else S.synth_audio(16000 * 45, 11)
    p = sf.diarize(x)
    within_floor(meta, f"diarize/{name}", p, A[f"diarize/{name}"])
    assert SF.to_rttm(p, 0.5, 11, f"/x/{name}.wav", lib=LIB) == meta["results"][f"rttm/{name}"]


@pytest.mark.gpu
def test_diarize_fifo_config(sf_model, sfg, test60):
    import sortformer as SF

    meta, A = sfg
    s = SF.Sortformer(sf_model, lib=LIB, chunk_len=48, fifo_len=40, spkcache_update_period=64, right_context=2,
                      chunk_left_context=2)
    within_floor(meta, "diarize_fifo/test60", s.diarize(test60), A["diarize_fifo/test60"])
    s.close()


@pytest.mark.gpu
def test_diarize_errors(sf):
    L = sf.L
    out = np.zeros((4, 4), np.float32)
    fp = out.ctypes.data_as(C.POINTER(C.c_float))
    assert L.sortformer_diarize(sf.ctx, fp, 0, fp, 4) == -1
    assert L.sortformer_diarize(None, fp, 10, fp, 4) == -1
    # n_frames_max caps the output
    x = np.zeros(16000 * 20, np.float32)
    n = L.sortformer_diarize(sf.ctx, x.ctypes.data_as(C.POINTER(C.c_float)), len(x), fp, 4)
    assert n == 4


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(STREAMS))
def test_stream(sf, sfg, test60, name):
    meta, A = sfg
    preset, blocks = STREAMS[name]
    st = sf.stream(preset)
    outs, counts, pos, i = [], [], 0, 0
    while pos < len(test60):
        n = min(blocks[i % len(blocks)], len(test60) - pos)
        o = st.feed(test60[pos:pos + n])
        outs.append(o)
        counts.append(o.shape[0])
        pos += n
        i += 1
    fl = st.flush()
    outs.append(fl)
    counts.append(fl.shape[0])
    assert counts == meta["results"][f"stream_counts/{name}"]
    within_floor(meta, f"stream/{name}", np.concatenate(outs), A[f"stream/{name}"])
    # reset -> the same feeds reproduce the first run bit for bit (deterministic kernels)
    st.reset()
    pos = 0
    for i in range(6):
        n = blocks[i % len(blocks)]
        assert np.array_equal(st.feed(test60[pos:pos + n]), outs[i])
        pos += n
    st.close()


@pytest.mark.gpu
def test_stream_feed_batch(sf, sfg, test60):
    """owk_sortformer_stream_feed_batch: the three golden stream
    configurations plus ragged copies fed as ONE batch per round of blocks. Every stream
    reproduces the reference's golden outputs within the noise floor, its per-feed frame
    counts exactly, and the same stream fed alone within the same noise floor (the stacked
    GEMMs sum in another order than a lone stream's split-K ones; AOSC amplifies it)."""
    import sortformer as SF

    meta, A = sfg
    names = list(STREAMS) + list(STREAMS)
    streams = [sf.stream(STREAMS[nm][0]) for nm in names]
    solo = [sf.stream(STREAMS[nm][0]) for nm in names]
    pos = [0] * len(names)
    outs = [[] for _ in names]
    counts = [[] for _ in names]
    solo_outs = [[] for _ in names]
    i = 0
    while any(p < len(test60) for p in pos):
        act, pcms = [], []
        for k, nm in enumerate(names):
            blocks = STREAMS[nm][1]
            if pos[k] >= len(test60):
                continue
            b = blocks[i % len(blocks)] if k < len(STREAMS) else blocks[(i + 1) % len(blocks)]
            n = min(b, len(test60) - pos[k])
            act.append(k)
            pcms.append(test60[pos[k]:pos[k] + n])
            pos[k] += n
        for k, o in zip(act, SF.feed_batch([streams[k] for k in act], pcms)):
            outs[k].append(o)
            counts[k].append(o.shape[0])
        for k, pcm in zip(act, pcms):
            solo_outs[k].append(solo[k].feed(pcm))
        i += 1
    for k, nm in enumerate(names):
        fl = streams[k].flush()
        outs[k].append(fl)
        counts[k].append(fl.shape[0])
        solo_outs[k].append(solo[k].flush())
        got = np.concatenate(outs[k])
        within_floor(meta, f"stream/{nm}", got, np.concatenate(solo_outs[k]))
        if k < len(STREAMS):
            assert counts[k] == meta["results"][f"stream_counts/{nm}"]
            within_floor(meta, f"stream/{nm}", got, A[f"stream/{nm}"])
    for st in streams + solo:
        st.close()

