"""Quantized streaming-SortFormer GGUFs: the files the reference's own
sortformer-quantize writes (streaming-sortformer/tools/quantize.cpp, built from its sources into
oracle/_ref/ by oracle/ref/Makefile -- test infrastructure) for q8_0, q4_k and q5_k, run by
libsortformer.so against tests/golden/sfq_golden.* (make_golden_sfq.py: the reference's CPU path on
the same files).

The reference rounds every f32 mul_mat activation row to the weight's vec_dot_type (Q8_0 per 32,
Q8_K per 256) before the integer block dots; libsortformer.so does the same from f32 producer
outputs (sortformer.cpp sf_lin). Q8 rounding turns f32 re-association differences into whole
quantization steps, so the deep stacks and end-to-end outputs are held to 2x the reference's own
noise floor (the same run on input perturbed by 1e-7 relative noise, recorded per case) as the F16
tests are; the single layer-0 conformer, whose activations are rounded a handful of times, to an
absolute 2e-3 (the F16 stage bar).

CPU: the quantizer output is the pinned file (SHA-256); init fails loudly without a GPU.
GPU: stage, diarization, RTTM speaker activity (frame by frame against the reference's threshold
noise band, as tests/test_gpu_c4.py) and 2 s streaming parity.
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(ROOT, "open-whisper-kit_amd", "lib", "libsortformer.so")
QUANT = os.path.join(ROOT, "oracle", "_ref", "sortformer-quantize")
KINDS = ("q8_0", "q4_k", "q5_k")


@pytest.fixture(scope="module")
def sfq():
    meta = json.load(open(os.path.join(GOLDEN, "sfq_golden.json")))
    arrays = np.load(os.path.join(GOLDEN, "sfq_golden.npz"))
    f16 = np.load(os.path.join(GOLDEN, "sf_golden.npz"))
    return meta, arrays, f16


def model_path(meta, kind):
    """the reference quantizer's file for `kind` (regenerated from the pinned F16 GGUF)"""
    import owk_synth as S
    import sortformer_synth as SS

    if not os.path.exists(QUANT):
        pytest.skip("reference quantizer not built (make -C oracle/ref)")
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    dst = os.path.join(cache, f"synth-sortformer-s{meta['seed']}-{kind}.gguf")
    want = meta["models"][kind]["sha256"]
    if os.path.exists(dst) and S.file_sha256(dst) == want:
        return dst
    src = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
    SS.write_model(src, meta["seed"])
    subprocess.run([QUANT, src, dst, kind], check=True, capture_output=True)
    assert S.file_sha256(dst) == want, f"{kind}: quantized GGUF differs from the fixture's"
    return dst


@pytest.mark.parametrize("kind", KINDS)
def test_quantized_gguf_pinned(sfq, kind):
    meta, _, _ = sfq
    assert os.path.getsize(model_path(meta, kind)) > 0


def test_fails_loudly_without_gpu(sfq):
    """no CPU fallback for quantized models either: without a GPU sortformer_init returns NULL"""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import sortformer as SF

    meta, _, _ = sfq
    with pytest.raises(RuntimeError):
        SF.Sortformer(model_path(meta, "q4_k"), lib=LIB)


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module", params=KINDS)
def qsf(request, sfq):
    import sortformer as SF

    meta, _, _ = sfq
    s = SF.Sortformer(model_path(meta, request.param), lib=LIB)
    s.kind = request.param
    yield s
    s.close()


def within_floor(meta, key, got, want):
    fl = meta["results"]["noise_floor/" + key]
    got = np.asarray(got, np.float64)
    assert got.shape == want.shape, (got.shape, want.shape)
    d = np.abs(got - want)
    print(f"[sfq] {key}: max|diff| {d.max():.3e} mean {d.mean():.3e} (floor {fl['max']:.3e} / {fl['mean']:.3e})")
    assert d.max() <= 2 * fl["max"] + 1e-4, f"{key}: max|diff| {d.max():.3e} vs floor {fl['max']:.3e}"
    assert d.mean() <= 2 * fl["mean"] + 1e-5, f"{key}: mean|diff| {d.mean():.3e} vs floor {fl['mean']:.3e}"


@pytest.mark.gpu
def test_conformer_layer0(qsf, sfq):
    meta, A, F = sfq
    got = qsf.conformer(F["stage/preenc"], 0)
    d = np.abs(got.astype(np.float64) - A[f"{qsf.kind}/conf0"]).max()
    print(f"[sfq] {qsf.kind}/conf0: max|diff| {d:.3e}")
    assert d <= 2e-3


@pytest.mark.gpu
def test_conformer_stack(qsf, sfq):
    meta, A, F = sfq
    within_floor(meta, f"{qsf.kind}/conf16", qsf.conformer(F["stage/preenc"], 16), A[f"{qsf.kind}/conf16"])


@pytest.mark.gpu
def test_transformer_stack(qsf, sfq):
    meta, A, F = sfq
    within_floor(meta, f"{qsf.kind}/trans17", qsf.transformer(F["stage/proj"], 17), A[f"{qsf.kind}/trans17"])


@pytest.mark.gpu
def test_diarize(qsf, sfq):
    import owk_synth as S
    import sortformer as SF

    from parity_util import rttm_activity_diff

    meta, A, _ = sfq
    x = S.read_wav_16k_mono(os.path.join(GOLDEN, "sf_test60.wav"))
    key = f"{qsf.kind}/diarize/test60"
    p = qsf.diarize(x)
    within_floor(meta, key, p, A[key])
    # RTTM: with quantized weights the probabilities move by whole Q8 steps (the floor above), so
    # threshold crossings are compared frame by frame against the reference's threshold noise band
    rttm = SF.to_rttm(p, 0.5, 11, "/x/test60.wav", lib=LIB)
    n_diff, bad = rttm_activity_diff(rttm, meta["results"][f"rttm/{qsf.kind}/test60"], A[key],
                                     meta["results"]["noise_floor/" + key]["max"])
    print(f"[sfq] {qsf.kind} RTTM: {n_diff} of {A[key].size} speaker-frames differ, {int(bad.sum())} outside the "
          f"reference's threshold noise band")
    assert not bad.any(), np.argwhere(bad)[:10]


@pytest.mark.gpu
def test_stream_2s(qsf, sfq):
    import owk_synth as S

    meta, A, _ = sfq
    x = S.read_wav_16k_mono(os.path.join(GOLDEN, "sf_test60.wav"))
    st = qsf.stream("2s")
    outs, pos = [], 0
    while pos < len(x):
        outs.append(st.feed(x[pos:pos + 8000]))
        pos += 8000
    outs.append(st.flush())
    st.close()
    within_floor(meta, f"{qsf.kind}/stream/2s_blocks8000", np.concatenate(outs, 0), A[f"{qsf.kind}/stream/2s_blocks8000"])
