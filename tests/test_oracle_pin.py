"""CPU: the numpy restatement of the reference numerics (oracle/whisper_np.py) pinned
against the golden vectors the compiled reference produced (tests/golden/), and the
host-built pieces of the drop-in library checked against it. No GPU needed."""
import json
import os

import numpy as np
import pytest

import owk
import whisper_np as O

LOGIT_RTOL = 1e-3
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def tiny(model_path):
    hp, filters, t = O.read_model(model_path("tiny.en"))
    return hp, filters, t


@pytest.mark.parametrize("model", ["tiny.en", "l3-mini"])
@pytest.mark.parametrize("clip", ["jfk", "synth30"])
def test_mel_restatement(golden, model_path, clips, model, clip):
    meta, arr = golden
    _, filters, _ = O.read_model(model_path(model))
    mel, n_len_org = O.log_mel(clips[clip], filters)
    n_mel, n_len, n_org = meta["results"][f"{model}/{clip}/mel_shape"]
    assert mel.shape == (n_mel, n_len) and n_len_org == n_org
    key = f"{model}/{clip}"
    np.testing.assert_allclose(mel[:, :400], arr[key + "/mel_head"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(mel[:, ::10], arr[key + "/mel_stride10"], atol=1e-4, rtol=0)


def test_encoder_and_decoder_restatement(golden, clips, tiny):
    meta, arr = golden
    hp, filters, t = tiny
    key = "tiny.en/jfk"
    mel, _ = O.log_mel(clips["jfk"], filters)
    enc = O.encoder(hp, t, mel)
    rows = np.concatenate([enc[:16], enc[740:756], enc[1484:]])
    err = np.abs(rows - arr[key + "/enc_rows"])
    assert err.max() < 5e-3 and err.mean() < 5e-4, (err.max(), err.mean())
    cross = O.cross_kv(hp, t, enc)
    # cross K of layer 0 (f16 bits): within one f16 ulp-scale of the reference
    ck = np.asarray(cross[0][0][:16]).reshape(-1).astype(np.float32)
    rk = arr[key + "/cross_k_l0"].view(np.float16).astype(np.float32)
    assert np.abs(ck - rk).max() < 2e-2
    dec = O.Decoder(hp, t, cross)
    prompt = meta["results"][key + "/prefill_prompt"]
    lg = dec.step(prompt, 0)
    tol = LOGIT_RTOL * np.abs(arr[key + "/prefill_top_val"]).max()
    np.testing.assert_allclose(lg[arr[key + "/prefill_top_idx"]], arr[key + "/prefill_top_val"], atol=tol, rtol=0)
    assert int(lg.argmax()) == meta["results"][key + "/prefill_stats"][2]
    lg2 = dec.step([meta["results"][key + "/step1_token"]], len(prompt))
    tol = LOGIT_RTOL * np.abs(arr[key + "/step1_top_val"]).max()
    np.testing.assert_allclose(lg2[arr[key + "/step1_top_idx"]], arr[key + "/step1_top_val"], atol=tol, rtol=0)


def test_gelu_table_matches_library():
    """The library's host-built GELU table (uploaded to HBM for the GEMM epilogues) equals
    the restatement of ggml's F16 table on every finite entry (NaN payloads may differ)."""
    L = owk.load()
    import ctypes as C

    lib = np.ctypeslib.as_array(L.owk_debug_gelu_table(), shape=(65536,)).copy()
    ref = O.gelu_table()
    x = np.arange(65536, dtype=np.uint16).view(np.float16)
    finite = np.isfinite(x) & np.isfinite(ref.view(np.float16))
    assert np.array_equal(lib[finite], ref[finite])
    del C


def test_sortformer_oracle_reproduces_golden():
    """The compiled reference SortFormer (oracle/_ref/libsortformer_ref.so) regenerates the
    committed staged-API fixtures bit for bit (pins the fixtures to the reference)."""
    import sortformer as SF
    import sortformer_synth as SS

    ref = os.path.join(ROOT, "oracle", "_ref", "libsortformer_ref.so")
    if not os.path.exists(ref):
        pytest.skip("reference SortFormer oracle not built")
    meta = json.load(open(os.path.join(GOLDEN, "sf_golden.json")))
    A = np.load(os.path.join(GOLDEN, "sf_golden.npz"))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
    if not os.path.exists(path):
        assert SS.write_model(path, meta["seed"]) == meta["sha256"]
    import owk_synth as S

    sf = SF.Sortformer(path, lib=ref, n_threads=min(8, os.cpu_count() or 1))
    x = S.read_wav_16k_mono(os.path.join(GOLDEN, "sf_test60.wav"))[:16000 * 15]
    mel, seq = sf.mel(x)
    assert np.array_equal(mel, A["stage/mel"])
    assert np.array_equal(sf.preenc(A["stage/mel"], seq), A["stage/preenc"])
    assert np.array_equal(sf.conformer(A["stage/preenc"], 0), A["stage/conf0"])
    assert np.array_equal(sf.prediction(A["stage/trans17"]), A["stage/pred"])
    sf.close()
