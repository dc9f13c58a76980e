"""CPU: synthetic-weight generator and golden-fixture integrity."""
import hashlib
import os

import numpy as np

import owk_synth as S


def test_slaney_filters_match_reference_80_bin_filterbank():
    ref = np.load(os.path.join(S.ASSETS, "mel_filters_80.npy"))
    ours = S.slaney_mel_filters(80)
    assert ours.shape == ref.shape == (80, 201)
    assert np.abs(ours - ref).max() < 1e-7


def test_model_bytes_reproducible(golden, tmp_path):
    meta, _ = golden
    p = tmp_path / "m.bin"
    assert S.write_model(str(p), "tiny.en", meta["seed"]) == meta["models"]["tiny.en"]["sha256"]
    h = hashlib.sha256(p.read_bytes()).hexdigest()
    assert h == meta["models"]["tiny.en"]["sha256"]


def test_golden_covers_every_config(golden):
    meta, arr = golden
    for model in ("tiny.en", "base.en", "tiny", "l3-mini"):
        for clip in ("jfk", "synth30"):
            assert f"{model}/{clip}/full/greedy" in meta["results"]
            assert f"{model}/{clip}/full/beam5" in meta["results"]
            assert f"{model}/{clip}/full/beam5/rec_idx" in arr.files
