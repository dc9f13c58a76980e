import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        meta = json.load(f)
    arrays = np.load(os.path.join(GOLDEN, "golden.npz"))
    return meta, arrays


@pytest.fixture(scope="session")
def model_path(golden):
    """Synthetic model files regenerated from the seed; SHA-256 must match the fixtures."""
    import owk_synth as S

    meta, _ = golden
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    made = {}

    def get(model):
        if model not in made:
            path = os.path.join(cache, f"synth-{model}-s{meta['seed']}.bin")
            want = meta["models"][model]["sha256"]
            sha_file = path + ".sha256"
            ok = os.path.exists(path) and os.path.exists(sha_file) and open(sha_file).read().strip() == want
            if not ok:
                sha = S.write_model(path, model, meta["seed"])
                assert sha == want, f"synthetic {model} differs from the fixture's model ({sha} != {want})"
                with open(sha_file, "w") as f:
                    f.write(sha)
            made[model] = path
        return made[model]

    return get


@pytest.fixture(scope="session")
def clips():
    import owk_synth as S

    return {"jfk": S.read_wav_16k_mono(os.path.join(GOLDEN, "jfk.wav")), "synth30": S.synth_audio(480000, 7)}


@pytest.fixture(scope="session")
def tf_golden():
    """Teacher-forced reference decisions and per-step floors (tests/golden/make_golden_tf.py); None
    before they are generated"""
    path = os.path.join(GOLDEN, "tf_golden.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        meta = json.load(f)
    return meta, np.load(os.path.join(GOLDEN, "tf_golden.npz"))
