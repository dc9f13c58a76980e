"""GPU parity of the long-audio window loop, reduced audio_ctx and whisper_full_parallel against
the reference (tests/golden/make_golden_extra.py -> extra_golden.json).

* long: ONE whisper_full over 60 s of real speech (sf_test60.wav): the sequential 30 s window loop,
  seek advance from timestamp tokens and the rolling prompt (no_context = false) as
  whisper_full_with_state runs them (ref whisper.cpp:7034-7769) -- not the chunk-split batching of
  tools/pipeline_bench.py's batch mode.
* audio_ctx = 768: conv / encoder / cross-KV / decoder cross-attention over 768 positions
  (ref whisper.cpp:1982-2044, 2278, 2383, 2479, 6981-6986).
* whisper_full_parallel, n_processors = 2 (ref whisper.cpp:7801-7929): the chunks run as one batch
  here; merged segments (offset and non-overlap fix-up) must equal the reference's.
Token ids, segment bounds, text and token timestamps identical up to a near-tie bounded by the
measured logit error (parity_util).
"""
import json
import os

import numpy as np
import pytest

import owk
from parity_util import LogitError, compare_segments

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def extra():
    return json.load(open(os.path.join(GOLDEN, "extra_golden.json")))


@pytest.fixture(scope="module")
def extra_arrays():
    return np.load(os.path.join(GOLDEN, "extra_golden.npz"))


@pytest.fixture(scope="module")
def test60():
    import owk_synth as S

    return S.read_wav_16k_mono(os.path.join(GOLDEN, "sf_test60.wav"))


_ctx = {}


def whisper(model_path, model):
    if model not in _ctx:
        _ctx[model] = owk.Whisper(model_path(model))
    return _ctx[model]


def _tie(w, golden, model, clips, clip):
    meta, arr = golden
    return LogitError.tie(w, meta, arr, f"{model}/{clip}", clips[clip])


def _tie60(w, extra, extra_arrays, model, test60):
    """near-tie bound measured on the first window of the same 60 s audio"""
    return LogitError.tie(w, extra, extra_arrays, f"{model}/test60", test60)


def _params(w, kw):
    kw = dict(kw)
    kw.pop("n_processors", None)
    return w.params(0, language="en", **kw)


@pytest.mark.parametrize("case", ["long/tiny.en/greedy", "long/tiny.en/token_ts", "long/base.en/greedy",
                                  "long/l3-mini/greedy"])
def test_long_audio_window_loop(extra, extra_arrays, model_path, test60, case):
    c = extra["cases"][case]
    owk.quiet()
    w = whisper(model_path, c["model"])
    st = w.new_state()
    assert w.full(st, test60, _params(w, c["params"])) == c["ret"]
    got = w.segments(st)
    assert len(c["segments"]) > 1 and c["segments"][-1]["t1"] > 3000, "fixture must span several windows"
    compare_segments(got, c["segments"], case, tie=_tie60(w, extra, extra_arrays, c["model"], test60))


@pytest.mark.parametrize("case", ["audio_ctx/tiny.en/jfk", "audio_ctx/tiny.en/synth30", "audio_ctx/l3-mini/jfk"])
def test_reduced_audio_ctx(extra, golden, model_path, clips, case):
    c = extra["cases"][case]
    owk.quiet()
    w = whisper(model_path, c["model"])
    st = w.new_state()
    assert c["params"]["audio_ctx"] == 768
    assert w.full(st, clips[c["clip"]], _params(w, c["params"])) == c["ret"]
    compare_segments(w.segments(st), c["segments"], case, tie=_tie(w, golden, c["model"], clips, c["clip"]))
    # the full-width call on the same state afterwards is the reference's plain result again
    meta, _ = golden
    st2 = w.new_state()
    assert w.full(st2, clips[c["clip"]], _params(w, dict(temperature_inc=0.0))) == 0
    want = meta["results"][f"{c['model']}/{c['clip']}/full/greedy"]["segments"]
    compare_segments(w.segments(st2), want, case + "/then-full", tie=_tie(w, golden, c["model"], clips, c["clip"]))


@pytest.mark.parametrize("case", ["parallel/tiny.en/test60", "parallel/base.en/test60"])
def test_full_parallel(extra, extra_arrays, model_path, test60, case):
    c = extra["cases"][case]
    owk.quiet()
    w = whisper(model_path, c["model"])
    L = w.L
    p = _params(w, c["params"])
    pcm = np.ascontiguousarray(test60, np.float32)
    assert L.whisper_full_parallel(w.ctx, p, owk.fptr(pcm), len(pcm), c["params"]["n_processors"]) == c["ret"]
    got = []
    for i in range(L.whisper_full_n_segments(w.ctx)):
        toks = []
        for j in range(L.whisper_full_n_tokens(w.ctx, i)):
            t = L.whisper_full_get_token_data(w.ctx, i, j)
            toks.append((t.id, t.tid, t.p, t.plog, t.pt, t.ptsum, t.t0, t.t1))
        got.append(dict(t0=L.whisper_full_get_segment_t0(w.ctx, i), t1=L.whisper_full_get_segment_t1(w.ctx, i),
                        text=L.whisper_full_get_segment_text(w.ctx, i).decode("utf-8", "replace"), tokens=toks))
    compare_segments(got, c["segments"], case, tie=_tie60(w, extra, extra_arrays, c["model"], test60))
