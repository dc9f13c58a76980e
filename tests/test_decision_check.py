"""CPU checks of the every-step comparison (tests/parity_util.StepForcer / decision_check) and of the
fixtures it reads (tests/golden/tf_golden.*, the cli_default injected goldens).

A scripted greedy decoder stands in for whisper_full: it calls the logits_filter_callback once per step
with its own preferred token on top, takes the argmax afterwards (so a forced token wins), and ends a
window on <|endoftext|> or at a step limit -- the call pattern of whisper_full_with_state at t = 0
(ref src/whisper.cpp:7130-7557). Planted disagreements must be found at exactly their steps, each
judged by the reference's per-step floor, and the final forced run must end on the reference's tokens.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import owk
from parity_util import StepForcer, decision_check, decision_ties

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EOT, BEG, NV = 50, 60, 80


def fake_run(windows, open_end, plant, limit=12):
    """run(cfunc) -> segments of a scripted decoder: at global step g (counted as StepForcer does) it
    prefers plant[g] (-1: end the window) when its prefix is the reference's, the reference's token
    otherwise-equal, and token 7 once its prefix has left the reference's"""
    n_steps = [len(w) + (0 if o else 1) for w, o in zip(windows, open_end)]
    start = np.concatenate([[0], np.cumsum(n_steps)]).astype(int)

    def run(cfunc):
        toks_all = []
        for w, win in enumerate(windows):
            prefix = []
            while True:
                k = len(prefix)
                g = start[w] + k
                on_ref = prefix == win[:k]
                want = (win[k] if k < len(win) else EOT) if on_ref else 7
                if on_ref and g in plant:
                    want = EOT if plant[g] == -1 else plant[g]
                lg = np.zeros(NV, np.float32)
                lg[want] = 1.0
                td = (owk.TokenData * max(k, 1))()
                for i, t in enumerate(prefix):
                    td[i].id = t
                cfunc(None, None, td, k, lg.ctypes.data_as(C.POINTER(C.c_float)), None)
                pick = int(lg.argmax())
                if pick == EOT:
                    break
                prefix.append(pick)
                if len(prefix) >= limit or (open_end[w] and on_ref and len(prefix) == len(win) and prefix == win):
                    break
            toks_all.append(prefix)
        return [{"tokens": [[t] for t in p]} for p in toks_all]
    return run


def fixture(windows, open_end, floor=1.0):
    n = sum(len(w) + (0 if o else 1) for w, o in zip(windows, open_end))
    cand = np.tile(np.arange(16, dtype=np.int32), (n, 1))
    cand[:, 15] = EOT
    cval = np.linspace(1.0, 0.0, 16, dtype=np.float32)[None].repeat(n, 0)
    arr = {"k/cand": cand, "k/cand_logit": cval, "k/floor": np.full(n, floor, np.float32),
           "k/floor_ts": np.full(n, floor, np.float32), "k/ts_margin": np.zeros(n, np.float32)}
    tf = {"windows": windows, "open_end": open_end, "realisations": {"v3": {"flips": [[4, 9, 3]]}}}
    return tf, arr


def want_of(windows):
    return [{"tokens": [[t] for t in w]} for w in windows]


def test_agreeing_decoder_compares_every_step():
    windows, open_end = [[1, 2, 3], [4, 5]], [False, False]
    tf, arr = fixture(windows, open_end)
    n, found = decision_check(fake_run(windows, open_end, {}), tf, arr, "k", EOT, BEG, NV, owk.TokenData,
                              want_of(windows))
    assert n == 4 + 3 and found == []


def test_planted_disagreements_found_in_order():
    windows, open_end = [[1, 2, 3, 4, 5], [6, 7]], [False, False]
    tf, arr = fixture(windows, open_end)
    plant = {1: 9, 4: 9, 7: -1}  # a different token, a reference self-flip step, an early end of window 2
    n, found = decision_check(fake_run(windows, open_end, plant), tf, arr, "k", EOT, BEG, NV, owk.TokenData,
                              want_of(windows))
    assert [(g, p, t) for g, p, t, _ in found] == [(1, 9, 2), (4, 9, 5), (7, -1, 7)]
    assert "self-flip" in found[1][3] and "logit gap" in found[0][3]


def test_disagreement_beyond_the_floor_fails():
    windows, open_end = [[1, 2, 3]], [False]
    tf, arr = fixture(windows, open_end, floor=0.01)  # the reference's own spread far below its gap
    with pytest.raises(AssertionError, match="above 2x its own per-step floor"):
        decision_check(fake_run(windows, open_end, {2: 9}), tf, arr, "k", EOT, BEG, NV, owk.TokenData,
                       want_of(windows))


def test_open_window_has_no_eot_step():
    windows, open_end = [[1, 2, 3, 4]], [True]
    f = StepForcer({"windows": windows, "open_end": open_end}, EOT, NV, owk.TokenData, -1)
    assert f.n_steps == [4] and f.start == [0, 4]
    tf, arr = fixture(windows, open_end)
    n, found = decision_check(fake_run(windows, open_end, {}, limit=4), tf, arr, "k", EOT, BEG, NV, owk.TokenData,
                              want_of(windows))
    assert n == 4 and found == []


def flat_of(windows):
    return [t for w in windows for t in w]


def test_decision_ties_judged_on_own_logits():
    """decision_ties (configs[4] at 10 minutes): each disagreement judged by the decoder's own logit gap
    (1.0 in the scripted decoder) against the tie bound"""
    windows, open_end = [[1, 2, 3, 4], [5, 6]], [False, False]
    plant = {1: 9, 6: -1}  # a different token; window 2 ended early (<|endoftext|> at its step 1)
    n, total, out = decision_ties(fake_run(windows, open_end, plant, limit=6), windows, open_end, EOT, BEG, NV,
                                  owk.TokenData, 1.5, "k", 8, log=lambda s: None, want_tokens=flat_of(windows))
    assert n == total == 8 and [(g, p, t) for g, p, t, _ in out] == [(1, 9, 2), (6, -1, 6)]
    with pytest.raises(AssertionError, match="above the tie bound"):
        decision_ties(fake_run(windows, open_end, plant, limit=6), windows, open_end, EOT, BEG, NV, owk.TokenData,
                      0.5, "k", 8, log=lambda s: None)


def test_decision_ties_reads_open_window_end_from_result():
    """the last step of an open window (a timestamp reaching the end of the audio) follows no call: the
    decoder's pick there is checked through the final run's result tokens"""
    windows, open_end = [[1, 2, 3]], [True]
    run = fake_run(windows, open_end, {2: 9}, limit=3)
    with pytest.raises(AssertionError, match="does not end on the reference's tokens"):
        decision_ties(run, windows, open_end, EOT, BEG, NV, owk.TokenData, 1.5, "k", 8, log=lambda s: None,
                      want_tokens=flat_of(windows))
    n, total, out = decision_ties(fake_run(windows, open_end, {}, limit=3), windows, open_end, EOT, BEG, NV,
                                  owk.TokenData, 1.5, "k", 8, log=lambda s: None, want_tokens=flat_of(windows))
    assert n == total == 3 and out == []


def test_tf_golden_fixture_consistent():
    path = os.path.join(GOLDEN, "tf_golden.json")
    if not os.path.exists(path):
        pytest.skip("tf_golden.json not generated")
    meta = json.load(open(path))
    arr = np.load(os.path.join(GOLDEN, "tf_golden.npz"))
    assert meta["cases"], "no cases"
    for key, c in meta["cases"].items():
        n = sum(len(w) + (0 if o else 1) for w, o in zip(c["windows"], c["open_end"]))
        assert n == c["n_steps"], key
        for a in ("cand", "cand_logit", "floor", "floor_ts", "ts_margin"):
            assert arr[f"{key}/{a}"].shape[0] == n, (key, a)
        assert np.isfinite(arr[key + "/floor"]).all() and (arr[key + "/floor"] >= 0).all()
        # the reference's own token is its best-ranked candidate whenever the step is a text decision
        steps = [(w, k) for w, o in zip(c["windows"], c["open_end"]) for k in range(len(w) + (0 if o else 1))]
        assert len(steps) == n
        assert {"v3", "v4/p0"} <= set(c["realisations"]), key


def test_cli_default_golden_runs_the_fallback():
    """the cli_default fixtures decode every window with beam search first and at least one window again
    by sampled best-of at t = 0.2 (make_golden_cli_default.py counts the attempts)"""
    meta = json.load(open(os.path.join(GOLDEN, "golden.json")))
    keys = [k for k in meta["results"] if k.endswith("/full/cli_default")]
    assert len(keys) >= 4
    for k in keys:
        r = meta["results"][k]
        assert r["params"] == dict(strategy=1, beam_size=5, best_of=5, temperature=0.0, temperature_inc=0.2)
        assert r["attempts"] >= 2, k
