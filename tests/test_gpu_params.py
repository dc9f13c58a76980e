"""GPU parity of the whisper_full_params branches the SDKs and the CLI set, and of the callback
contract, against the reference (tests/golden/make_golden_params.py -> params_golden.json):
initial_prompt (whisper_tokenize), carry_initial_prompt, n_max_text_ctx, translate, language auto,
max_len / split_on_word, tdrz_enable + speaker_turn_next, single_segment, offset_ms / duration_ms,
suppress_regex, suppress_nst, print_special, and the Swift SDK's parameter set.

Every case runs whisper_full_with_state on a fresh state with recording callbacks installed exactly
as the golden run installed them (oracle/ref/ref_probe.cpp ref_cb_*): the sequence of progress
values, encoder_begin calls, abort_callback checks (the reference checks once per encode and per
decode call, ref whisper.cpp:2455, 2977), new_segment n_new and the segments a Swift
CallbackBridge reads at each call (t0, t1, text) must equal the reference's, as must the return
code (a progress-driven cancel returns -6; an encoder_begin returning false stops with 0).
Token ids, segment bounds, text, token timestamps and speaker_turn_next are identical up to a
near-tie bounded by the measured logit error (parity_util); the callback log is compared in full
when no near-tie parted the runs.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import owk
from parity_util import compare_all_steps, LogitError, compare_segments

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

PROGRESS_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p)
ENC_BEGIN_CB = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.c_void_p, C.c_void_p)
ABORT_CB = C.CFUNCTYPE(C.c_bool, C.c_void_p)
NEW_SEG_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p)


@pytest.fixture(scope="module")
def pg():
    return json.load(open(os.path.join(GOLDEN, "params_golden.json")))


@pytest.fixture(scope="module")
def pg_arrays():
    return np.load(os.path.join(GOLDEN, "params_golden.npz"))


@pytest.fixture(scope="module")
def audio(clips):
    import owk_synth as S

    a = dict(clips)
    a["test60"] = S.read_wav_16k_mono(os.path.join(GOLDEN, "sf_test60.wav"))
    return a


_ctx = {}


def whisper(model_path, model):
    if model not in _ctx:
        _ctx[model] = owk.Whisper(model_path(model))
    return _ctx[model]


class Recorder:
    """The golden run's callbacks (ref_probe.cpp ref_cb_*), for the drop-in library."""

    def __init__(self, L, cancel_at_progress=-1, enc_begin_false_at=0):
        self.L = L
        self.events, self.texts = [], []
        self.cancel_at, self.false_at = cancel_at_progress, enc_begin_false_at
        self.cancel, self.enc_calls = False, 0
        self.c_progress = PROGRESS_CB(self._progress)
        self.c_enc = ENC_BEGIN_CB(self._enc)
        self.c_abort = ABORT_CB(self._abort)
        self.c_seg = NEW_SEG_CB(self._seg)

    def _progress(self, ctx, st, progress, ud):
        self.events.append([1, progress, self.L.whisper_full_n_segments_from_state(st)])
        if self.cancel_at >= 0 and progress >= self.cancel_at:
            self.cancel = True

    def _enc(self, ctx, st, ud):
        self.enc_calls += 1
        ret = self.enc_calls != self.false_at
        self.events.append([2, self.enc_calls, int(ret)])
        return ret

    def _abort(self, ud):
        if self.events and self.events[-1][0] == 3 and self.events[-1][2] == int(self.cancel):
            self.events[-1][1] += 1
        else:
            self.events.append([3, 1, int(self.cancel)])
        return self.cancel

    def _seg(self, ctx, st, n_new, ud):
        L = self.L
        total = L.whisper_full_n_segments_from_state(st)
        self.events.append([4, n_new, total])
        for i in range(max(0, total - n_new), total):
            self.texts.append(f"{L.whisper_full_get_segment_t0_from_state(st, i)}|"
                              f"{L.whisper_full_get_segment_t1_from_state(st, i)}|"
                              + L.whisper_full_get_segment_text_from_state(st, i).decode("utf-8", "surrogateescape"))

    def install(self, p):
        p.progress_callback = C.cast(self.c_progress, C.c_void_p)
        p.encoder_begin_callback = C.cast(self.c_enc, C.c_void_p)
        p.abort_callback = C.cast(self.c_abort, C.c_void_p)
        p.new_segment_callback = C.cast(self.c_seg, C.c_void_p)


class TdrzBoost:
    """ref_probe.cpp ref_tdrz_boost_cb: solm := 1000 when finite and n_tokens % 5 == 2."""

    def __init__(self, w):
        self.n_vocab = w.n_vocab
        self.solm = w.L.whisper_token_solm(w.ctx)
        self.cfunc = owk.LOGITS_FILTER_CB(self._cb)

    def _cb(self, ctx, st, tokens, n_tokens, logits, ud):
        lg = np.ctypeslib.as_array(logits, shape=(self.n_vocab,))
        if n_tokens % 5 == 2 and np.isfinite(lg[self.solm]):
            lg[self.solm] = 1000.0


FULL_KEYS = {"temperature_inc", "no_context", "token_timestamps", "single_segment", "language", "suppress_nst"}
EXT_KEYS = {"initial_prompt", "carry_initial_prompt", "translate", "max_len", "split_on_word", "tdrz_enable",
            "offset_ms", "duration_ms", "suppress_regex", "n_max_text_ctx", "print_special", "max_initial_ts",
            "suppress_blank", "detect_language"}


def run_case(w, c, pcm, force=None):
    kw = dict(c["params"])
    assert set(kw) <= FULL_KEYS, set(kw) - FULL_KEYS
    ext = dict(c["ext"])
    lang = kw.pop("language", "en")
    p = w.params(0, language=lang, **kw)
    for k, v in ext.items():
        if k in ("callbacks", "cancel_at_progress", "enc_begin_false_at", "tdrz_boost"):
            continue
        assert k in EXT_KEYS, k
        if k in ("max_initial_ts",) and v < 0:
            continue
        if k == "suppress_blank" and v < 0:
            continue
        if k == "n_max_text_ctx" and v <= 0:
            continue
        if isinstance(v, str) or k in c["bytes_fields"]:
            # bytes into a c_char_p field: ctypes keeps the object alive with the struct
            setattr(p, k, bytes.fromhex(v) if k in c["bytes_fields"] else v.encode("utf-8"))
        elif v is None:
            continue
        else:
            setattr(p, k, v)
    rec = Recorder(w.L, ext.get("cancel_at_progress", -1), ext.get("enc_begin_false_at", 0))
    rec.install(p)
    boost = None
    if ext.get("tdrz_boost"):
        boost = TdrzBoost(w)
        p.logits_filter_callback = C.cast(boost.cfunc, C.c_void_p)
    if force is not None:  # parity_util.StepForcer (it applies the boost itself, first)
        p.logits_filter_callback = C.cast(force, C.c_void_p)
    st = w.new_state()
    ret = w.full(st, pcm, p)
    segs = w.segments(st)
    for i, s in enumerate(segs):
        s["speaker_turn_next"] = bool(w.L.whisper_full_get_segment_speaker_turn_next_from_state(st, i))
    w.free_state(st)
    return ret, segs, rec


CASES = sorted(json.load(open(os.path.join(GOLDEN, "params_golden.json")))["cases"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_params_case(pg, pg_arrays, tf_golden, model_path, audio, case):
    c = pg["cases"][case]
    owk.quiet()
    w = whisper(model_path, c["model"])
    ret, got, rec = run_case(w, c, audio[c["clip"]])
    assert ret == c["ret"], f"{case}: whisper_full returned {ret}, reference {c['ret']}"
    want = c["segments"]
    tie = LogitError.tie(w, pg, pg_arrays, f"{c['model']}/{c['clip']}", audio[c["clip"]])
    n_cmp = compare_segments(got, want, case, tie=tie)
    n_ref = sum(len(s["tokens"]) for s in want)
    if n_cmp == n_ref:
        assert [s["speaker_turn_next"] for s in got] == [s["speaker_turn_next"] for s in want], case
        assert rec.events == c["callbacks"]["events"], f"{case}: callback sequence differs"
        assert rec.texts == c["callbacks"]["texts"], f"{case}: new_segment texts differ"
    else:
        # parted at a near-tie: callbacks up to the first new_segment after the parting agree, and every
        # later decode step is compared on the reference's prefixes (parity_util.decision_check); the run
        # forced through the last disagreement reproduces the reference's callback log exactly
        print(f"[params] {case}: near-tie parting, callback log compared up to the first segment")
        ev = c["callbacks"]["events"]
        k = next((i for i, e in enumerate(ev) if e[0] == 4), len(ev))
        assert rec.events[:k] == ev[:k]
        last = {}

        def run(cfunc):
            r, segs, rr = run_case(w, c, audio[c["clip"]], force=cfunc)
            assert r == c["ret"]
            last["rec"] = rr
            return segs
        pre = TdrzBoost(w)._cb if c["ext"].get("tdrz_boost") else None
        if compare_all_steps(w, tf_golden, "params/" + case, run, want, n_cmp, pre=pre) is not None:
            assert last["rec"].events == c["callbacks"]["events"], f"{case}: callback sequence differs on the forced run"
            assert last["rec"].texts == c["callbacks"]["texts"], f"{case}: new_segment texts differ on the forced run"
    if "tdrz" in case and "boost" in case and "off" not in case:
        assert any(s["speaker_turn_next"] for s in want), "fixture must contain speaker turns"


def test_params_fixture_coverage(pg):
    """(CPU) the golden set exercises every branch the SDKs set (guards against a silently shrunk fixture)"""
    cs = pg["cases"]
    assert any(c["ret"] == -6 for c in cs.values())
    assert any(any(e[0] == 2 and e[2] == 0 for e in c["callbacks"]["events"]) for c in cs.values())
    assert any(sum(s["speaker_turn_next"] for s in c["segments"]) > 0 for c in cs.values())
    assert any(any(e[0] == 4 and e[1] > 1 for e in c["callbacks"]["events"]) for c in cs.values())  # wrap n_new > 1
    for k in ("initial_prompt", "carry_initial_prompt", "translate", "max_len", "split_on_word", "tdrz_enable",
              "offset_ms", "duration_ms", "suppress_regex", "print_special", "n_max_text_ctx"):
        assert any(c["ext"].get(k) for c in cs.values()), k
    for k in ("single_segment", "suppress_nst"):
        assert any(c["params"].get(k) for c in cs.values()), k
