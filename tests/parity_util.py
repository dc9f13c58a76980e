"""Shared GPU-vs-reference comparison rules (test infrastructure).

Token-level comparison of whisper_full results (`compare_segments`) and the measured logit error
that bounds a legitimate numerical near-tie (`LogitError`). A parting where one run takes the
timestamp rule and the other a text token is measured on the rule's own comparison (timestamp mass
against the best text token).

Near-ties. The engine's logits differ from the reference's by re-associated f32 sums (bounded by
the measured error eps of the same model and clip: prefill + teacher-forced step-1 logits against
the reference's, `LogitError.of`). When the two runs first pick different tokens g (GPU) and r
(reference), r >= g in the reference's logits and g >= r in the GPU's, so the two tokens' logits
are within 2 eps of each other; their log-probabilities (each run's own normaliser, also within
eps) within 3 eps. A divergence is accepted only if |logprob_g - logprob_r| <= TIE_FACTOR * eps
(4 eps: one eps of margin for the error growing over later decode steps); everything decided
before it must match exactly and every case must compare a minimum number of tokens, unless the
parting is a hard tie (margin <= 1 eps: below the measured error itself).
"""
import ctypes as C

import numpy as np

LOGIT_RTOL = 1e-3      # logits |diff| <= LOGIT_RTOL * max|logit| (north star: 1e-3)
TIE_FACTOR = 4.0       # near-tie threshold = TIE_FACTOR * measured max |logit diff|
MIN_COMPARED = 8       # every case compares at least min(MIN_COMPARED, reference tokens) tokens


def is_ts(t):
    """a sampled timestamp token: its id is its own best timestamp (tid)"""
    return t[0] == t[1]


def flat_tokens(segs):
    return [(si, t) for si, s in enumerate(segs) for t in s["tokens"]]


def compare_segments(got, want, key, tie, exact=False, p_atol=None, min_compared=MIN_COMPARED, log=print):
    """Token ids, segment bounds, text, token timestamps identical to the reference's `want`.

    Compared up to the first step where the runs pick different tokens whose log-probabilities
    are within `tie` (exact=True: no divergence allowed). Token probabilities agree within p_atol
    (default max(2e-3, tie / 2): a logit error eps moves a probability p by at most ~2 eps p, and
    tie = 4 eps). Returns the number of tokens compared identical; asserts it is at least
    min(min_compared, reference tokens)."""
    if p_atol is None:
        p_atol = max(2e-3, 0.5 * tie)
    fg, fw = flat_tokens(got), flat_tokens(want)
    n_cmp, margin = len(fw), None
    for i, ((sg, g), (sw, r)) in enumerate(zip(fg, fw)):
        if g[0] != r[0]:
            margin = abs(g[3] - r[3])
            if is_ts(g) != is_ts(r):
                # one run took the timestamp rule, the other a text token: the decision is the rule's
                # comparison of the timestamp mass with the best text token (whisper_process_logits, ref
                # whisper.cpp:6339-6354). The run that chose text kept every probability, so its own
                # margin is |log p_text - log ptsum| (ptsum = the timestamp mass, whisper_token_data)
                t = r if is_ts(g) else g
                margin = min(margin, abs(t[3] - float(np.log(max(t[5], 1e-30)))))
            assert not exact and margin <= tie, (
                f"{key}: token {i} is {g[0]} vs reference {r[0]} (logprob {g[3]:.5f} vs {r[3]:.5f}, "
                f"margin {margin:.2e} > near-tie bound {tie:.2e})")
            n_cmp = i
            n_done = min(sg, sw)  # finished segments before the divergence must agree completely
            got, want = got[:n_done], want[:n_done]
            break
    else:
        assert len(fg) == len(fw), f"{key}: {len(fg)} tokens vs reference {len(fw)}"
    assert len(got) == len(want), f"{key}: {len(got)} segments vs reference {len(want)}"
    for g, r in zip(got, want):
        assert [t[0] for t in g["tokens"]] == [t[0] for t in r["tokens"]], f"{key}: token ids differ"
        assert (g["t0"], g["t1"]) == (r["t0"], r["t1"]), f"{key}: segment bounds differ"
        assert g["text"] == r["text"]
        gp = np.array([t[2] for t in g["tokens"]])
        rp = np.array([t[2] for t in r["tokens"]])
        np.testing.assert_allclose(gp, rp, atol=p_atol)
        assert [(t[6], t[7]) for t in g["tokens"]] == [(t[6], t[7]) for t in r["tokens"]], \
            f"{key}: token timestamps differ"
    note = "" if margin is None else f" (parted at a near-tie, margin {margin:.2e} <= {tie:.2e})"
    log(f"[parity] {key}: {n_cmp}/{len(fw)} tokens compared identical{note}")
    # a parting within ONE measured logit error (tie / TIE_FACTOR) is a tie no implementation with that
    # error can decide; the minimum applies to partings in the wider (1, TIE_FACTOR] eps band
    if margin is not None and margin <= tie / TIE_FACTOR and n_cmp < min(min_compared, len(fw)):
        log(f"[parity] {key}: hard tie (margin {margin:.2e} <= 1 eps = {tie / TIE_FACTOR:.2e}), minimum waived")
        return n_cmp
    assert n_cmp >= min(min_compared, len(fw)), \
        f"{key}: only {n_cmp} of {len(fw)} tokens compared before a near-tie{note} (minimum {min_compared})"
    return n_cmp


class LogitError:
    """Measured max |logit - reference| of a (context, model, clip): prefill + teacher-forced
    step-1 top-64 logits of the golden set, through the staged C API on a fresh state."""

    _cache = {}

    @classmethod
    def of(cls, w, meta, arr, key):
        ck = (id(w), key)
        if ck not in cls._cache:
            cls._cache[ck] = cls.measure(w, meta, arr, key)
        return cls._cache[ck]

    @staticmethod
    def measure(w, meta, arr, key, pcm=None):
        import owk

        L = w.L
        st = w.new_state()
        if pcm is None:
            raise ValueError("pcm required on first measurement")
        assert L.whisper_pcm_to_mel_with_state(w.ctx, st, owk.fptr(pcm), len(pcm), 1) == 0
        assert L.whisper_encode_with_state(w.ctx, st, 0, 1) == 0
        prompt = meta["results"][key + "/prefill_prompt"]
        toks = (C.c_int32 * len(prompt))(*prompt)
        assert L.whisper_decode_with_state(w.ctx, st, toks, len(prompt), 0, 1) == 0
        lg = np.ctypeslib.as_array(L.whisper_get_logits_from_state(st), shape=(len(prompt) * w.n_vocab,))
        lg = lg[(len(prompt) - 1) * w.n_vocab:].copy()
        e1 = float(np.abs(lg[arr[key + "/prefill_top_idx"]] - arr[key + "/prefill_top_val"]).max())
        one = (C.c_int32 * 1)(meta["results"][key + "/step1_token"])
        assert L.whisper_decode_with_state(w.ctx, st, one, 1, len(prompt), 1) == 0
        lg2 = np.ctypeslib.as_array(L.whisper_get_logits_from_state(st), shape=(w.n_vocab,)).copy()
        e2 = float(np.abs(lg2[arr[key + "/step1_top_idx"]] - arr[key + "/step1_top_val"]).max())
        L.whisper_free_state(st)
        w._states.remove(st)
        return max(e1, e2)

    @classmethod
    def tie(cls, w, meta, arr, key, pcm):
        ck = (id(w), key)
        if ck not in cls._cache:
            cls._cache[ck] = cls.measure(w, meta, arr, key, pcm)
        return TIE_FACTOR * cls._cache[ck]


class Forcer:
    """logits_filter_callback that teacher-forces a greedy decode onto the reference's token
    sequence: `windows` is one token list per 30 s window (each followed by <|endoftext|>); every
    logit but the forced token's is set to -inf (whisper.cpp:6254 is where the reference's own
    callback point sits). A call with no decoded tokens yet starts the next window (greedy,
    temperature_inc = 0: one call per step). Used to compare what is computed FROM a token sequence
    (DTW timestamps) independently of a near-tie parting of the free runs. `open_end[i]`: window i
    stopped at the decode-step limit after its last listed token's step, so the step after it is
    left to the decoder (its token followed no traced call)."""

    def __init__(self, windows, eot, n_vocab, token_data_type, open_end=None):
        self.windows, self.eot, self.n_vocab = [list(w) for w in windows], eot, n_vocab
        self.open_end = list(open_end) if open_end is not None else [False] * len(self.windows)
        self.calls = 0
        self.window = -1
        TD = C.POINTER(token_data_type)
        proto = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, TD, C.c_int, C.POINTER(C.c_float), C.c_void_p)
        self.cfunc = proto(self._cb)

    def _cb(self, ctx, state, tokens, n_tokens, logits, user):
        self.calls += 1
        if n_tokens == 0:
            self.window += 1
        lg = np.ctypeslib.as_array(logits, shape=(self.n_vocab,))
        win = self.windows[self.window] if 0 <= self.window < len(self.windows) else []
        if n_tokens >= len(win) and 0 <= self.window < len(self.windows) and self.open_end[self.window]:
            return
        t = win[n_tokens] if n_tokens < len(win) else self.eot
        # the forced token far above every other logit (the others are kept, so the timestamp
        # distribution -- the token's best timestamp "tid" and pt -- stays the decoder's own)
        fin = np.isfinite(lg)
        lg[t] = (float(lg[fin].max()) if fin.any() else 0.0) + 40.0


def check_cross_rows(w, st, arr, key, layer, name, n_rows=16):
    """The engine's cross-attention K/V cache rows 0..n_rows-1 of `layer` (slot 0, [t][d] f16 via
    owk_debug_cross) against the reference's kv_cross rows (whisper_build_graph_cross,
    whisper.cpp:2272-2346: K pre-scaled by 64^-0.25, V + bias). Same bar as the encoder output
    they are computed from (|diff| max < 2e-2 and mean < 1e-3, relative to max|ref| when > 1)."""
    L = w.L
    n = L.owk_debug_cross(w.ctx, st, 0, layer, None, None)
    k = np.zeros(n, np.uint16)
    v = np.zeros(n, np.uint16)
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint16))
    assert L.owk_debug_cross(w.ctx, st, 0, layer, P(k), P(v)) == n
    out = {}
    for t, got in (("k", k), ("v", v)):
        ref = arr[f"{key}/cross_{t}_{name}"].view(np.float16).astype(np.float32)
        g = got[: ref.size].view(np.float16).astype(np.float32)
        scale = max(1.0, float(np.abs(ref).max()))
        err = np.abs(g - ref)
        assert err.max() < 2e-2 * scale and err.mean() < 1e-3 * scale, (key, t, name, err.max(), err.mean(), scale)
        out[t] = float(err.max())
    return out


def rttm_activity(rttm, n_frames, spk=4, frame=0.08):
    """RTTM text -> [frame][speaker] activity (frames of 80 ms, the SortFormer output rate)"""
    m = np.zeros((n_frames, spk), bool)
    for line in rttm.splitlines():
        f = line.split()
        if len(f) < 8 or f[0] != "SPEAKER":
            continue
        s = int(f[7].rsplit("_", 1)[1])
        a = int(round(float(f[3]) / frame))
        b = int(round((float(f[3]) + float(f[4])) / frame))
        m[a:min(b, n_frames), s] = True
    return m


def rttm_activity_diff(got_rttm, ref_rttm, ref_probs, floor_max, threshold=0.5, median=11):
    """Speaker activity of two RTTMs compared frame by frame. A frame may differ only where the
    reference's own probability is within 2x its noise floor of the threshold somewhere in the
    median-filter window (a threshold crossing the reference itself makes under 1e-7 input noise).
    Returns (frames that differ, mask of differing frames outside that band)."""
    n = len(ref_probs)
    got_m, ref_m = rttm_activity(got_rttm, n), rttm_activity(ref_rttm, n)
    near = np.abs(np.asarray(ref_probs) - threshold) <= 2 * floor_max
    near_w = np.zeros_like(near)
    for s in range(-(median // 2), median // 2 + 1):
        near_w |= np.roll(near, s, axis=0)
    return int((got_m != ref_m).sum()), (got_m != ref_m) & ~near_w
