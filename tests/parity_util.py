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


class StepForcer:
    """logits_filter_callback of the decision check: teacher-forces the reference's decoded tokens
    (tf_golden.json `windows`) at every global step <= `upto` and leaves every later step to the
    decoder, recording the prefix each call sees -- so the decoder's own greedy pick at each step after
    `upto` is read back from the next call (tokens[n_tokens - 1]) or from where its window ended.
    Global step index: windows in order, a window contributing len(tokens) steps plus its
    <|endoftext|> step (none for an open window, which ended at the step limit or on a timestamp
    reaching the end of the audio). `watch`: the one state of a batch to force (None: every call)."""

    def __init__(self, tf, eot, n_vocab, token_data_type, upto, watch=None, pre=None):
        self.pre = pre  # the case's own logits filter (a Python callback), applied first
        self.windows, self.open_end = tf["windows"], tf["open_end"]
        self.eot, self.n_vocab, self.upto, self.watch = eot, n_vocab, upto, watch
        self.n_steps = [len(w) + (0 if o else 1) for w, o in zip(self.windows, self.open_end)]
        self.start = np.concatenate([[0], np.cumsum(self.n_steps)]).astype(int).tolist()
        self.seen = []  # per window: the decoder's picks at steps 0 .. calls - 2
        self.window = -1
        TD = C.POINTER(token_data_type)
        proto = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, TD, C.c_int, C.POINTER(C.c_float), C.c_void_p)
        self.cfunc = proto(self._cb)

    def _cb(self, ctx, state, tokens, n_tokens, logits, user):
        if self.watch is not None and state != self.watch:
            return
        if self.pre is not None:
            self.pre(ctx, state, tokens, n_tokens, logits, user)
        if n_tokens == 0:
            self.window += 1
            self.seen.append([])
        w = self.window
        if n_tokens > 0:
            self.seen[w].append(int(tokens[n_tokens - 1].id))
        keep = getattr(self, "kept", None) is not None and w < len(self.windows) and n_tokens <= len(self.windows[w])
        if w >= len(self.windows) or self.start[w] + n_tokens > self.upto:
            if keep:
                self._keep_step(w, n_tokens, tokens, logits)
            return
        if keep and self.every:  # decision_forced: the decoder's view of this step before it is forced
            self._keep_step(w, n_tokens, tokens, logits)
        win = self.windows[w]
        if n_tokens > len(win) or (n_tokens == len(win) and self.open_end[w]):
            return
        t = win[n_tokens] if n_tokens < len(win) else self.eot
        lg = np.ctypeslib.as_array(logits, shape=(self.n_vocab,))
        fin = np.isfinite(lg)
        lg[t] = (float(lg[fin].max()) if fin.any() else 0.0) + 40.0

    def _keep_step(self, w, n_tokens, tokens, logits):
        win = self.windows[w]
        self._keep(self.start[w] + n_tokens, win[n_tokens] if n_tokens < len(win) else self.eot,
                   np.ctypeslib.as_array(logits, shape=(self.n_vocab,)), [int(tokens[i].id) for i in range(n_tokens)])

    def keep_logits(self, beg, space=-1, tid_initial=-1, every=False):
        """record, at every step the decoder decides itself (global step > upto), what a decision between two
        tokens needs from the logits this call sees (the callback point, ref whisper.cpp:6254), after the
        filters the reference applies between that point and its timestamp rule (6258-6329: blank suppression
        at the first step, timestamps in pairs, the initial-timestamp limit `tid_initial` (round(max_initial_ts
        / 0.02)), timestamps increasing): the top 8 ids' logits, the reference token's logit and the rule's
        margin |logsumexp(timestamp logits) - max(text logits)| (decision_ties) and the decoder's own pick from
        those logits: the timestamp rule (ref 6331-6357: every text logit dropped when the timestamp log-mass
        exceeds the best text logit), then the greedy argmax of whisper_sample_token. every: record the steps
        that are forced too (decision_forced), from the logits the decoder computed before the forcing"""
        self.beg, self.space, self.tid_initial, self.kept, self.every = beg, space, tid_initial, {}, every
        return self

    def _keep(self, g, t, lg, prefix):
        lg = np.where(np.isfinite(lg), lg, -np.inf).astype(np.float64)
        beg = self.beg
        if not prefix:
            if self.space >= 0:
                lg[self.space] = -np.inf
            lg[self.eot] = -np.inf
            if self.tid_initial >= 0:
                lg[beg + self.tid_initial + 1:] = -np.inf
        else:
            last_ts = prefix[-1] >= beg
            penult_ts = len(prefix) < 2 or prefix[-2] >= beg
            if last_ts:
                if penult_ts:
                    lg[beg:] = -np.inf
                else:
                    lg[:self.eot] = -np.inf
        ts_seen = [x for x in prefix if x >= beg]
        if ts_seen:
            lg[beg:ts_seen[-1]] = -np.inf  # decoder.seek_delta / 2 = the last timestamp's index
        ts = lg[beg:]
        m = float(ts.max())
        lse = m + float(np.log(np.exp(ts - m).sum())) if np.isfinite(m) else -np.inf
        top = np.argpartition(-lg, 8)[:8]
        text_max = float(lg[:beg].max())
        pick = beg + int(np.argmax(ts)) if lse > text_max else int(np.argmax(lg))
        self.kept[g] = ({int(i): float(lg[i]) for i in top}, float(lg[t]), abs(lse - text_max), pick)

    def first_disagreement(self):
        """(global step, decoder pick (-1: ended the window there), reference token) of the first step
        after `upto` where the decoder's own pick is not the reference's; None if every step agrees"""
        for w, picks in enumerate(self.seen):
            if w >= len(self.windows):
                return self.start[-1], -2, -1  # a window the reference never decoded
            win = self.windows[w]
            for k, p in enumerate(picks):
                g = self.start[w] + k
                t = win[k] if k < len(win) else self.eot
                if g > self.upto and p != t:
                    return g, p, t
            if len(picks) + 1 < self.n_steps[w]:  # the window ended at step len(picks); the reference went on
                g = self.start[w] + len(picks)
                if g > self.upto:
                    return g, -1, win[len(picks)]
        if len(self.seen) < len(self.windows):
            return self.start[len(self.seen)], -2, -1
        return None


def decision_check(run, tf, arr, key, eot, beg, n_vocab, token_data_type, want_segments, watch=None, max_iter=16,
                   log=print, pre=None):
    """Every decode step of a greedy run compared with the reference's decision on the same prefix.

    `run(cfunc)` runs the case's whisper_full with `cfunc` as logits_filter_callback and returns its
    segments. Iteratively: force the reference's tokens up to the last disagreement found, leave the
    rest to the decoder, find the next step whose greedy pick differs (StepForcer). Each disagreement
    must be a step the reference does not decide itself (tests/golden/make_golden_tf.py): one of its own
    realisations (its x86-64-v3 / baseline x86-64 builds, 1e-7 input perturbations) flips it, or its
    own gap between the two choices is within 2x the largest movement of those logits across its
    realisations at that step (the timestamp rule's margin when a timestamp is involved). The final run
    (forced through the last disagreement, free after it) must give the reference's tokens. Returns
    (steps compared, [(step, pick, reference, reason)])."""
    upto, found = -1, []
    for _ in range(max_iter):
        f = StepForcer(tf, eot, n_vocab, token_data_type, upto, watch, pre)
        segs = run(f.cfunc)
        d = f.first_disagreement()
        if d is None:
            break
        assert d[1] != -2, f"{key}: the decoder's windows differ from the reference's at step {d[0]}"
        found.append(d)
        upto = d[0]
    else:
        raise AssertionError(f"{key}: more than {max_iter} disagreeing steps: {found}")
    assert [t[0] for s in segs for t in s["tokens"]] == [t[0] for s in want_segments for t in s["tokens"]], \
        f"{key}: the run forced through step {upto} does not end on the reference's tokens"
    out = judge_disagreements(found, tf, arr, key, eot, beg)
    n = sum(StepForcer(tf, eot, n_vocab, token_data_type, -1).n_steps)
    log(f"[decisions] {key}: {n}/{n} steps compared on the reference's prefixes, {len(out)} disagreement(s)"
        + "".join(f"; step {g}: {p} vs {t} ({why})" for g, p, t, why in out))
    return n, out


def judge_disagreements(found, tf, arr, key, eot, beg):
    """[(global step, decoder pick (-1: ended the window), reference token)] -> the reason each is a step the
    reference does not decide itself (tf_golden format: `realisations` flips, per-step `floor` / `floor_ts`,
    the base run's candidates and timestamp margin); an AssertionError for any other"""
    flips = {}
    for name, r in tf["realisations"].items():
        for g, _, _ in r["flips"]:
            flips.setdefault(g, []).append(name)
    cand, cval = arr[key + "/cand"], arr[key + "/cand_logit"]
    floor, floor_ts, ts_margin = arr[key + "/floor"], arr[key + "/floor_ts"], arr[key + "/ts_margin"]
    out = []
    for g, p, t in found:
        if g in flips:
            out.append((g, p, t, f"reference self-flip ({', '.join(flips[g])})"))
            continue
        pp = eot if p == -1 else p
        if pp >= beg or t >= beg:  # a timestamp on either side: the timestamp rule decided the step
            gap, bound, what = abs(float(ts_margin[g])), 2.0 * float(floor_ts[g]), "timestamp-rule margin"
        else:
            ids = cand[g].tolist()
            assert pp in ids and t in ids, f"{key} step {g}: pick {pp} / reference {t} not among the reference's candidates"
            gap = float(cval[g][ids.index(t)] - cval[g][ids.index(pp)])
            bound, what = 2.0 * float(floor[g]), "logit gap"
        assert gap <= bound, (f"{key} step {g}: decoder picks {p}, reference {t}: the reference's {what} {gap:.3e} is "
                              f"above 2x its own per-step floor {bound / 2:.3e} and no realisation of it flips the step")
        out.append((g, p, t, f"{what} {gap:.2e} <= 2 x reference floor {bound / 2:.2e}"))
    return out


def decision_forced(run, tf, arr, key, eot, beg, n_vocab, token_data_type, want_tokens, space=-1, tid_initial=-1,
                    watch=None, log=print, pre=None):
    """Every decode step compared with the reference's decision on the same prefix, in ONE run: the run is
    teacher-forced onto the reference's tokens at every step, and at each step the decoder's own greedy pick
    is derived from the logits it computed on that prefix, through the reference's filters between the
    callback point and its pick (StepForcer.keep_logits: blank suppression at a window's first step
    (`space`), timestamp pairs, the initial-timestamp limit `tid_initial`, increasing timestamps, the
    timestamp rule, argmax). Each step whose pick differs from the reference's token is judged as
    decision_check judges it (judge_disagreements: a reference self-flip or within 2x its per-step floor).
    The run must end on `want_tokens` (an open window's last pick, which no later callback sees, included).
    Returns (steps compared, [(step, pick, reference, reason)])."""
    total = sum(StepForcer(tf, eot, n_vocab, token_data_type, -1).n_steps)
    f = StepForcer(tf, eot, n_vocab, token_data_type, total, watch, pre).keep_logits(beg, space, tid_initial, every=True)
    segs = run(f.cfunc)
    assert [t[0] for s in segs for t in s["tokens"]] == list(want_tokens), f"{key}: the forced run left the reference's tokens"
    assert len(f.kept) == total, f"{key}: {len(f.kept)} of {total} steps seen"
    found = []
    for w, win in enumerate(tf["windows"]):
        for k in range(f.n_steps[w]):
            g = f.start[w] + k
            t = win[k] if k < len(win) else eot
            p = f.kept[g][3]
            if p != t:
                found.append((g, -1 if p == eot else p, t))
    out = judge_disagreements(found, tf, arr, key, eot, beg)
    log(f"[decisions] {key}: {total}/{total} steps compared on the reference's prefixes (one forced run), "
        f"{len(out)} disagreement(s)" + "".join(f"; step {g}: {p} vs {t} ({why})" for g, p, t, why in out))
    return total, out


def decision_ties(run, windows, open_end, eot, beg, n_vocab, token_data_type, tie, key, max_iter, log=print, space=-1,
                  tid_initial=-1, want_tokens=None):
    """The every-step check for a run no teacher-forced reference fixture covers (configs[4] at 10 minutes,
    14 312 steps): as decision_check -- force the reference's tokens up to the last disagreement, leave the
    rest to the decoder, find the next step whose greedy pick differs -- but each disagreement is judged on
    the GPU's own logits at that step: the two choices (or the timestamp rule's two sides, when a timestamp
    is involved) must lie within `tie`, the near-tie bound the free-run comparison uses (TIE_FACTOR x the
    measured logit error). A pick no later call sees (an open window's last step) is read from the result:
    the run forced through the last disagreement must end on `want_tokens`, the reference's result tokens.
    At most `max_iter` runs; returns (steps compared on the reference's prefixes, total steps,
    [(step, pick, reference, gap)])."""
    tf = {"windows": windows, "open_end": open_end}
    total = sum(StepForcer(tf, eot, n_vocab, token_data_type, -1).n_steps)
    upto, out = -1, []
    for _ in range(max_iter):
        f = StepForcer(tf, eot, n_vocab, token_data_type, upto).keep_logits(beg, space, tid_initial)
        segs = run(f.cfunc)
        d = f.first_disagreement()
        if d is None:
            upto = total
            if want_tokens is not None:
                assert [t[0] for s in segs for t in s["tokens"]] == list(want_tokens), \
                    f"{key}: the run forced through step {max([-1] + [o[0] for o in out])} does not end on the reference's tokens"
            break
        g, p, t = d
        assert p != -2, f"{key}: the decoder's windows differ from the reference's at step {g}"
        top, lt, ts_margin, _ = f.kept[g]
        pp = eot if p == -1 else p  # -1: the decoder ended the window at this step (its pick: <|endoftext|>)
        if pp >= beg or t >= beg:  # a timestamp on either side: the timestamp rule decided the step
            gap, what = ts_margin, "timestamp-rule margin"
        else:
            assert pp in top, f"{key} step {g}: the decoder's pick {pp} is not among its own top logits"
            gap, what = top[pp] - lt, "logit gap"
        assert gap <= tie, f"{key} step {g}: decoder picks {p}, reference {t}: {what} {gap:.3e} above the tie bound {tie:.3e}"
        out.append((g, p, t, f"{what} {gap:.2e}"))
        log(f"[decisions] {key}: run {len(out)}: step {g}: decoder {p}, reference {t} ({what} {gap:.2e})")
        upto = g
    n = min(upto, total)
    log(f"[decisions] {key}: {n}/{total} steps compared on the reference's prefixes, {len(out)} disagreement(s), "
        f"each within the tie bound {tie:.2e} of the GPU's own logits"
        + "".join(f"; step {g}: {p} vs {t} ({why})" for g, p, t, why in out)
        + ("" if n >= total else f"; steps after {n} not compared ({max_iter} runs)"))
    return n, total, out


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


def compare_all_steps(w, tf_golden, key, run, want_segments, n_cmp, watch=None, log=print, pre=None):
    """After a free-run comparison (compare_segments) that parted from the reference at a near-tie
    (n_cmp < the reference's token count), compare every remaining step with decision_check on the
    reference's prefixes. A parting without a teacher-forced fixture is logged as such (its tail stays
    unverified). Returns the steps compared (None when the free run already matched completely or no
    fixture covers the case)."""
    import owk

    n_ref = sum(len(s["tokens"]) for s in want_segments)
    if n_cmp >= n_ref:
        return None
    if tf_golden is None or key not in tf_golden[0]["cases"]:
        # no teacher-forced fixture for this case yet (make_golden_tf.py): the free-run comparison above is
        # all that is checked -- logged, so a missing fixture is visible in every run
        log(f"[decisions] {key}: parted at token {n_cmp}; NO teacher-forced fixture -- steps after the parting unchecked")
        return None
    meta, arr = tf_golden
    L = w.L
    L.whisper_token_beg.argtypes = [C.c_void_p]
    n, _ = decision_check(run, meta["cases"][key], arr, key, L.whisper_token_eot(w.ctx), L.whisper_token_beg(w.ctx),
                          w.n_vocab, owk.TokenData, want_segments, watch=watch, log=log, pre=pre)
    return n
