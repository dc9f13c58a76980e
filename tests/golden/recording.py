"""Recorded-logit substitution for the stochastic decoding configs (test infrastructure).

Sampling at t > 0, beam search (whose candidates are mt19937 draws, whisper.cpp:6577-6580)
and temperature fallback pick tokens by where a uniform draw lands in the CDF of the
probabilities, so f32 reordering noise in the logits can flip a pick. To compare the
decoding *logic* exactly, the golden run (tests/golden/make_golden.py) truncates every
decoder's logits at the logits_filter_callback point (whisper.cpp:6254) to a recorded
top set (oracle/ref/ref_probe.cpp ref_record_cb), and the GPU test installs `Injector`
as the callback of the drop-in library: it replaces the logits with exactly the recorded
values. Entries are keyed by a hash of the decoder's token prefix; when a prefix repeats
(a new window, another temperature) the entry nearest to the device logits is used.
"""
import ctypes as C

import numpy as np

FNV_OFF, FNV_PRIME, MASK = 0xCBF29CE484222325, 0x100000001B3, 0xFFFFFFFFFFFFFFFF


def prefix_hash(tokens):
    """64-bit FNV-1a over the little-endian int32 bytes of the token ids."""
    h = FNV_OFF
    for t in tokens:
        for b in int(t).to_bytes(4, "little", signed=True):
            h = ((h ^ b) * FNV_PRIME) & MASK
    return h


class Injector:
    def __init__(self, arrays, key, n_vocab, token_data_type):
        self.n_vocab = n_vocab
        self.by_hash = {}
        hashes, idx, val = arrays[key + "/rec_hash"], arrays[key + "/rec_idx"], arrays[key + "/rec_val"]
        for h, i, v in zip(hashes.tolist(), idx, val):
            keep = i != 65535
            self.by_hash.setdefault(h, []).append((i[keep].astype(np.int64), v[keep]))
        self.misses = 0
        self.calls = 0
        self.log = []  # (prefix, matched) of every call, for diagnostics
        TD = C.POINTER(token_data_type)
        proto = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, TD, C.c_int, C.POINTER(C.c_float), C.c_void_p)
        self.cfunc = proto(self._cb)

    def _cb(self, ctx, state, tokens, n_tokens, logits, user):
        self.calls += 1
        lg = np.ctypeslib.as_array(logits, shape=(self.n_vocab,))
        prefix = [tokens[i].id for i in range(n_tokens)]
        cands = self.by_hash.get(prefix_hash(prefix))
        self.log.append((prefix, bool(cands)))
        if not cands:
            self.misses += 1
            return
        best, best_err = None, np.inf
        for idx, val in cands:
            err = float(np.max(np.abs(lg[idx].astype(np.float64) - val))) if len(idx) else 0.0
            if not np.isfinite(err):
                err = 1e30
            if err < best_err:
                best, best_err = (idx, val), err
        lg[:] = -np.inf
        lg[best[0]] = best[1]
