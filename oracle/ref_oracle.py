"""TEST INFRASTRUCTURE -- ctypes driver of the compiled reference (oracle/_ref/libwhisper_ref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
It runs the reference ggml CPU implementation (built from /root/reference sources by
oracle/ref/Makefile) through the accessors of oracle/ref/ref_probe.cpp.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_LIB = os.environ.get("OWK_REF_LIB", os.path.join(HERE, "_ref", "libwhisper_ref.so"))


class RefFullCfg(C.Structure):
    _fields_ = [("strategy", C.c_int), ("n_threads", C.c_int), ("best_of", C.c_int), ("beam_size", C.c_int),
                ("temperature", C.c_float), ("temperature_inc", C.c_float), ("no_timestamps", C.c_int),
                ("max_tokens", C.c_int), ("suppress_eot", C.c_int), ("token_timestamps", C.c_int),
                ("no_context", C.c_int), ("single_segment", C.c_int), ("language", C.c_char_p),
                ("suppress_nst", C.c_int), ("length_penalty", C.c_float),
                ("record_topk", C.c_int), ("audio_ctx", C.c_int), ("n_processors", C.c_int)]


class RefFullExt(C.Structure):  # ref_probe.cpp ref_full_ext
    _fields_ = [("initial_prompt", C.c_char_p), ("carry_initial_prompt", C.c_int), ("translate", C.c_int),
                ("max_len", C.c_int), ("split_on_word", C.c_int), ("tdrz_enable", C.c_int), ("offset_ms", C.c_int),
                ("duration_ms", C.c_int), ("suppress_regex", C.c_char_p), ("n_max_text_ctx", C.c_int),
                ("print_special", C.c_int), ("callbacks", C.c_int), ("cancel_at_progress", C.c_int),
                ("enc_begin_false_at", C.c_int), ("tdrz_boost", C.c_int), ("max_initial_ts", C.c_float),
                ("suppress_blank", C.c_int), ("detect_language", C.c_int)]


EXT_DEFAULTS = dict(initial_prompt=None, carry_initial_prompt=False, translate=False, max_len=0, split_on_word=False,
                    tdrz_enable=False, offset_ms=0, duration_ms=0, suppress_regex=None, n_max_text_ctx=0,
                    print_special=False, callbacks=False, cancel_at_progress=-1, enc_begin_false_at=0,
                    tdrz_boost=False, max_initial_ts=-1.0, suppress_blank=-1, detect_language=False)


def make_ext(**kw):
    v = dict(EXT_DEFAULTS)
    for k in kw:
        if k not in v:
            raise KeyError(k)
    v.update(kw)
    e = RefFullExt()
    for k, x in v.items():
        if isinstance(x, str):
            x = x.encode("utf-8", "surrogateescape")
        elif isinstance(x, bool):
            x = int(x)
        setattr(e, k, x)
    return e


class RefTokenData(C.Structure):
    _fields_ = [("id", C.c_int32), ("tid", C.c_int32), ("p", C.c_float), ("plog", C.c_float), ("pt", C.c_float),
                ("ptsum", C.c_float), ("t0", C.c_int64), ("t1", C.c_int64), ("t_dtw", C.c_int64),
                ("vlen", C.c_float)]


def available() -> bool:
    return os.path.exists(REF_LIB)


_libs = {}
# the reference's other x86 SIMD builds (oracle/ref/Makefile `variants`): the same ggml CPU path on a host
# without AVX-512 (x86-64-v3: AVX2 + F16C + FMA) or with SSE only (x86-64: the scalar / SSE kernels)
VARIANTS = {"v4": REF_LIB, "v3": os.path.join(HERE, "_ref", "v3", "libwhisper_ref.so"),
            "v1": os.path.join(HERE, "_ref", "v1", "libwhisper_ref.so")}


def lib(path=None):
    path = path or REF_LIB
    if path not in _libs:
        if not os.path.exists(path):
            raise FileNotFoundError(f"reference oracle not built: {path} (make -C oracle/ref)")
        L = C.CDLL(path)
        vp, ip, fp = C.c_void_p, C.c_int, C.POINTER(C.c_float)
        L.ref_init.restype = vp
        L.ref_init.argtypes = [C.c_char_p, ip, ip]
        L.ref_decoder_seek_delta.argtypes = [vp, ip]
        L.ref_dtw_data.restype = C.c_long
        L.ref_dtw_data.argtypes = [vp, fp, C.c_long]
        L.ref_init_ex.restype = vp
        L.ref_init_ex.argtypes = [C.c_char_p, ip, ip, ip]
        L.ref_free.argtypes = [vp]
        L.ref_mel.argtypes = [vp, fp, ip, ip, fp, ip, C.POINTER(ip), C.POINTER(ip), C.POINTER(ip)]
        L.ref_encode.argtypes = [vp, ip, ip]
        L.ref_get_enc.argtypes = [vp, fp, ip]
        L.ref_get_cross.restype = C.c_long
        L.ref_get_cross.argtypes = [vp, C.POINTER(C.c_uint16), C.POINTER(C.c_uint16), C.c_long]
        L.ref_decode.argtypes = [vp, C.POINTER(C.c_int), ip, ip, ip]
        L.ref_logits.restype = fp
        L.ref_logits.argtypes = [vp]
        L.ref_full.argtypes = [vp, fp, ip, C.POINTER(RefFullCfg)]
        L.ref_full_ex.argtypes = [vp, fp, ip, C.POINTER(RefFullCfg), C.POINTER(RefFullExt)]
        L.ref_cb_log.argtypes = [C.POINTER(ip), ip]
        L.ref_cb_text.restype = C.c_char_p
        L.ref_cb_text.argtypes = [ip]
        L.ref_tokenize.argtypes = [vp, C.c_char_p, C.POINTER(ip), ip]
        L.whisper_full_get_segment_speaker_turn_next.restype = C.c_bool
        L.whisper_full_get_segment_speaker_turn_next.argtypes = [vp, ip]
        L.ref_record_get.argtypes = [C.POINTER(ip), C.POINTER(ip), C.POINTER(ip), fp, C.POINTER(ip)]
        L.ref_timings.argtypes = [vp] + [C.POINTER(C.c_double)] * 6 + [C.POINTER(ip)]
        L.ref_tf_set.argtypes = [C.POINTER(ip), C.POINTER(ip), ip, ip]
        L.ref_tf_set_open.argtypes = [C.POINTER(ip), ip]
        L.ref_tf_get.argtypes = [C.POINTER(ip), fp]
        L.whisper_full_n_segments.argtypes = [vp]
        L.whisper_full_get_segment_t0.restype = C.c_int64
        L.whisper_full_get_segment_t0.argtypes = [vp, ip]
        L.whisper_full_get_segment_t1.restype = C.c_int64
        L.whisper_full_get_segment_t1.argtypes = [vp, ip]
        L.whisper_full_get_segment_text.restype = C.c_char_p
        L.whisper_full_get_segment_text.argtypes = [vp, ip]
        L.whisper_full_get_segment_no_speech_prob.restype = C.c_float
        L.whisper_full_get_segment_no_speech_prob.argtypes = [vp, ip]
        L.whisper_full_n_tokens.argtypes = [vp, ip]
        L.whisper_full_get_token_data.restype = RefTokenData
        L.whisper_full_get_token_data.argtypes = [vp, ip, ip]
        L.whisper_n_vocab.argtypes = [vp]
        L.whisper_token_sot.argtypes = [vp]
        L.whisper_lang_auto_detect.argtypes = [vp, ip, ip, fp]
        _libs[path] = L
    return _libs[path]


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Ref:
    def __init__(self, model_path: str, flash_attn: bool = True, dtw_preset: int = 0, dtw_n_top: int = -1,
                 lib_path: str | None = None):
        self.L = lib(lib_path)
        self.ctx = self.L.ref_init_ex(model_path.encode(), 1 if flash_attn else 0, dtw_preset, dtw_n_top)
        if not self.ctx:
            raise RuntimeError("reference init failed")
        self.n_vocab = self.L.whisper_n_vocab(self.ctx)
        self.dtw = dtw_preset > 0

    def close(self):
        if self.ctx:
            self.L.ref_free(self.ctx)
            self.ctx = None

    def mel(self, pcm, n_threads=8):
        pcm = np.ascontiguousarray(pcm, np.float32)
        nl, nlo, nm = C.c_int(), C.c_int(), C.c_int()
        n = self.L.ref_mel(self.ctx, fptr(pcm), len(pcm), n_threads, None, 0, nl, nlo, nm)
        out = np.zeros(n, np.float32)
        self.L.ref_mel(self.ctx, fptr(pcm), len(pcm), n_threads, fptr(out), n, nl, nlo, nm)
        return out.reshape(nm.value, nl.value), nlo.value

    def encode(self, offset=0, n_threads=8):
        assert self.L.ref_encode(self.ctx, offset, n_threads) == 0
        n = self.L.ref_get_enc(self.ctx, None, 0)
        out = np.zeros(n, np.float32)
        self.L.ref_get_enc(self.ctx, fptr(out), n)
        return out

    def cross(self):
        n = self.L.ref_get_cross(self.ctx, None, None, 0)
        k = np.zeros(n, np.uint16)
        v = np.zeros(n, np.uint16)
        self.L.ref_get_cross(self.ctx, k.ctypes.data_as(C.POINTER(C.c_uint16)),
                             v.ctypes.data_as(C.POINTER(C.c_uint16)), n)
        return k, v

    def decode(self, tokens, n_past, n_threads=8):
        arr = (C.c_int * len(tokens))(*tokens)
        assert self.L.ref_decode(self.ctx, arr, len(tokens), n_past, n_threads) == 0
        lg = np.ctypeslib.as_array(self.L.ref_logits(self.ctx), shape=(len(tokens) * self.n_vocab,))
        return lg[(len(tokens) - 1) * self.n_vocab:].copy()

    def decode_steps(self, tokens, n_threads=8):
        """Teacher-forced decode, one token per call from position 0 (the reference only
        computes the last row of a call, whisper.cpp:2950-2955): [len(tokens)][n_vocab]."""
        return np.stack([self.decode([t], i, n_threads) for i, t in enumerate(tokens)])

    def full(self, pcm, strategy=0, n_threads=8, best_of=5, beam_size=5, temperature=0.0, temperature_inc=0.2,
             no_timestamps=False, max_tokens=0, suppress_eot=False, token_timestamps=False, no_context=True,
             single_segment=False, language="en", suppress_nst=False, length_penalty=-1.0, record_topk=False,
             audio_ctx=0, n_processors=1):
        cfg = RefFullCfg(strategy, n_threads, best_of, beam_size, temperature, temperature_inc, int(no_timestamps),
                         max_tokens, int(suppress_eot), int(token_timestamps), int(no_context), int(single_segment),
                         language.encode() if language else None, int(suppress_nst), length_penalty,
                         int(record_topk), int(audio_ctx), int(n_processors))
        pcm = np.ascontiguousarray(pcm, np.float32)
        ret = self.L.ref_full(self.ctx, fptr(pcm), len(pcm), C.byref(cfg))
        return ret, self.segments(dtw=self.dtw)

    def full_ex(self, pcm, ext: dict, **kw):
        """ref_full with the whisper_full_params fields of ref_full_ext (initial_prompt, translate,
        max_len, tdrz, offsets, suppress_regex, callbacks ...). Returns (ret, segments, callback log)."""
        full_kw = {k: v for k, v in kw.items()}
        cfg_fields = dict(strategy=0, n_threads=8, best_of=5, beam_size=5, temperature=0.0, temperature_inc=0.2,
                          no_timestamps=False, max_tokens=0, suppress_eot=False, token_timestamps=False,
                          no_context=True, single_segment=False, language="en", suppress_nst=False,
                          length_penalty=-1.0, record_topk=False, audio_ctx=0, n_processors=1)
        for k in full_kw:
            if k not in cfg_fields:
                raise KeyError(k)
        cfg_fields.update(full_kw)
        c = cfg_fields
        cfg = RefFullCfg(c["strategy"], c["n_threads"], c["best_of"], c["beam_size"], c["temperature"],
                         c["temperature_inc"], int(c["no_timestamps"]), c["max_tokens"], int(c["suppress_eot"]),
                         int(c["token_timestamps"]), int(c["no_context"]), int(c["single_segment"]),
                         c["language"].encode() if c["language"] else None, int(c["suppress_nst"]),
                         c["length_penalty"], int(c["record_topk"]), int(c["audio_ctx"]), int(c["n_processors"]))
        e = make_ext(**ext)
        pcm = np.ascontiguousarray(pcm, np.float32)
        ret = self.L.ref_full_ex(self.ctx, fptr(pcm), len(pcm), C.byref(cfg), C.byref(e))
        segs = self.segments(dtw=self.dtw)
        for i, s in enumerate(segs):
            s["speaker_turn_next"] = bool(self.L.whisper_full_get_segment_speaker_turn_next(self.ctx, i))
        return ret, segs, self.cb_log()

    def tf_set(self, windows=None, force=True, open_end=None):
        """Teacher forcing for the following full() / full_ex() calls (ref_probe.cpp ref_tf_set): the
        per-window decoded token lists to force (None: off; [] with force=False: record only). Every
        greedy step records the reference's own pick on the forced prefix (its whisper_process_logits +
        whisper_sample_token on a copy of the decoder)."""
        if windows is None:
            self.L.ref_tf_set((C.c_int * 1)(0), (C.c_int * 1)(0), -1, 0)
            return
        flat = [t for w in windows for t in w]
        off = np.cumsum([0] + [len(w) for w in windows]).astype(np.int32)
        tok = np.asarray(flat + [0], np.int32)
        P = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
        self.L.ref_tf_set(P(tok), P(off), len(windows), int(force))
        if open_end is not None:  # open windows: nothing forced after the last listed token
            o = np.asarray([1 if x else 0 for x in open_end], np.int32)
            self.L.ref_tf_set_open(P(o), len(o))

    TF_NC = 16

    def tf_steps(self):
        """Steps of the last run (ref_probe.cpp ref_tf_get): dict of arrays -- window, step, pick, teacher
        (-1: none), lp_pick, lp_teacher (the reference's final logprobs), cand [n][16] / cand_logit [n][16]
        (the largest text / EOT logits at the callback point), ts_lse / text_max (the timestamp rule's two
        sides in logits)."""
        nc = self.TF_NC
        n = self.L.ref_tf_get(None, None)
        rec = np.zeros(max((5 + nc) * n, 1), np.int32)
        lp = np.zeros(max((4 + nc) * n, 1), np.float32)
        self.L.ref_tf_get(rec.ctypes.data_as(C.POINTER(C.c_int)), fptr(lp))
        rec = rec[:(5 + nc) * n].reshape(n, 5 + nc)
        lp = lp[:(4 + nc) * n].reshape(n, 4 + nc)
        return {"window": rec[:, 0], "step": rec[:, 1], "pick": rec[:, 2], "teacher": rec[:, 3],
                "lp_pick": lp[:, 0], "lp_teacher": lp[:, 1], "cand": rec[:, 5:], "cand_logit": lp[:, 2:2 + nc],
                "ts_lse": lp[:, 2 + nc], "text_max": lp[:, 3 + nc]}

    def cb_log(self):
        n = self.L.ref_cb_log(None, 0)
        buf = (C.c_int * max(n, 1))()
        self.L.ref_cb_log(buf, n)
        ev = [tuple(buf[i:i + 3]) for i in range(0, n, 3)]
        texts = []
        i = 0
        while True:
            t = self.L.ref_cb_text(i)
            if t is None:
                break
            texts.append(t.decode("utf-8", "surrogateescape"))
            i += 1
        return {"events": [list(x) for x in ev], "texts": texts}

    def tokenize(self, text: bytes):
        n = self.L.ref_tokenize(self.ctx, text, None, 0)
        n = -n if n < 0 else n
        buf = (C.c_int * max(n, 1))()
        m = self.L.ref_tokenize(self.ctx, text, buf, n)
        assert m == n, (m, n)
        return list(buf[:n])

    def dtw_data(self):
        """Alignment-head attention of the last DTW re-decode, flat [head][n_audio_ctx][n_tok]."""
        n = self.L.ref_dtw_data(self.ctx, None, 0)
        out = np.zeros(n, np.float32)
        self.L.ref_dtw_data(self.ctx, fptr(out), n)
        return out

    def recorded(self):
        """Logit entries recorded by the last full(record_topk=True): (off, prefix, idx, val)."""
        w = C.c_int()
        n = self.L.ref_record_get(None, None, None, None, C.byref(w))
        off = np.zeros(n + 1, np.int32)
        # prefix length is off[n]; query it through a first copy of the offsets
        plen = self.L.ref_record_prefix_len()
        prefix = np.zeros(max(plen, 1), np.int32)
        idx = np.zeros(n * w.value, np.int32)
        val = np.zeros(n * w.value, np.float32)
        P = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
        self.L.ref_record_get(P(off), P(prefix), P(idx), fptr(val), C.byref(w))
        return off, prefix[:plen], idx.reshape(n, w.value), val.reshape(n, w.value)

    def segments(self, dtw=False):
        L = self.L
        out = []
        for i in range(L.whisper_full_n_segments(self.ctx)):
            toks = []
            for j in range(L.whisper_full_n_tokens(self.ctx, i)):
                t = L.whisper_full_get_token_data(self.ctx, i, j)
                toks.append((t.id, t.tid, t.p, t.plog, t.pt, t.ptsum, t.t0, t.t1) + ((t.t_dtw,) if dtw else ()))
            out.append(dict(t0=L.whisper_full_get_segment_t0(self.ctx, i), t1=L.whisper_full_get_segment_t1(self.ctx, i),
                            text=L.whisper_full_get_segment_text(self.ctx, i).decode("utf-8", "replace"),
                            no_speech_prob=L.whisper_full_get_segment_no_speech_prob(self.ctx, i), tokens=toks))
        return out

    def timings(self):
        v = [C.c_double() for _ in range(6)]
        n = C.c_int()
        self.L.ref_timings(self.ctx, *[C.byref(x) for x in v], C.byref(n))
        return dict(mel_ms=v[0].value, enc_ms=v[1].value, dec_ms=v[2].value, batchd_ms=v[3].value,
                    prompt_ms=v[4].value, sample_ms=v[5].value, n_decode=n.value)
