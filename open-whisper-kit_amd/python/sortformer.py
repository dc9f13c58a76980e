"""ctypes binding of the streaming-SortFormer C ABI (include/sortformer.h).

The header is the reference's streaming-sortformer/src/sortformer.h, so the same binding
drives the MI355X library (open-whisper-kit_amd/lib/libsortformer.so) and -- in tests only --
the compiled reference (oracle/_ref/libsortformer_ref.so). Buffers the C API returns through
`float **` are malloc'd by the library and released here with libc free() (sortformer.h:38).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "lib", "libsortformer.so")

_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]


class Params(C.Structure):
    _fields_ = [("chunk_len", C.c_int), ("right_context", C.c_int), ("fifo_len", C.c_int),
                ("spkcache_len", C.c_int), ("spkcache_update_period", C.c_int), ("threshold", C.c_float),
                ("median_filter", C.c_int), ("n_threads", C.c_int), ("chunk_left_context", C.c_int)]


class StreamParams(C.Structure):
    _fields_ = [("chunk_len", C.c_int), ("right_context", C.c_int), ("left_context", C.c_int),
                ("fifo_len", C.c_int), ("spkcache_len", C.c_int), ("spkcache_update_period", C.c_int)]


PRESETS = {"low": 0, "2s": 1, "3s": 2, "5s": 3}

_cache: dict[str, C.CDLL] = {}


def load(path: str | None = None) -> C.CDLL:
    path = os.path.abspath(path or os.environ.get("OWK_SF_LIB", LIB))
    if path in _cache:
        return _cache[path]
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (make)")
    L = C.CDLL(path)
    vp, ip, fp = C.c_void_p, C.c_int, C.POINTER(C.c_float)
    fpp = C.POINTER(fp)
    L.sortformer_default_params.restype = Params
    L.sortformer_init.restype = vp
    L.sortformer_init.argtypes = [C.c_char_p, Params]
    L.sortformer_free.argtypes = [vp]
    L.sortformer_load_wav.argtypes = [C.c_char_p, fpp]
    L.sortformer_compute_mel.argtypes = [vp, fp, ip, fpp, C.POINTER(ip), C.POINTER(ip)]
    L.sortformer_compute_preenc.argtypes = [vp, fp, ip, ip, ip, fpp, C.POINTER(ip)]
    L.sortformer_compute_conformer.argtypes = [vp, fp, ip, ip, ip, fpp]
    L.sortformer_compute_projection.argtypes = [vp, fp, ip, ip, fpp, C.POINTER(ip)]
    L.sortformer_compute_transformer.argtypes = [vp, fp, ip, ip, ip, fpp]
    L.sortformer_compute_prediction.argtypes = [vp, fp, ip, ip, fpp]
    L.sortformer_diarize.argtypes = [vp, fp, ip, fp, ip]
    L.sortformer_to_rttm.argtypes = [fp, ip, C.c_float, ip, C.c_char_p, C.c_char_p, ip]
    L.sortformer_stream_preset_params.restype = StreamParams
    if hasattr(L, "owk_sortformer_stream_feed_batch"):  # include/owk_sortformer.h
        L.owk_sortformer_stream_feed_batch.argtypes = [C.POINTER(vp), C.POINTER(fp), C.POINTER(ip), ip, C.POINTER(fp),
                                                       C.POINTER(ip), C.POINTER(ip)]
    L.sortformer_stream_preset_params.argtypes = [ip]
    L.sortformer_stream_init.restype = vp
    L.sortformer_stream_init.argtypes = [vp, ip]
    L.sortformer_stream_init_with_params.restype = vp
    L.sortformer_stream_init_with_params.argtypes = [vp, StreamParams]
    L.sortformer_stream_feed.argtypes = [vp, fp, ip, fp, ip]
    L.sortformer_stream_flush.argtypes = [vp, fp, ip]
    L.sortformer_stream_reset.argtypes = [vp]
    L.sortformer_stream_free.argtypes = [vp]
    _cache[path] = L
    return L


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _take(p, n: int) -> np.ndarray:
    out = np.ctypeslib.as_array(p, shape=(n,)).copy()
    _libc.free(C.cast(p, C.c_void_p))
    return out


class Sortformer:
    """One sortformer_context. `lib` is a path to a library exporting sortformer.h."""

    def __init__(self, model_path: str, lib: str | None = None, **params):
        self.L = load(lib)
        p = self.L.sortformer_default_params()
        for k, v in params.items():
            setattr(p, k, v)
        self.params = p
        self.ctx = self.L.sortformer_init(model_path.encode(), p)
        if not self.ctx:
            raise RuntimeError(f"sortformer_init failed for {model_path}")

    def close(self):
        if self.ctx:
            self.L.sortformer_free(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- staged API (sortformer.h:38-121) ----
    def mel(self, pcm: np.ndarray):
        pcm = np.ascontiguousarray(pcm, np.float32)
        out = C.POINTER(C.c_float)()
        nm, sl = C.c_int(), C.c_int()
        T = self.L.sortformer_compute_mel(self.ctx, _fp(pcm), len(pcm), C.byref(out), C.byref(nm), C.byref(sl))
        if T < 0:
            raise RuntimeError("sortformer_compute_mel failed")
        return _take(out, nm.value * T).reshape(nm.value, T), sl.value

    def preenc(self, mel: np.ndarray, seq_len: int):
        mel = np.ascontiguousarray(mel, np.float32)
        out = C.POINTER(C.c_float)()
        d = C.c_int()
        T = self.L.sortformer_compute_preenc(self.ctx, _fp(mel), mel.shape[0], mel.shape[1], seq_len,
                                             C.byref(out), C.byref(d))
        if T < 0:
            raise RuntimeError("sortformer_compute_preenc failed")
        return _take(out, T * d.value).reshape(T, d.value)

    def conformer(self, x: np.ndarray, target_layer: int = 16):
        x = np.ascontiguousarray(x, np.float32)
        out = C.POINTER(C.c_float)()
        T = self.L.sortformer_compute_conformer(self.ctx, _fp(x), x.shape[0], x.shape[1], target_layer, C.byref(out))
        if T < 0:
            raise RuntimeError("sortformer_compute_conformer failed")
        return _take(out, T * x.shape[1]).reshape(T, x.shape[1])

    def projection(self, x: np.ndarray):
        x = np.ascontiguousarray(x, np.float32)
        out = C.POINTER(C.c_float)()
        d = C.c_int()
        T = self.L.sortformer_compute_projection(self.ctx, _fp(x), x.shape[0], x.shape[1], C.byref(out), C.byref(d))
        if T < 0:
            raise RuntimeError("sortformer_compute_projection failed")
        return _take(out, T * d.value).reshape(T, d.value)

    def transformer(self, x: np.ndarray, target_layer: int = 17):
        x = np.ascontiguousarray(x, np.float32)
        out = C.POINTER(C.c_float)()
        T = self.L.sortformer_compute_transformer(self.ctx, _fp(x), x.shape[0], x.shape[1], target_layer,
                                                  C.byref(out))
        if T < 0:
            raise RuntimeError("sortformer_compute_transformer failed")
        return _take(out, T * x.shape[1]).reshape(T, x.shape[1])

    def prediction(self, x: np.ndarray):
        x = np.ascontiguousarray(x, np.float32)
        out = C.POINTER(C.c_float)()
        T = self.L.sortformer_compute_prediction(self.ctx, _fp(x), x.shape[0], x.shape[1], C.byref(out))
        if T < 0:
            raise RuntimeError("sortformer_compute_prediction failed")
        return _take(out, T * 4).reshape(T, 4)

    # ---- offline diarization (sortformer.h:126-131) ----
    def diarize(self, pcm: np.ndarray, n_frames_max: int | None = None) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, np.float32)
        n_max = n_frames_max if n_frames_max is not None else len(pcm) // 1280 + 16
        out = np.zeros((max(n_max, 1), 4), np.float32)
        n = self.L.sortformer_diarize(self.ctx, _fp(pcm), len(pcm), _fp(out), n_max)
        if n < 0:
            raise RuntimeError("sortformer_diarize failed")
        return out[:n]

    def stream(self, preset: str | None = "2s", params: StreamParams | None = None) -> "Stream":
        return Stream(self, preset, params)


def to_rttm(probs: np.ndarray, threshold: float = 0.5, median_filter: int = 11, filename: str = "audio",
            lib: str | None = None, buf_size: int = 1 << 20) -> str | None:
    L = load(lib)
    probs = np.ascontiguousarray(probs, np.float32)
    buf = C.create_string_buffer(buf_size)
    n = L.sortformer_to_rttm(_fp(probs), probs.shape[0] if probs.size else 0, threshold, median_filter,
                             filename.encode() if filename is not None else None, buf, buf_size)
    if n < 0:
        return None
    return buf.raw[:n].decode()


class Stream:
    """sortformer_stream_state (sortformer.h:169-205)."""

    def __init__(self, sf: Sortformer, preset: str | None, params: StreamParams | None):
        self.sf = sf
        L = sf.L
        if params is not None:
            self.st = L.sortformer_stream_init_with_params(sf.ctx, params)
        else:
            self.st = L.sortformer_stream_init(sf.ctx, PRESETS[preset])
        if not self.st:
            raise RuntimeError("sortformer_stream_init failed")

    def feed(self, pcm: np.ndarray) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, np.float32)
        n_max = len(pcm) // 1280 + 64
        out = np.zeros((n_max, 4), np.float32)
        n = self.sf.L.sortformer_stream_feed(self.st, _fp(pcm), len(pcm), _fp(out), n_max)
        if n < 0:
            raise RuntimeError("sortformer_stream_feed failed")
        return out[:n]

    def flush(self, n_max: int = 4096) -> np.ndarray:
        out = np.zeros((n_max, 4), np.float32)
        n = self.sf.L.sortformer_stream_flush(self.st, _fp(out), n_max)
        if n < 0:
            raise RuntimeError("sortformer_stream_flush failed")
        return out[:n]

    def reset(self):
        self.sf.L.sortformer_stream_reset(self.st)

    def close(self):
        if self.st:
            self.sf.L.sortformer_stream_free(self.st)
            self.st = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def feed_batch(streams, pcms):
    """owk_sortformer_stream_feed_batch: feed pcms[i] to streams[i] (one context) in one call;
    returns the per-stream [n_out, 4] outputs."""
    n = len(streams)
    L = streams[0].sf.L
    arrs = [np.ascontiguousarray(p, np.float32) for p in pcms]
    outs = [np.zeros((len(a) // 1280 + 64, 4), np.float32) for a in arrs]
    n_out = (C.c_int * n)()
    ret = L.owk_sortformer_stream_feed_batch((C.c_void_p * n)(*[s.st for s in streams]),
                                             (C.POINTER(C.c_float) * n)(*[_fp(a) for a in arrs]),
                                             (C.c_int * n)(*[len(a) for a in arrs]), n,
                                             (C.POINTER(C.c_float) * n)(*[_fp(o) for o in outs]),
                                             (C.c_int * n)(*[o.shape[0] for o in outs]), n_out)
    if ret != 0:
        raise RuntimeError("owk_sortformer_stream_feed_batch failed")
    return [o[:k] for o, k in zip(outs, n_out)]

