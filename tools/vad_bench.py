"""Silero VAD throughput on the MI355X, next to the reference CPU VAD.

  single stream : whisper_vad_detect_speech over 10 min of audio (the reference's API,
                  one LSTM recurrence of 18 750 chunks -> latency-bound)
  batched       : owk_vad_detect_batch over N independent 60 s streams (one LSTM
                  workgroup per stream; the encoder fills the chip)
  reference CPU : oracle/_ref whisper_vad_detect_speech (default context params: 4
                  threads) on the first 60 s, when oracle/_ref is present

Audio: tests/golden clips (jfk + the composite clip) tiled; input is host memory (the
C ABI's contract), so times include the H2D copy. Prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import owk  # noqa: E402
from make_golden_vad import vad_clips  # noqa: E402

MODEL = os.path.join(ROOT, "tests", "golden", "silero-v6.2.0-ggml.bin")
SR = 16000


def audio(seconds, seed):
    c = vad_clips()
    base = np.concatenate([c["jfk"], c["composite"]])
    rng = np.random.default_rng(seed)
    out = np.tile(base, int(seconds * SR // len(base)) + 2)
    start = int(rng.integers(0, len(base)))
    return np.ascontiguousarray(out[start:start + int(seconds * SR)], np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=600.0)
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--stream-seconds", type=float, default=60.0)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    L = owk.load()
    owk.quiet()
    v = L.whisper_vad_init_from_file_with_params(MODEL.encode(), L.whisper_vad_default_context_params())
    assert v
    res = {"metric": "VAD real-time factor (audio-s/wall-s)", "model": "silero v6.2.0 (reference test weights)"}

    pcm = audio(a.seconds, 1)
    assert L.whisper_vad_detect_speech(v, owk.fptr(pcm), len(pcm))  # warm-up
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        assert L.whisper_vad_detect_speech(v, owk.fptr(pcm), len(pcm))
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    res["single"] = {"audio_s": a.seconds, "chunks": int(L.whisper_vad_n_probs(v)), "wall_ms": round(1e3 * t, 3),
                     "rtf": round(a.seconds / t, 1), "us_per_chunk": round(1e6 * t / L.whisper_vad_n_probs(v), 3)}

    streams = [audio(a.stream_seconds, 100 + i) for i in range(a.streams)]
    outs = [np.zeros((len(s) + 511) // 512, np.float32) for s in streams]
    n = len(streams)
    sp = (C.POINTER(C.c_float) * n)(*[owk.fptr(s) for s in streams])
    ns = (C.c_int * n)(*[len(s) for s in streams])
    op = (C.POINTER(C.c_float) * n)(*[owk.fptr(o) for o in outs])
    assert L.owk_vad_detect_batch(v, sp, ns, n, op) == 0
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        assert L.owk_vad_detect_batch(v, sp, ns, n, op) == 0
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    tot = a.streams * a.stream_seconds
    res["batched"] = {"streams": a.streams, "stream_s": a.stream_seconds, "wall_ms": round(1e3 * t, 3),
                      "rtf": round(tot / t, 1)}
    L.whisper_vad_free(v)

    if not a.no_cpu:
        try:
            import ref_oracle as R

            if R.available():
                from make_golden_vad import lib as reflib

                RL = reflib()
                rv = RL.whisper_vad_init_from_file_with_params(MODEL.encode(), RL.whisper_vad_default_context_params())
                cpcm = np.ascontiguousarray(pcm[:60 * SR])
                t0 = time.perf_counter()
                assert RL.whisper_vad_detect_speech(rv, cpcm.ctypes.data_as(C.POINTER(C.c_float)), len(cpcm))
                t = time.perf_counter() - t0
                ref = np.ctypeslib.as_array(RL.whisper_vad_probs(rv), (RL.whisper_vad_n_probs(rv),)).copy()
                RL.whisper_vad_free(rv)
                v2 = L.whisper_vad_init_from_file_with_params(MODEL.encode(), L.whisper_vad_default_context_params())
                assert L.whisper_vad_detect_speech(v2, owk.fptr(cpcm), len(cpcm))
                mine = np.ctypeslib.as_array(L.whisper_vad_probs(v2), (L.whisper_vad_n_probs(v2),)).copy()
                L.whisper_vad_free(v2)
                res["cpu_baseline"] = {"kind": "reference", "cores": 4, "sample": "first 60 s of the single stream",
                                       "wall_ms": round(1e3 * t, 1), "rtf": round(60.0 / t, 1),
                                       "max_abs_prob_diff_vs_gpu": float(np.abs(ref - mine).max())}
        except Exception as e:  # baseline is informational
            res["cpu_baseline"] = {"error": str(e)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
