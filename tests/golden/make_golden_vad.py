"""Generate tests/golden/vad_golden.{json,npz} by running the REFERENCE Silero VAD.

Runs the reference's whisper_vad_* C API (ref/src/whisper.cpp:4345-5496, compiled from
/root/reference by oracle/ref/Makefile into oracle/_ref/libwhisper_ref.so) on the real
Silero v6.2.0 weights the reference ships for its own test (ref/models/
for-tests-silero-v6.2.0-ggml.bin, copied here as tests/golden/silero-v6.2.0-ggml.bin) and
on deterministic clips built from samples/jfk.wav. Also records whisper_full with
params.vad = true (ref/src/whisper.cpp:7778-7799, 6643-6826, 7947-8025) on the synthetic
tiny.en model of make_golden.py.

Usage (in a container that has /root/reference):  python tests/golden/make_golden_vad.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import ref_oracle as R  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
VAD_MODEL = os.path.join(OUT, "silero-v6.2.0-ggml.bin")
SEED = 1234


class VadParams(C.Structure):  # whisper.h:192-199
    _fields_ = [("threshold", C.c_float), ("min_speech_duration_ms", C.c_int),
                ("min_silence_duration_ms", C.c_int), ("max_speech_duration_s", C.c_float),
                ("speech_pad_ms", C.c_int), ("samples_overlap", C.c_float)]


class VadCtxParams(C.Structure):  # whisper.h:682-686
    _fields_ = [("n_threads", C.c_int), ("use_gpu", C.c_bool), ("gpu_device", C.c_int)]


def vad_clips():
    """Deterministic clips: jfk, a composite with speech/silence/noise stretches, silence, tiny."""
    jfk = S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav"))
    rng = np.random.default_rng(5)
    noise = (0.01 * rng.standard_normal(32000)).astype(np.float32)
    comp = np.concatenate([np.zeros(16000, np.float32), jfk, noise, np.zeros(8000, np.float32),
                           jfk[::-1].copy(), np.zeros(4000, np.float32), jfk[:48000], 0.3 * noise[:20000],
                           S.synth_audio(64000, 11)]).astype(np.float32)
    return {"jfk": jfk, "composite": comp, "silence": np.zeros(40000, np.float32),
            "short": jfk[40000:40300].copy()}


PARAM_VARIANTS = {
    "default": {},
    "thr03": dict(threshold=0.3),
    "thr08": dict(threshold=0.8),
    "minsil500": dict(min_silence_duration_ms=500),
    "minspeech1000": dict(min_speech_duration_ms=1000),
    "maxspeech3": dict(max_speech_duration_s=3.0),
    "maxspeech1": dict(max_speech_duration_s=1.0),
    "pad0": dict(speech_pad_ms=0),
    "pad200": dict(speech_pad_ms=200),
}


def lib():
    L = R.lib()
    L.whisper_vad_default_params.restype = VadParams
    L.whisper_vad_default_context_params.restype = VadCtxParams
    L.whisper_vad_init_from_file_with_params.restype = C.c_void_p
    L.whisper_vad_init_from_file_with_params.argtypes = [C.c_char_p, VadCtxParams]
    for f in ("whisper_vad_detect_speech", "whisper_vad_detect_speech_stateful"):
        getattr(L, f).restype = C.c_bool
        getattr(L, f).argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int]
    L.whisper_vad_reset_state.argtypes = [C.c_void_p]
    L.whisper_vad_n_probs.argtypes = [C.c_void_p]
    L.whisper_vad_probs.restype = C.POINTER(C.c_float)
    L.whisper_vad_probs.argtypes = [C.c_void_p]
    L.whisper_vad_segments_from_probs.restype = C.c_void_p
    L.whisper_vad_segments_from_probs.argtypes = [C.c_void_p, VadParams]
    L.whisper_vad_segments_n_segments.argtypes = [C.c_void_p]
    L.whisper_vad_segments_get_segment_t0.restype = C.c_float
    L.whisper_vad_segments_get_segment_t0.argtypes = [C.c_void_p, C.c_int]
    L.whisper_vad_segments_get_segment_t1.restype = C.c_float
    L.whisper_vad_segments_get_segment_t1.argtypes = [C.c_void_p, C.c_int]
    L.whisper_vad_free_segments.argtypes = [C.c_void_p]
    L.whisper_vad_free.argtypes = [C.c_void_p]
    L.ref_set_vad.argtypes = [C.c_char_p]
    return L


def params(L, **kw):
    p = L.whisper_vad_default_params()
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def probs(L, vctx):
    n = L.whisper_vad_n_probs(vctx)
    return np.ctypeslib.as_array(L.whisper_vad_probs(vctx), (n,)).copy() if n else np.zeros(0, np.float32)


def segments(L, vctx, p):
    s = L.whisper_vad_segments_from_probs(vctx, p)
    out = [[L.whisper_vad_segments_get_segment_t0(s, i), L.whisper_vad_segments_get_segment_t1(s, i)]
           for i in range(L.whisper_vad_segments_n_segments(s))]
    L.whisper_vad_free_segments(s)
    return out


def main():
    L = lib()
    vctx = L.whisper_vad_init_from_file_with_params(VAD_MODEL.encode(), L.whisper_vad_default_context_params())
    assert vctx
    meta = {"model": os.path.basename(VAD_MODEL), "probs": {}, "segments": {}, "full": {}}
    arrays = {}
    clips = vad_clips()
    for name, pcm in clips.items():
        pcm = np.ascontiguousarray(pcm, np.float32)
        assert L.whisper_vad_detect_speech(vctx, pcm.ctypes.data_as(C.POINTER(C.c_float)), len(pcm))
        arrays[f"probs/{name}"] = probs(L, vctx)
        meta["probs"][name] = int(len(pcm))
        for vname, kw in PARAM_VARIANTS.items():
            if name != "composite" and vname != "default":
                continue
            meta["segments"][f"{name}/{vname}"] = segments(L, vctx, params(L, **kw))
    # stateful calls: jfk in three irregular pieces, LSTM state carried across calls
    jfk = np.ascontiguousarray(clips["jfk"])
    L.whisper_vad_reset_state(vctx)
    parts = []
    for a, b in ((0, 100000), (100000, 150000), (150000, len(jfk))):
        piece = np.ascontiguousarray(jfk[a:b])
        assert L.whisper_vad_detect_speech_stateful(vctx, piece.ctypes.data_as(C.POINTER(C.c_float)), len(piece))
        parts.append(probs(L, vctx))
    arrays["probs/jfk_stateful"] = np.concatenate(parts)
    meta["stateful_splits"] = [0, 100000, 150000, len(jfk)]
    L.whisper_vad_free(vctx)

    # whisper_full with VAD on the synthetic tiny.en model (make_golden.py's weights)
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-tiny.en-s{SEED}.bin")
    meta["full_model_sha256"] = S.write_model(path, "tiny.en", SEED)
    ref = R.Ref(path)
    L.ref_set_vad(VAD_MODEL.encode())
    for cname in ("jfk", "composite"):
        for cfg, kw in {"greedy": dict(temperature_inc=0.0),
                        "fixed": dict(temperature_inc=0.0, max_tokens=20, suppress_eot=True)}.items():
            ret, segs = ref.full(clips[cname], **kw)
            meta["full"][f"{cname}/{cfg}"] = {"ret": ret, "segments": [
                {"t0": s["t0"], "t1": s["t1"], "tokens": [t[0] for t in s["tokens"]]} for s in segs]}
    L.ref_set_vad(None)
    ref.close()
    json.dump(meta, open(os.path.join(OUT, "vad_golden.json"), "w"), indent=1)
    np.savez_compressed(os.path.join(OUT, "vad_golden.npz"), **arrays)
    print({k: len(v) for k, v in meta["segments"].items()}, {k: v.shape for k, v in arrays.items()})
    print(json.dumps(meta["full"])[:600])


if __name__ == "__main__":
    main()
