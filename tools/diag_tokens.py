"""Diagnostic: whisper_full over a clip with the library at OWK_LIB, tokens and segments to a JSON file.
    OWK_LIB=... python tools/diag_tokens.py MODEL CLIP OUT.json [key=value params...]"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk  # noqa: E402
import owk_synth as S  # noqa: E402

model, clip, out = sys.argv[1:4]
kw = {}
for a in sys.argv[4:]:
    k, v = a.split("=")
    kw[k] = {"True": True, "False": False}.get(v, float(v) if "." in v else int(v) if v.lstrip("-").isdigit() else v)
G = os.path.join(ROOT, "tests", "golden")
pcm = {"jfk": lambda: S.read_wav_16k_mono(os.path.join(G, "jfk.wav")), "synth30": lambda: S.synth_audio(480000, 7),
       "test60": lambda: S.read_wav_16k_mono(os.path.join(G, "sf_test60.wav"))}[clip]()
owk.quiet()
w = owk.Whisper(S.ensure_model(model))
st = w.new_state()
lang = kw.pop("language", "en")
ret = w.full(st, pcm, w.params(0, language=lang, **kw))
segs = w.segments(st)
json.dump({"ret": ret, "segments": segs}, open(out, "w"))
print(model, clip, ret, len(segs), sum(len(s["tokens"]) for s in segs))
