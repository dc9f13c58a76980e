"""Diagnostic: nofa (flash_attn = false) whisper_full on tiny.en/synth30 with the whole-K chain on/off;
first token where each run leaves the reference golden."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk  # noqa: E402
import owk_synth as S  # noqa: E402

meta = json.load(open(os.path.join(ROOT, "tests", "golden", "nofa_golden.json")))
L = owk.load()
owk.quiet()
L.owk_debug_set_whole_k_rows.argtypes = [C.c_int]
pcm = S.synth_audio(480000, 7)
for model in ("tiny.en",):
    preset, n_top = meta["dtw"][model]
    want = meta["results"][f"{model}/synth30/full/greedy_dtw"]
    r_ids = [t[0] for s in want["segments"] for t in s["tokens"]]
    for dtw in (True, False):
        w = owk.Whisper(S.ensure_model(model), flash_attn=False, dtw_preset=preset if dtw else 0, dtw_n_top=n_top)
        for lim in (0, 8):
            L.owk_debug_set_whole_k_rows(lim)
            st = w.new_state()
            ret = w.full(st, pcm, w.params(0, language="en", temperature_inc=0.0, no_timestamps=want["no_timestamps"]))
            g = [t[0] for s in w.segments(st) for t in s["tokens"]]
            first = next((i for i, (a, b) in enumerate(zip(g, r_ids)) if a != b), None)
            print(model, "dtw" if dtw else "nodtw", "whole_k_rows", lim, "ret", ret, "tokens", len(g), "ref", len(r_ids),
                  "first diff", first, flush=True)
        w.close()
