"""configs[4]'s transcription leg alone: ONE whisper_full over a synthetic buffer (sequential 30 s
windows, prompt carry, greedy, token timestamps), large-v3 F16, flash_attn = false + DTW (LARGE_V3
heads) unless --fa / --no-dtw. Prints wall time, tokens and ms per token (for profiling under rocprofv3).

    python tools/seq_asr.py [--minutes 2] [--fa] [--no-dtw] [--model large-v3-turbo]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk  # noqa: E402
import owk_synth as S  # noqa: E402

AHEADS_LARGE_V3 = 13  # whisper_alignment_heads_preset WHISPER_AHEADS_LARGE_V3 (as tools/pipeline_bench.py)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=2.0)
    ap.add_argument("--fa", action="store_true", help="flash_attn = true")
    ap.add_argument("--no-dtw", action="store_true")
    ap.add_argument("--model", default="large-v3", help="a bench model (large-v3-turbo: 4 decoder layers)")
    a = ap.parse_args()
    model = S.ensure_model(a.model, cache_dir=os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models"))
    n = int(a.minutes * 60 * 16000)
    pcm = S.synth_audio(n, 5)
    owk.quiet()
    w = owk.Whisper(model, flash_attn=a.fa, dtw_preset=0 if a.no_dtw else AHEADS_LARGE_V3)
    p = w.params(0, language="en", temperature_inc=0.0, token_timestamps=True, no_context=False)
    warm = w.new_state()
    w.full(warm, pcm[:480000], p)
    w.free_state(warm)
    st = w.new_state()
    t0 = time.perf_counter()
    ret = w.full(st, pcm, p)
    dt = time.perf_counter() - t0
    toks = sum(len(s["tokens"]) for s in w.segments(st))
    print(json.dumps({"ret": ret, "audio_s": n / 16000, "wall_s": round(dt, 3), "rtf": round(n / 16000 / dt, 2),
                      "tokens": toks, "ms_per_token": round(1e3 * dt / max(toks, 1), 3), "fa": a.fa, "dtw": not a.no_dtw, "model": a.model}))


if __name__ == "__main__":
    main()
