"""Golden fixtures for the long-audio, reduced-audio_ctx and whisper_full_parallel paths
(extra_golden.json), produced by the REFERENCE whisper.cpp + ggml CPU path (oracle/_ref via
ref_oracle.py) on the synthetic models of make_golden.py (SHA-256 in golden.json).

* long: one whisper_full over the 60 s of real speech in sf_test60.wav (the first minute of the
  reference's streaming-sortformer/test.wav) -- the sequential 30 s window loop with seek advance
  and prompt carry (no_context = false; ref whisper.cpp:7034-7769), greedy t = 0, with and without
  timestamp tokens / token timestamps.
* audio_ctx: whisper_full with audio_ctx = 768 (ref whisper.cpp:6981-6986; conv / encoder / cross
  graphs over 768 positions, 1982-2044, 2278, 2383, 2479).
* parallel: whisper_full_parallel with n_processors = 2 (ref whisper.cpp:7801-7929) on sf_test60.

Usage (container with /root/reference):  python tests/golden/make_golden_extra.py
"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import ref_oracle as R  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 1234

CASES = {
    # name: (model, clip, whisper_full kwargs)
    "long/tiny.en/greedy": ("tiny.en", "test60", dict(temperature_inc=0.0, no_context=False)),
    "long/tiny.en/token_ts": ("tiny.en", "test60", dict(temperature_inc=0.0, no_context=False, token_timestamps=True)),
    "long/base.en/greedy": ("base.en", "test60", dict(temperature_inc=0.0, no_context=False)),
    "long/l3-mini/greedy": ("l3-mini", "test60", dict(temperature_inc=0.0, no_context=False)),
    "audio_ctx/tiny.en/jfk": ("tiny.en", "jfk", dict(temperature_inc=0.0, audio_ctx=768)),
    "audio_ctx/tiny.en/synth30": ("tiny.en", "synth30", dict(temperature_inc=0.0, audio_ctx=768)),
    "audio_ctx/l3-mini/jfk": ("l3-mini", "jfk", dict(temperature_inc=0.0, audio_ctx=768)),
    "parallel/tiny.en/test60": ("tiny.en", "test60", dict(temperature_inc=0.0, n_processors=2)),
    "parallel/base.en/test60": ("base.en", "test60", dict(temperature_inc=0.0, n_processors=2)),
}


def clips():
    return {"jfk": S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav")), "synth30": S.synth_audio(480000, 7),
            "test60": S.read_wav_16k_mono(os.path.join(OUT, "sf_test60.wav"))}


def main():
    import numpy as np

    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    audio = clips()
    meta = {"seed": SEED, "cases": {}, "results": {}}
    arrays = {}
    for name, (model, clip, kw) in CASES.items():
        # a fresh context per case: with no_context = false the reference carries the prompt
        # history of the state from one whisper_full to the next (ref whisper.cpp:890-892, 7122)
        ref = R.Ref(S.ensure_model(model, SEED, cache))
        ret, segs = ref.full(audio[clip], language="en", **kw)
        ref.close()
        meta["cases"][name] = {"model": model, "clip": clip, "params": kw, "ret": ret, "segments": segs}
        print(name, ret, len(segs), "segments", sum(len(s["tokens"]) for s in segs), "tokens",
              [(s["t0"], s["t1"]) for s in segs][:6], flush=True)
    # prefill + teacher-forced step-1 logits of the first window of test60 per model: the logit
    # error the GPU shows on this audio bounds its near-ties (tests/parity_util.LogitError)
    for model in sorted({m for m, c, _ in CASES.values() if c == "test60"}):
        ref = R.Ref(S.ensure_model(model, SEED, cache))
        key = f"{model}/test60"
        ref.mel(audio["test60"])
        ref.encode(0)
        sot = ref.L.whisper_token_sot(ref.ctx)
        prompt = [sot]
        if S.MODELS[model][0] >= 51865:
            prompt = [sot, sot + 1, 50358 + (S.MODELS[model][0] - 51765 - 1 - 98)]
        lg = ref.decode(prompt, 0)
        top = np.argsort(-lg)[:64]
        arrays[key + "/prefill_top_idx"] = top.astype(np.int32)
        arrays[key + "/prefill_top_val"] = lg[top]
        meta["results"][key + "/prefill_prompt"] = prompt
        t1 = int(lg.argmax())
        lg2 = ref.decode([t1], len(prompt))
        top2 = np.argsort(-lg2)[:64]
        arrays[key + "/step1_top_idx"] = top2.astype(np.int32)
        arrays[key + "/step1_top_val"] = lg2[top2]
        meta["results"][key + "/step1_token"] = t1
        ref.close()
    np.savez_compressed(os.path.join(OUT, "extra_golden.npz"), **arrays)
    with open(os.path.join(OUT, "extra_golden.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
