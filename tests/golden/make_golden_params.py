"""Golden fixtures for the whisper_full_params branches the SDKs and the CLI set
(params_golden.json / .npz), produced by the REFERENCE whisper.cpp + ggml CPU path
(oracle/_ref via ref_oracle.Ref.full_ex) on the synthetic models of make_golden.py:

* initial_prompt -> whisper_tokenize (ref whisper.cpp:6944-6979, 3272-3320): ASCII, multi-byte
  UTF-8, bytes outside the vocabulary, a prompt longer than the prompt budget;
* carry_initial_prompt over 60 s (ref 6958-6971, 7120-7140, 7626-7629), with and without;
* n_max_text_ctx (the prompt budget, ref 6941, 7122-7141);
* translate (ref 6990-6996) on the multilingual tiny, language en and de; language "auto";
* max_len / split_on_word (whisper_wrap_segment, ref 6077-6128, 7689, 7734), with token timestamps;
* tdrz_enable / speaker_turn_next (ref 7654-7657; the solm suppression of whisper_process_logits)
  on the device logits path, and on the host path with a logits_filter_callback that raises solm;
* single_segment, offset_ms / duration_ms (ref 6869-6880), suppress_regex, suppress_nst,
  print_special;
* the callback contract the Swift CallbackBridge wires (ref Sources/OpenWhisperKit/
  CallbackBridge.swift:75-87): progress values (ref 7035-7040), encoder_begin (7047-7052), every
  abort_callback check (2455, 2977: once per encode and per decode call) and new_segment n_new
  with the segments the bridge reads (7693, 7738); a progress-driven cancel (the bridge's
  shouldCancel -> abort -> return -6) and an encoder_begin that returns false.

Each case: ret, segments (token data, text, t0/t1, speaker_turn_next) and the callback log.
Per (model, clip) the prefill / step-1 top-64 logits bound near-ties (tests/parity_util).

Usage (container with /root/reference):  python tests/golden/make_golden_params.py
"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 1234

P_ASCII = "So my fellow Americans, ask not what your country can do for you. 1961, Washington D.C.!"
P_UTF8 = "Ça va? Größe, naïve café — 日本語のテキスト 😀 and some plain ASCII words."
P_OOV = b"\x01\x02 ctrl \xc3\x28 bad \xff\xfe bytes \xe2\x82 cut"
P_LONG = " ".join(["the quick brown fox jumps over the lazy dog"] * 40)  # > n_text_ctx/2 tokens

G0 = dict(temperature_inc=0.0)  # greedy, no fallback (deterministic at the logit level)

CASES = {
    # name: (model, clip, ref_full kwargs, ref_full_ext kwargs)
    "prompt/tiny.en/jfk/ascii": ("tiny.en", "jfk", G0, dict(initial_prompt=P_ASCII)),
    "prompt/tiny/jfk/utf8": ("tiny", "jfk", G0, dict(initial_prompt=P_UTF8)),
    "prompt/tiny.en/jfk/oov": ("tiny.en", "jfk", G0, dict(initial_prompt=P_OOV)),
    "prompt/tiny.en/synth30/long": ("tiny.en", "synth30", G0, dict(initial_prompt=P_LONG)),
    "prompt/base.en/jfk/ts": ("base.en", "jfk", dict(G0, token_timestamps=True), dict(initial_prompt=P_ASCII)),
    "carry/tiny.en/test60": ("tiny.en", "test60", dict(G0, no_context=False),
                             dict(initial_prompt=P_ASCII, carry_initial_prompt=True)),
    "carry/tiny.en/test60/long": ("tiny.en", "test60", dict(G0, no_context=False),
                                  dict(initial_prompt=P_LONG, carry_initial_prompt=True)),
    "nocarry/tiny.en/test60": ("tiny.en", "test60", dict(G0, no_context=False), dict(initial_prompt=P_ASCII)),
    "n_max_text_ctx/tiny.en/test60": ("tiny.en", "test60", dict(G0, no_context=False),
                                      dict(initial_prompt=P_ASCII, n_max_text_ctx=24, carry_initial_prompt=True)),
    "translate/tiny/jfk/en": ("tiny", "jfk", G0, dict(translate=True)),
    "translate/tiny/synth30/de": ("tiny", "synth30", dict(G0, language="de"), dict(translate=True)),
    "translate/tiny/test60/auto": ("tiny", "test60", dict(G0, language="auto", no_context=False),
                                   dict(translate=True, initial_prompt=P_UTF8)),
    "max_len/tiny.en/test60/16": ("tiny.en", "test60", dict(G0, token_timestamps=True, no_context=False),
                                  dict(max_len=16)),
    "max_len/tiny.en/test60/16sow": ("tiny.en", "test60", dict(G0, token_timestamps=True, no_context=False),
                                     dict(max_len=16, split_on_word=True)),
    "max_len/tiny.en/jfk/1sow": ("tiny.en", "jfk", dict(G0, token_timestamps=True), dict(max_len=1, split_on_word=True)),
    "max_len/tiny/jfk/3": ("tiny", "jfk", dict(G0, token_timestamps=True), dict(max_len=3, initial_prompt=P_UTF8)),
    "tdrz/tiny.en/test60": ("tiny.en", "test60", dict(G0, no_context=False), dict(tdrz_enable=True)),
    "tdrz/tiny.en/test60/boost": ("tiny.en", "test60", dict(G0, no_context=False),
                                  dict(tdrz_enable=True, tdrz_boost=True)),
    "tdrz/tiny.en/jfk/off_boost": ("tiny.en", "jfk", G0, dict(tdrz_boost=True)),
    "single_segment/tiny.en/test60": ("tiny.en", "test60", dict(G0, single_segment=True, no_context=False), {}),
    "offset/tiny.en/test60/12s+30s": ("tiny.en", "test60", dict(G0, no_context=False),
                                      dict(offset_ms=12000, duration_ms=30000)),
    "offset/tiny.en/test60/31s": ("tiny.en", "test60", dict(G0, no_context=False), dict(offset_ms=31000)),
    "offset/tiny.en/jfk/too_short": ("tiny.en", "jfk", G0, dict(offset_ms=1000, duration_ms=90)),
    "suppress_regex/tiny.en/jfk": ("tiny.en", "jfk", G0, dict(suppress_regex="^ [a-mA-M].*")),
    "suppress_regex/tiny.en/synth30": ("tiny.en", "synth30", G0, dict(suppress_regex="[0-9]+|.*[.,!?].*")),
    "suppress_nst/tiny.en/jfk": ("tiny.en", "jfk", dict(G0, suppress_nst=True), {}),
    "suppress_nst/tiny/synth30": ("tiny", "synth30", dict(G0, suppress_nst=True), dict(initial_prompt=P_ASCII)),
    "print_special/tiny.en/jfk": ("tiny.en", "jfk", G0, dict(print_special=True)),
    "cancel/tiny.en/test60": ("tiny.en", "test60", dict(G0, no_context=False), dict(cancel_at_progress=1)),
    "enc_begin_false/tiny.en/test60": ("tiny.en", "test60", dict(G0, no_context=False), dict(enc_begin_false_at=2)),
    # the Swift SDK's whisper_full_params (ref Sources/OpenWhisperKit/WhisperContext.swift:37-79 with
    # DecodingOptions defaults, Configuration.swift:108-140): word timestamps, suppress_blank,
    # max_initial_ts 1.0, initial prompt, language auto; temperature fallback off (the fallback's
    # mt19937 sampling is pinned by recorded-logit substitution in test_gpu_parity)
    "swift/tiny/test60": ("tiny", "test60", dict(G0, language="auto", token_timestamps=True, no_context=False),
                          dict(initial_prompt=P_ASCII, max_initial_ts=1.0, suppress_blank=1)),
    "swift/tiny/jfk/translate": ("tiny", "jfk", dict(G0, language="auto", token_timestamps=True),
                                 dict(initial_prompt=P_ASCII, translate=True, max_initial_ts=1.0)),
}


def clips():
    return {"jfk": S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav")), "synth30": S.synth_audio(480000, 7),
            "test60": S.read_wav_16k_mono(os.path.join(OUT, "sf_test60.wav"))}


def main():
    import numpy as np
    import ref_oracle as R

    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    audio = clips()
    meta = {"seed": SEED, "cases": {}, "results": {}}
    arrays = {}
    for name, (model, clip, kw, ext) in CASES.items():
        ref = R.Ref(S.ensure_model(model, SEED, cache))
        ext = dict(ext, callbacks=True)
        ret, segs, log = ref.full_ex(audio[clip], ext, **kw)
        ref.close()
        ext_json = {k: (v.hex() if isinstance(v, bytes) else v) for k, v in ext.items()}
        meta["cases"][name] = {"model": model, "clip": clip, "params": kw, "ext": ext_json,
                               "bytes_fields": [k for k, v in ext.items() if isinstance(v, bytes)],
                               "ret": ret, "segments": segs, "callbacks": log}
        print(name, ret, len(segs), "segments", sum(len(s["tokens"]) for s in segs), "tokens",
              sum(s["speaker_turn_next"] for s in segs), "turns", len(log["events"]), "events", flush=True)
    # near-tie bound per (model, clip): prefill + teacher-forced step-1 logits of the first window
    for model, clip in sorted({(m, c) for m, c, _, _ in CASES.values()}):
        ref = R.Ref(S.ensure_model(model, SEED, cache))
        key = f"{model}/{clip}"
        ref.mel(audio[clip])
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
    np.savez_compressed(os.path.join(OUT, "params_golden.npz"), **arrays)
    with open(os.path.join(OUT, "params_golden.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
