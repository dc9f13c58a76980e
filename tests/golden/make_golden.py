"""Generate the golden fixtures of tests/golden/ by running the REFERENCE implementation.

The reference whisper.cpp + ggml CPU path is compiled from /root/reference sources by
oracle/ref/Makefile into oracle/_ref/libwhisper_ref.so and driven through
oracle/ref_oracle.py. Inputs are deterministic: synthetic-weight models written by
open-whisper-kit_amd/python/owk_synth.py (SHA-256 recorded so the GPU box regenerates
byte-identical files) and two clips: samples/jfk.wav (the reference's own test audio,
copied here as data) and a seeded synthetic 30 s clip.

Usage (in a container that has /root/reference):  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import ref_oracle as R  # noqa: E402
from recording import prefix_hash  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 1234
MODELS = ["tiny.en", "base.en", "tiny", "l3-mini"]

CONFIGS = {
    "greedy": dict(temperature_inc=0.0),
    "greedy_fallback": dict(),
    "beam5": dict(strategy=1, temperature_inc=0.0),
    "fixed_work": dict(no_timestamps=True, max_tokens=40, suppress_eot=True, temperature_inc=0.0),
    "token_ts": dict(temperature_inc=0.0, token_timestamps=True),
    "sampled": dict(temperature=0.4, temperature_inc=0.0, best_of=5),
}
# Configs whose result depends on mt19937 draws (sampling at t > 0, beam search's
# topk draws, temperature fallback). Their golden runs record and truncate the logits
# at the logits_filter_callback point (oracle/ref/ref_probe.cpp ref_record_cb); the GPU
# test substitutes the recorded values so the decoding logic is compared exactly.
STOCHASTIC = ("greedy_fallback", "beam5", "sampled")


def clips():
    return {"jfk": S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav")), "synth30": S.synth_audio(480000, 7)}


def row_stats(x):
    return np.stack([x.sum(axis=1, dtype=np.float64), (x.astype(np.float64) ** 2).sum(axis=1)], axis=1)


def main():
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    meta = {"seed": SEED, "models": {}, "results": {}}
    arrays = {}
    audio = clips()
    for model in MODELS:
        path = os.path.join(cache, f"synth-{model}-s{SEED}.bin")
        sha = S.write_model(path, model, SEED)
        meta["models"][model] = {"sha256": sha}
        ref = R.Ref(path)
        multilingual = S.MODELS[model][0] >= 51865
        lang = "en"
        for cname, pcm in audio.items():
            key = f"{model}/{cname}"
            mel, n_len_org = ref.mel(pcm)
            arrays[key + "/mel_head"] = mel[:, :400].copy()
            arrays[key + "/mel_stride10"] = mel[:, ::10].copy()
            arrays[key + "/mel_framesum"] = mel.sum(axis=0, dtype=np.float64)
            meta["results"][key + "/mel_shape"] = [int(mel.shape[0]), int(mel.shape[1]), int(n_len_org)]
            enc = ref.encode(0).reshape(1500, -1)
            arrays[key + "/enc_rows"] = np.concatenate([enc[:16], enc[740:756], enc[1484:]])
            arrays[key + "/enc_rowstats"] = row_stats(enc)
            k, v = ref.cross()
            d = enc.shape[1]
            arrays[key + "/cross_k_l0"] = k[: 16 * d].copy()
            arrays[key + "/cross_v_l0"] = v[: 16 * d].copy()
            sot = ref.L.whisper_token_sot(ref.ctx)
            prompt = [sot] if not multilingual else [sot, sot + 1, sot + 1 + 100 + (S.MODELS[model][0] - 51865)]
            # transcribe token: token_transcribe = 50358 + dt (dt = n_lang - 98), multilingual only
            if multilingual:
                n_lang = S.MODELS[model][0] - 51765 - 1
                prompt = [sot, sot + 1, 50358 + (n_lang - 98)]
            lg = ref.decode(prompt, 0)
            top = np.argsort(-lg)[:64]
            arrays[key + "/prefill_top_idx"] = top.astype(np.int32)
            arrays[key + "/prefill_top_val"] = lg[top]
            rng = np.random.default_rng(0)
            sub = np.sort(rng.choice(len(lg), 2048, replace=False))
            arrays[key + "/prefill_sub_idx"] = sub.astype(np.int32)
            arrays[key + "/prefill_sub_val"] = lg[sub]
            meta["results"][key + "/prefill_prompt"] = prompt
            meta["results"][key + "/prefill_stats"] = [float(lg.mean()), float(lg.std()), int(lg.argmax())]
            # teacher-forced step: feed the greedy token, check the next logits
            t1 = int(lg.argmax())
            lg2 = ref.decode([t1], len(prompt))
            top2 = np.argsort(-lg2)[:64]
            arrays[key + "/step1_top_idx"] = top2.astype(np.int32)
            arrays[key + "/step1_top_val"] = lg2[top2]
            meta["results"][key + "/step1_token"] = t1
            if multilingual:
                probs = np.zeros(100, np.float32)
                import ctypes as C
                lid = ref.L.whisper_lang_auto_detect(ref.ctx, 0, 8, probs.ctypes.data_as(C.POINTER(C.c_float)))
                meta["results"][key + "/lang_detect"] = [int(lid), probs.tolist()]
            for cfg_name, cfg in CONFIGS.items():
                if model in ("base.en", "l3-mini") and cfg_name in ("sampled", "greedy_fallback") and cname == "synth30":
                    continue
                rec = cfg_name in STOCHASTIC
                ret, segs = ref.full(pcm, language=lang, record_topk=rec, **cfg)
                meta["results"][f"{key}/full/{cfg_name}"] = {"ret": ret, "segments": segs}
                if rec:
                    off, prefix, idx, val = ref.recorded()
                    k = f"{key}/full/{cfg_name}"
                    arrays[k + "/rec_hash"] = np.array(
                        [prefix_hash(prefix[off[i]:off[i + 1]]) for i in range(len(off) - 1)], np.uint64)
                    arrays[k + "/rec_idx"] = np.where(idx < 0, 65535, idx).astype(np.uint16)
                    arrays[k + "/rec_val"] = val
            print(model, cname, "done", flush=True)
        if multilingual:
            ret, segs = ref.full(audio["jfk"], language="auto", temperature_inc=0.0)
            meta["results"][f"{model}/jfk/full/auto_lang"] = {"ret": ret, "segments": segs}
        ref.close()
    np.savez_compressed(os.path.join(OUT, "golden.npz"), **arrays)
    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(meta, f, indent=0)
    print("wrote", os.path.join(OUT, "golden.npz"), os.path.getsize(os.path.join(OUT, "golden.npz")))


if __name__ == "__main__":
    main()
