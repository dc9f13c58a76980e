"""Full-depth golden fixtures for the headline BASELINE models (large_golden.json / .npz), produced
by the REFERENCE whisper.cpp + ggml CPU path (oracle/_ref/libwhisper_ref.so via ref_oracle.py).

SURVEY 8(c) "large-v3-turbo/large-v3 synthetic: SHA-256 + stats + 1k-element slices of the same
tensors, token ids; q5_0 large-v3: same". Models: synthetic large-v3 (32 + 32 layers), large-v3-turbo
(32 + 4 layers) and large-v3 Q5_0 (owk_synth.quantize_q5_0, byte-identical to the reference's
whisper-quantize; tests/test_q5.py). Clips: samples/jfk.wav and the seeded synthetic 30 s clip.

Per (model, clip): mel slices (large-v3 only: all three share the 128-bin front end), encoder
rows + per-row stats, layer-0 and last-layer cross K/V rows, prefill / teacher-forced step-1
top-64 logits, whisper_full greedy (temperature_inc = 0) and the bench's fixed-work decode
(no_timestamps, EOT suppressed, max_tokens = 219 -> 220 tokens). flash_attn = false + DTW with
the WHISPER_AHEADS_LARGE_V3 / _LARGE_V3_TURBO presets (ref whisper.cpp:394-395).

Usage (container with /root/reference; ~10 min on 8 cores):  python tests/golden/make_golden_large.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import ref_oracle as R  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 1234
MODELS = ["large-v3", "large-v3-turbo", "large-v3-q5_0"]
FIXED_MAX_TOKENS = 219
CONFIGS = {
    "greedy": dict(temperature_inc=0.0),
    "fixed_work": dict(no_timestamps=True, max_tokens=FIXED_MAX_TOKENS, suppress_eot=True, temperature_inc=0.0),
}
# model -> whisper_alignment_heads_preset (include/whisper.h enum: LARGE_V3 = 13, LARGE_V3_TURBO = 14)
DTW = {"large-v3": 13, "large-v3-turbo": 14}
N_AHEADS = {13: 10, 14: 6}  # ref whisper.cpp:394-395
NT = int(os.environ.get("REF_THREADS", "8"))


def clips():
    return {"jfk": S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav")), "synth30": S.synth_audio(480000, 7)}


def row_stats(x):
    return np.stack([x.sum(axis=1, dtype=np.float64), (x.astype(np.float64) ** 2).sum(axis=1)], axis=1)


def prompt_of(ref):
    sot = ref.L.whisper_token_sot(ref.ctx)
    n_lang = S.MODELS["large-v3"][0] - 51765 - 1
    return [sot, sot + 1, 50358 + (n_lang - 98)]


def main():
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    meta = {"seed": SEED, "models": {}, "results": {}, "dtw": DTW}
    arrays = {}
    audio = clips()
    n_len_org = {}
    for model in MODELS:
        t_model = time.time()
        path = S.ensure_model(model, SEED, cache)
        meta["models"][model] = {"sha256": S.file_sha256(path)}
        ref = R.Ref(path)
        L_dec = S.MODELS[model.replace("-q5_0", "")][8]
        for cname, pcm in audio.items():
            key = f"{model}/{cname}"
            mel, n_len_org[cname] = ref.mel(pcm, n_threads=NT)
            if model == "large-v3":
                arrays[key + "/mel_head"] = mel[:, :400].copy()
                arrays[key + "/mel_stride10"] = mel[:, ::10].copy()
                arrays[key + "/mel_framesum"] = mel.sum(axis=0, dtype=np.float64)
            meta["results"][key + "/mel_shape"] = [int(mel.shape[0]), int(mel.shape[1]), int(n_len_org[cname])]
            enc = ref.encode(0, n_threads=NT).reshape(1500, -1)
            d = enc.shape[1]
            arrays[key + "/enc_rows"] = np.concatenate([enc[:16], enc[740:756], enc[1484:]])
            arrays[key + "/enc_rowstats"] = row_stats(enc)
            k, v = ref.cross()
            per_layer = k.size // L_dec  # [layer][1536 (FA padding)][d]
            last = (L_dec - 1) * per_layer
            arrays[key + "/cross_k_l0"] = k[: 16 * d].copy()
            arrays[key + "/cross_v_l0"] = v[: 16 * d].copy()
            arrays[key + "/cross_k_last"] = k[last: last + 16 * d].copy()
            arrays[key + "/cross_v_last"] = v[last: last + 16 * d].copy()
            meta["results"][key + "/cross_rows_per_layer"] = int(per_layer // d)
            prompt = prompt_of(ref)
            lg = ref.decode(prompt, 0, n_threads=NT)
            top = np.argsort(-lg)[:64]
            arrays[key + "/prefill_top_idx"] = top.astype(np.int32)
            arrays[key + "/prefill_top_val"] = lg[top]
            sub = np.sort(np.random.default_rng(0).choice(len(lg), 2048, replace=False))
            arrays[key + "/prefill_sub_idx"] = sub.astype(np.int32)
            arrays[key + "/prefill_sub_val"] = lg[sub]
            meta["results"][key + "/prefill_prompt"] = prompt
            meta["results"][key + "/prefill_stats"] = [float(lg.mean()), float(lg.std()), int(lg.argmax())]
            t1 = int(lg.argmax())
            lg2 = ref.decode([t1], len(prompt), n_threads=NT)
            top2 = np.argsort(-lg2)[:64]
            arrays[key + "/step1_top_idx"] = top2.astype(np.int32)
            arrays[key + "/step1_top_val"] = lg2[top2]
            meta["results"][key + "/step1_token"] = t1
            for cfg_name, cfg in CONFIGS.items():
                t = time.time()
                ret, segs = ref.full(pcm, n_threads=NT, language="en", **cfg)
                meta["results"][f"{key}/full/{cfg_name}"] = {"ret": ret, "segments": segs}
                print(model, cname, cfg_name, ret, len(segs), "segments",
                      sum(len(s["tokens"]) for s in segs), "tokens", f"{time.time() - t:.1f} s", flush=True)
        ref.close()
        if model in DTW:
            preset = DTW[model]
            ref = R.Ref(path, flash_attn=False, dtw_preset=preset)
            for cname, pcm in audio.items():
                key = f"{model}/{cname}"
                no_ts = cname == "synth30"
                ret, segs = ref.full(pcm, n_threads=NT, language="en", temperature_inc=0.0, no_timestamps=no_ts)
                meta["results"][key + "/full/greedy_dtw"] = {"ret": ret, "segments": segs, "no_timestamps": no_ts}
                cap = ref.dtw_data()
                n_ah = N_AHEADS[preset]
                arrays[key + "/dtw_cap_stats"] = np.array([cap.size, cap.sum(dtype=np.float64),
                                                           (cap.astype(np.float64) ** 2).sum()])
                if cname == "jfk":
                    arrays[key + "/dtw_cap"] = cap
                    seek_delta = ref.L.ref_decoder_seek_delta(ref.ctx, 0)
                    meta["results"][key + "/dtw_in"] = {"n_ah": n_ah, "n_tok": int(cap.size // (1500 * n_ah)),
                                                        "sot_len": 3, "n_frames": min(3000, seek_delta, n_len_org[cname])}
                print(model, cname, "dtw", ret, len(segs), "segments", flush=True)
            ref.close()
        print(model, f"done in {time.time() - t_model:.0f} s", flush=True)
    np.savez_compressed(os.path.join(OUT, "large_golden.npz"), **arrays)
    with open(os.path.join(OUT, "large_golden.json"), "w") as f:
        json.dump(meta, f, indent=0)
    print("wrote", os.path.join(OUT, "large_golden.npz"), os.path.getsize(os.path.join(OUT, "large_golden.npz")))


if __name__ == "__main__":
    main()
