"""Golden fixtures for flash_attn = false contexts and DTW token timestamps
(nofa_golden.json / nofa_golden.npz), produced by the REFERENCE whisper.cpp + ggml CPU path
(oracle/_ref/libwhisper_ref.so through oracle/ref_oracle.py).

flash_attn = false switches every attention of the reference to the soft_max path
(whisper.cpp:2163-2189 encoder, 2614-2628 decoder self, 2697-2738 cross over exactly
n_audio_ctx keys); dtw_token_timestamps re-decodes each window's text with alignment-head
capture (whisper.cpp:7744-7756, 8837-8998). Same synthetic models and clips as
make_golden.py (the SHA-256 of each model is in golden.json).

Usage (in a container that has /root/reference):  python tests/golden/make_golden_nofa.py
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

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 1234
# model -> (whisper_alignment_heads_preset, dtw_n_top): TINY_EN = 3, TINY = 4, N_TOP_MOST = 1 (l3-mini: the last text layer, 20 heads; 2 layers
# exceed the reference's 128 MB dtw_mem_size on a 220-token window and abort)
DTW = {"tiny.en": (3, -1), "tiny": (4, -1), "l3-mini": (1, 1)}


def clips():
    return {"jfk": S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav")), "synth30": S.synth_audio(480000, 7)}


def main():
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    meta = {"seed": SEED, "dtw": DTW, "results": {}}
    arrays = {}
    audio = clips()
    for model, (preset, n_top) in DTW.items():
        path = os.path.join(cache, f"synth-{model}-s{SEED}.bin")
        S.write_model(path, model, SEED)
        ref = R.Ref(path, flash_attn=False, dtw_preset=preset, dtw_n_top=n_top)
        multilingual = S.MODELS[model][0] >= 51865
        for cname, pcm in audio.items():
            key = f"{model}/{cname}"
            ref.mel(pcm)
            enc = ref.encode(0).reshape(1500, -1)
            arrays[key + "/enc_rows"] = np.concatenate([enc[:16], enc[740:756], enc[1484:]])
            arrays[key + "/enc_rowstats"] = np.stack(
                [enc.sum(axis=1, dtype=np.float64), (enc.astype(np.float64) ** 2).sum(axis=1)], axis=1)
            sot = ref.L.whisper_token_sot(ref.ctx)
            prompt = [sot]
            if multilingual:
                n_lang = S.MODELS[model][0] - 51765 - 1
                prompt = [sot, sot + 1, 50358 + (n_lang - 98)]
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
            # synth30 without timestamp tokens: its windows otherwise hit a timestamp-mass
            # near-tie (margin 0.03 logit) that f32 re-association cannot reproduce
            no_ts = cname == "synth30"
            ret, segs = ref.full(pcm, language="en", temperature_inc=0.0, no_timestamps=no_ts)
            meta["results"][key + "/full/greedy_dtw"] = {"ret": ret, "segments": segs, "no_timestamps": no_ts}
            if cname == "jfk":  # one window: the captured attention of its DTW re-decode
                cap = ref.dtw_data()
                n_ah = {"tiny.en": 8, "tiny": 6, "l3-mini": 20}[model]
                arrays[key + "/dtw_cap"] = cap
                seek_delta = ref.L.ref_decoder_seek_delta(ref.ctx, 0)
                n_len_org = ref.mel(pcm)[1]
                meta["results"][key + "/dtw_in"] = {"n_ah": n_ah, "n_tok": int(cap.size // (1500 * n_ah)),
                                                    "sot_len": 2 if multilingual else 1,
                                                    "n_frames": min(3000, seek_delta, n_len_org)}
            print(model, cname, ret, len(segs), "segments", flush=True)
        ref.close()
    np.savez_compressed(os.path.join(OUT, "nofa_golden.npz"), **arrays)
    with open(os.path.join(OUT, "nofa_golden.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
