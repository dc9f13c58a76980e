"""Golden fixtures for Q5_0 models (q5_golden.json / q5_golden.npz), produced by the REFERENCE
whisper.cpp + ggml CPU path (oracle/_ref/libwhisper_ref.so via oracle/ref_oracle.py).

The Q5_0 files are written by owk_synth.quantize_q5_0, the restatement of whisper-quantize
(tests/test_q5.py checks it byte-identical against the reference's own quantizer built into
oracle/_ref/whisper-quantize). The reference then runs ggml's q5_0 x q8_0 mul_mat path
(ggml-cpu/arch/x86/quants.c) on them.

Noise floors. Q8_0 rounds every activation to 8 bits per 32-block, so an f32-level change of
an activation (re-associated attention sums, a different reduction order) flips a rounding
and moves the product by a whole Q8 step: the path amplifies ulp noise ~2^4 more than the
F16 path. The reference itself moves by the recorded "noise_floor/*" when its input is
perturbed by 1e-7 relative noise (below the f32 ulp of most samples); tests/test_q5.py
bounds the GPU error by 2x that floor, and decoded sequences may part only where the two
tokens are within 2x the logit floor of each other.

Usage (in a container that has /root/reference):  python tests/golden/make_golden_q5.py [q8_0]
(q8_0 / q4_0 / q4_1 / q5_1: the same fixtures for those files -> q8_ / q4_ / q41_ / q51_golden.*)

K-quants (q2_k / q3_k / q4_k / q5_k / q6_k -> q2k_ .. q6k_golden.*): the files are written by the
reference's own quantizer (oracle/_ref/whisper-quantize, ggml quantize_row_q*_K_ref) -- there is no
Python restatement of its iterative scale search -- on base.en instead of tiny.en (K-quant rows are
multiples of 256: tiny's 384-wide rows do not quantize) and l3-mini. The reference runs its
q*_K x q8_K path (CPU repack 8x8 kernels for q4_K / q2_K, as x86 builds with AVX2 / AVX-512 do).
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
TF_TOKENS = 48
KIND = sys.argv[1] if len(sys.argv) > 1 else "q5_0"
K_KINDS = ("q2_k", "q3_k", "q4_k", "q5_k", "q6_k")
assert KIND in ("q5_0", "q8_0", "q4_0", "q4_1", "q5_1") + K_KINDS
MODELS = ["base.en", "l3-mini"] if KIND in K_KINDS else ["tiny.en", "l3-mini"]
QUANT = os.path.join(ROOT, "oracle", "_ref", "whisper-quantize")


def quantize(src, dst):
    """The quantized file's SHA-256: owk_synth's restatement for the 32-blocks, the reference's own
    whisper-quantize for the K-quants."""
    if KIND not in K_KINDS:
        return S.quantize_q5_0(src, dst, kind=KIND)
    import hashlib
    import subprocess

    subprocess.run([QUANT, src, dst, KIND], check=True, capture_output=True)
    return hashlib.sha256(open(dst, "rb").read()).hexdigest()


def main():
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    meta = {"seed": SEED, "models": {}, "results": {}}
    arrays = {}
    audio = {"jfk": S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav")), "synth30": S.synth_audio(480000, 7)}
    for model in MODELS:
        src = os.path.join(cache, f"synth-{model}-s{SEED}.bin")
        S.write_model(src, model, SEED)
        path = os.path.join(cache, f"synth-{model}-{KIND}-s{SEED}.bin")
        meta["models"][model] = {"sha256": quantize(src, path)}
        ref = R.Ref(path)
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
            runs = {"greedy": dict(temperature_inc=0.0),
                    "fixed_work": dict(no_timestamps=True, max_tokens=40, suppress_eot=True, temperature_inc=0.0)}
            for cfg, kw in runs.items():
                ret, segs = ref.full(pcm, language="en", **kw)
                meta["results"][f"{key}/full/{cfg}"] = {"ret": ret, "segments": segs}
            # teacher-forced decode: prompt + the greedy tokens one per call, the logits of every step
            flat = [t[0] for s in meta["results"][f"{key}/full/greedy"]["segments"] for t in s["tokens"]]
            seq = prompt + flat[:TF_TOKENS]
            meta["results"][key + "/tf_tokens"] = seq
            ref.mel(pcm)
            ref.encode(0)
            tf = ref.decode_steps(seq)
            tf_idx = np.argsort(-tf, axis=1)[:, :16]
            arrays[key + "/tf_top_idx"] = tf_idx.astype(np.int32)
            arrays[key + "/tf_top_val"] = np.take_along_axis(tf, tf_idx, axis=1)
            # the reference's own sensitivity: the same calls on the input perturbed by 1e-7
            rng = np.random.default_rng(0)
            pp = (pcm * (1 + 1e-7 * rng.standard_normal(len(pcm)))).astype(np.float32)
            ref.mel(pp)
            enc_p = ref.encode(0).reshape(1500, -1)
            rows_p = np.concatenate([enc_p[:16], enc_p[740:756], enc_p[1484:]])
            d = np.abs(rows_p - arrays[key + "/enc_rows"])
            meta["results"][key + "/noise_floor/enc_rows"] = {"max": float(d.max()), "mean": float(d.mean())}
            lgp = ref.decode(prompt, 0)
            lgp2 = ref.decode([t1], len(prompt))
            dl = max(float(np.abs(lgp[top] - lg[top]).max()), float(np.abs(lgp2[top2] - lg2[top2]).max()))
            meta["results"][key + "/noise_floor/logits"] = dl
            tfp = ref.decode_steps(seq)
            meta["results"][key + "/noise_floor/tf_logits"] = float(
                np.abs(np.take_along_axis(tfp, tf_idx, axis=1) - arrays[key + "/tf_top_val"]).max())
            # decoded sequences: leading tokens on which the reference agrees with itself when its
            # input carries 1e-7 relative noise (min over 3 perturbations)
            for cfg, kw in runs.items():
                want = [t[0] for s in meta["results"][f"{key}/full/{cfg}"]["segments"] for t in s["tokens"]]
                agree = []
                for seed in range(3):
                    r = np.random.default_rng(seed)
                    xp = (pcm * (1 + 1e-7 * r.standard_normal(len(pcm)))).astype(np.float32)
                    got = [t[0] for s in ref.full(xp, language="en", **kw)[1] for t in s["tokens"]]
                    agree.append(next((i for i, (a, b) in enumerate(zip(got, want)) if a != b), min(len(got), len(want))))
                meta["results"][f"{key}/noise_floor/agree/{cfg}"] = min(agree)
            print(model, cname, "floors", meta["results"][key + "/noise_floor/enc_rows"], dl, flush=True)
        ref.close()
    stem = {"q4_1": "q41", "q5_1": "q51"}.get(KIND, KIND[:2] + ("k" if KIND in K_KINDS else "")) + "_golden"
    meta["kind"] = KIND
    np.savez_compressed(os.path.join(OUT, stem + ".npz"), **arrays)
    with open(os.path.join(OUT, stem + ".json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
