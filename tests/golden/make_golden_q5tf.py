"""Teacher-forced per-step reference logits for large-v3 Q5_0 (q5tf_golden.json / .npz), produced by the
REFERENCE (oracle/_ref/libwhisper_ref.so) on the full-depth synthetic large-v3 Q5_0 model of
make_golden_large.py.

For each clip (jfk, synth30) the reference's 220 fixed-work tokens (large_golden.json
"large-v3-q5_0/<clip>/full/fixed_work": no_timestamps, EOT suppressed, greedy) are fed back one per
decode call after the fixed-work prompt [sot, en, transcribe, notimestamps] (whisper_decode, the
computation whisper_full runs for every step, ref whisper.cpp:7181, 7465-7496). Per step:
  * the candidate set: the 16 largest logits among the tokens the greedy pick can take (text
    tokens below <|endoftext|>, minus " " at the first step: the reference's filters, ref
    whisper.cpp:6213-6250, and the fixed-work EOT suppression);
  * their logits (unperturbed);
  * the noise floor: the largest |logit change| over the candidates when the reference's input is
    perturbed by 1e-7 relative noise (2 perturbations, each teacher-forced onto the same tokens).
The unperturbed argmax over the candidates must equal the reference's own token (asserted).

Usage (after make_golden_large.py; ~6 min on 8 cores):  python tests/golden/make_golden_q5tf.py
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
from make_golden_large import NT, clips  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MODEL = "large-v3-q5_0"
N_CAND = 16
N_PERTURB = 2


def allowed_mask(n_vocab, eot, blank, first):
    m = np.zeros(n_vocab, bool)
    m[:eot] = True
    if first:
        m[blank] = False
    return m


def forced_logits(ref, pcm, prompt, tokens):
    """[len(tokens)][n_vocab] logits of each fixed-work step, teacher-forced onto `tokens`."""
    ref.mel(pcm, n_threads=NT)
    ref.encode(0, n_threads=NT)
    out = [ref.decode(prompt, 0, n_threads=NT)]
    for i, t in enumerate(tokens[:-1]):
        out.append(ref.decode([t], len(prompt) + i, n_threads=NT))
    return np.stack(out)


def main():
    big = json.load(open(os.path.join(OUT, "large_golden.json")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    path = S.ensure_model(MODEL, big["seed"], cache)
    assert S.file_sha256(path) == big["models"][MODEL]["sha256"]
    ref = R.Ref(path)
    L = ref.L
    for f in ("whisper_token_eot", "whisper_token_transcribe", "whisper_token_not"):
        getattr(L, f).argtypes = [R.C.c_void_p]
    L.whisper_token_lang.argtypes = [R.C.c_void_p, R.C.c_int]
    eot = L.whisper_token_eot(ref.ctx)
    prompt = [L.whisper_token_sot(ref.ctx), L.whisper_token_lang(ref.ctx, 0), L.whisper_token_transcribe(ref.ctx),
              L.whisper_token_not(ref.ctx)]
    blank = 220  # " " in the GPT-2 byte-level vocabulary of every Whisper model
    meta = {"seed": big["seed"], "model": MODEL, "sha256": big["models"][MODEL]["sha256"], "prompt": prompt,
            "eot": eot, "blank": blank, "results": {}}
    arrays = {}
    for cname, pcm in clips().items():
        t0 = time.time()
        key = f"{MODEL}/{cname}"
        toks = [t[0] for s in big["results"][key + "/full/fixed_work"]["segments"] for t in s["tokens"]]
        assert len(toks) == 220
        lg = forced_logits(ref, pcm, prompt, toks)
        cand = np.zeros((len(toks), N_CAND), np.int32)
        for i in range(len(toks)):
            m = allowed_mask(ref.n_vocab, eot, blank, i == 0)
            v = np.where(m, lg[i], -np.inf)
            cand[i] = np.argsort(-v, kind="stable")[:N_CAND]
            assert cand[i, 0] == toks[i], f"{key} step {i}: teacher-forced argmax {cand[i, 0]} != token {toks[i]}"
        val = np.take_along_axis(lg, cand, axis=1)
        floor = np.zeros(len(toks), np.float32)
        for seed in range(N_PERTURB):
            r = np.random.default_rng(seed)
            xp = (pcm * (1 + 1e-7 * r.standard_normal(len(pcm)))).astype(np.float32)
            lp = forced_logits(ref, xp, prompt, toks)
            floor = np.maximum(floor, np.abs(np.take_along_axis(lp, cand, axis=1) - val).max(axis=1))
        arrays[key + "/tokens"] = np.array(toks, np.int32)
        arrays[key + "/cand"] = cand
        arrays[key + "/cand_val"] = val.astype(np.float32)
        arrays[key + "/floor"] = floor
        gap = val[:, 0] - val[:, 1]
        meta["results"][key] = {"n_steps": len(toks), "floor_max": float(floor.max()), "floor_median": float(np.median(floor)),
                                "steps_gap_below_2floor": int((gap <= 2 * floor).sum())}
        print(key, meta["results"][key], f"{time.time() - t0:.0f} s", flush=True)
    ref.close()
    np.savez_compressed(os.path.join(OUT, "q5tf_golden.npz"), **arrays)
    with open(os.path.join(OUT, "q5tf_golden.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
