"""Noise floors of the reference for the large-v3 Q5_0 fixtures of make_golden_large.py (merged into
large_golden.json), as make_golden_q5.py records them for the small models: the reference's own
movement when its input carries 1e-7 relative noise -- encoder rows (max, mean), prefill + step-1
top-64 logits, and the number of leading decoded tokens on which it agrees with its unperturbed
run (min over 2 perturbations) for the greedy and fixed-work configurations.

Also records, for every DTW fixture, the per-window token sequences of the reference's decode
(ref_full record_topk = 2 traces every decoder call's token prefix) so a teacher-forced GPU run can
be driven window by window.

Usage (after make_golden_large.py):  python tests/golden/make_golden_large_floor.py [dtw]
(dtw: only the window traces)
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
from make_golden_large import CONFIGS, NT, clips  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
N_PERTURB = 2


def windows_of(ref, flat, n_max=220):
    """Per-window DECODED token sequences (what the decoder sampled, before segment assembly folds
    timestamp pairs) from the traced decoder-call prefixes: a window starts where the traced prefix
    is empty again; a window that ended on <|endoftext|> decoded exactly its longest traced prefix.
    A window can also end on a kept token that is in no prefix: the n_text_ctx/2 - 4 = 220 step
    limit (ref whisper.cpp:7219) or a timestamp reaching the end of the audio (7359-7441); both only
    in the last window, whose kept token is then the last result token (an <|endoftext|> ending
    leaves the last decoded token last). None where that cannot be told."""
    off, prefix, _, _ = ref.recorded()
    longest = []
    for i in range(len(off) - 1):
        p = prefix[off[i]:off[i + 1]].tolist()
        if not p:
            longest.append([])
        elif len(p) > len(longest[-1]):
            longest[-1] = p
    for i, w in enumerate(longest[:-1]):
        if len(w) + 1 >= n_max:
            return None
    last = longest[-1]
    if len(last) + 1 >= n_max or (flat and (not last or last[-1] != flat[-1])):
        last.append(flat[-1])
    return longest


def main():
    meta = json.load(open(os.path.join(OUT, "large_golden.json")))
    arrays = dict(np.load(os.path.join(OUT, "large_golden.npz")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    audio = clips()
    dtw_only = len(sys.argv) > 1 and sys.argv[1] == "dtw"
    model = "large-v3-q5_0"
    ref = R.Ref(S.ensure_model(model, meta["seed"], cache))
    for cname, pcm in audio.items():
        if dtw_only:
            break
        key = f"{model}/{cname}"
        rng = np.random.default_rng(0)
        pp = (pcm * (1 + 1e-7 * rng.standard_normal(len(pcm)))).astype(np.float32)
        ref.mel(pp, n_threads=NT)
        enc = ref.encode(0, n_threads=NT).reshape(1500, -1)
        rows = np.concatenate([enc[:16], enc[740:756], enc[1484:]])
        d = np.abs(rows - arrays[key + "/enc_rows"])
        meta["results"][key + "/noise_floor/enc_rows"] = {"max": float(d.max()), "mean": float(d.mean())}
        prompt = meta["results"][key + "/prefill_prompt"]
        lg = ref.decode(prompt, 0, n_threads=NT)
        lg2 = ref.decode([meta["results"][key + "/step1_token"]], len(prompt), n_threads=NT)
        dl = max(float(np.abs(lg[arrays[key + "/prefill_top_idx"]] - arrays[key + "/prefill_top_val"]).max()),
                 float(np.abs(lg2[arrays[key + "/step1_top_idx"]] - arrays[key + "/step1_top_val"]).max()))
        meta["results"][key + "/noise_floor/logits"] = dl
        for cfg, kw in CONFIGS.items():
            want = [t[0] for s in meta["results"][f"{key}/full/{cfg}"]["segments"] for t in s["tokens"]]
            agree = []
            for seed in range(N_PERTURB):
                r = np.random.default_rng(seed)
                xp = (pcm * (1 + 1e-7 * r.standard_normal(len(pcm)))).astype(np.float32)
                got = [t[0] for s in ref.full(xp, n_threads=NT, language="en", **kw)[1] for t in s["tokens"]]
                agree.append(next((i for i, (a, b) in enumerate(zip(got, want)) if a != b), min(len(got), len(want))))
            meta["results"][f"{key}/noise_floor/agree/{cfg}"] = min(agree)
        print(key, "floors", meta["results"][key + "/noise_floor/enc_rows"], dl,
              {c: meta["results"][f"{key}/noise_floor/agree/{c}"] for c in CONFIGS}, flush=True)
    ref.close()
    for model, preset in meta["dtw"].items():
        ref = R.Ref(S.ensure_model(model, meta["seed"], cache), flash_attn=False, dtw_preset=preset)
        for cname, pcm in audio.items():
            key = f"{model}/{cname}"
            want = meta["results"][key + "/full/greedy_dtw"]
            ret, segs = ref.full(pcm, n_threads=NT, language="en", temperature_inc=0.0,
                                 no_timestamps=want["no_timestamps"], record_topk=2)
            flat = [t[0] for s in want["segments"] for t in s["tokens"]]
            assert [t[0] for s in segs for t in s["tokens"]] == flat
            wins = windows_of(ref, flat)
            if wins is not None:
                meta["results"][key + "/dtw_windows"] = wins
            print(key, "dtw windows", None if wins is None else [len(w) for w in wins], flush=True)
        ref.close()
    np.savez_compressed(os.path.join(OUT, "large_golden.npz"), **arrays)
    with open(os.path.join(OUT, "large_golden.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
