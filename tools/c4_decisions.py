"""configs[4] at 10 minutes: every decode step of the GPU's whisper_full compared on the reference's prefixes
(tests/parity_util.py decision_ties over tests/golden/c4_10m_golden.json's traced windows). The free run
parts from the reference at a near-tie early (token 667 of 14 312); each further run forces the reference's
tokens through the last disagreement found and reads the decoder's own picks after it. Each disagreement must
lie within the free run's tie bound (TIE_FACTOR x the measured logit error) of the GPU's own logits.

    python tools/c4_decisions.py [--runs 24] [--fixture c4_10m_golden]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in ("open-whisper-kit_amd/python", "tests", "tests/golden", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import owk  # noqa: E402
import owk_synth as S  # noqa: E402
import test_gpu_c4 as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=24)
    ap.add_argument("--fixture", default="c4_10m_golden")
    ap.add_argument("--probe", type=int, default=None, help="one run forced through this step: print the result's tail")
    a = ap.parse_args()
    g = os.path.join(ROOT, "tests", "golden", a.fixture)
    meta, arr = json.load(open(g + ".json")), np.load(g + ".npz")
    path = S.ensure_model("large-v3", meta["seed"], os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models"))
    assert S.file_sha256(path) == meta["model_sha256"]
    pcm = S.read_wav_16k_mono(os.path.join(ROOT, "tests", "golden", "sf_test60.wav")) if meta.get("minutes", 1) == 1 \
        else S.synth_audio(int(meta["minutes"] * 60 * 16000), 5)
    owk.quiet()
    w = owk.Whisper(path, flash_attn=False, dtw_preset=meta["aheads_preset"])
    if a.probe is not None:
        import ctypes as C
        from parity_util import StepForcer
        tf = {"windows": meta["results"]["windows"], "open_end": meta["results"]["windows_open"]}
        f = StepForcer(tf, w.L.whisper_token_eot(w.ctx), w.n_vocab, owk.TokenData, a.probe)
        p = T._params(w, meta)
        p.logits_filter_callback = C.cast(f.cfunc, C.c_void_p)
        st = w.new_state()
        ret = w.full(st, pcm, p)
        segs = w.segments(st)
        got = [t[0] for s in segs for t in s["tokens"]]
        ref = [t[0] for s in meta["results"]["full"]["segments"] for t in s["tokens"]]
        print("ret", ret, "tokens", len(got), "reference", len(ref), "first disagreement", f.first_disagreement())
        print("tail", got[-8:], "reference tail", ref[-8:])
        print("last segments", [(s["t0"], s["t1"], len(s["tokens"])) for s in segs[-3:]],
              "reference", [(s["t0"], s["t1"], len(s["tokens"])) for s in meta["results"]["full"]["segments"][-3:]])
        print("last window picks", f.seen[-1][-6:], "windows seen", len(f.seen))
        return
    eps = T._logit_error(w, meta, arr, pcm)
    print(f"measured logit error {eps:.3e}; tie bound {T.TIE_FACTOR * eps:.3e}", flush=True)
    t0 = time.time()
    n, total, out = T.c4_decisions(w, meta, pcm, eps, a.runs, log=lambda s: print(s, flush=True))
    print(json.dumps({"fixture": a.fixture, "steps_compared": n, "steps": total, "disagreements": len(out),
                      "runs_limit": a.runs, "wall_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
