"""The reference's per-step decisions and per-step noise floor over the configs[4] 10-minute fixture
(c4_10m_golden.json, make_golden_c4.py --minutes 10): the make_golden_tf.py method at configs[4]'s length.

The 10-minute free runs part at near-ties (the reference against itself on 1e-7-perturbed audio keeps
identical tokens for only 1 783 of 14 312), so tests/test_gpu_c4.py compares EVERY step on the reference's
prefixes: the GPU run is teacher-forced onto the fixture's traced windows and its own greedy pick at each
step must be the reference's token, or the step must be one the reference does not decide itself. This
script records what that judgement needs, from the reference (oracle/_ref builds of ref src/whisper.cpp):

  1. base: the fixture's whisper_full (synthetic large-v3 F16, flash_attn = false, DTW LARGE_V3 heads,
     PARAMS of make_golden_c4.py) teacher-forced onto its own traced windows (ref_probe.cpp ref_tf_set): at
     every step the reference's own pick on the forced prefix (its whisper_process_logits +
     whisper_sample_token, ref whisper.cpp:6177-6445, 6460-6592) must equal the forced token -- the
     mechanism checks itself; per step the 16 largest text / EOT logits at the callback point and the
     timestamp rule's margin (ts log-mass - best text logit) are the base values;
  2. REALISATIONS, each teacher-forced onto the same windows: the AVX-512 build on the audio perturbed by
     1e-7 relative noise (seed 0) and the x86-64-v3 (AVX2 + F16C + FMA) build -- another summation order of
     the same ggml CPU path; per step the steps it flips and the largest |logit - base| over the base
     candidates it also ranks (and of the timestamp margin) = the per-step floor.

Written to c4_10m_tf.json / .npz under case key "c4_10m" in tf_golden's format (tests/parity_util.py
decision_forced reads it). Each run is cached under OWK_MODEL_CACHE (about 1.5 h per run on 8 cores).

Usage (container with /root/reference, after make -C oracle/ref all variants):
    python tests/golden/make_golden_c4_tf.py [--realisations v4/p0,v3,...]
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
from make_golden_c4 import AHEADS_LARGE_V3, NT, OUT, PARAMS, workload  # noqa: E402
from make_golden_large import SEED  # noqa: E402
from make_golden_tf import floors  # noqa: E402

KEY = "c4_10m"
REALISATIONS = {"v4/p0": ("v4", 0), "v4/p1": ("v4", 1), "v3": ("v3", None), "v3/p0": ("v3", 0), "v1": ("v1", None)}


def forced_steps(name, var, seed, pcm, res, path, cache):
    """tf_steps of the reference (library variant `var`, 1e-7 perturbation `seed` or None) teacher-forced
    onto the fixture's windows; cached per run"""
    keep = os.path.join(cache, f"c4_10m_tf_{name.replace('/', '_')}-{S.file_sha256(path)[:16]}.npz")
    if os.path.exists(keep):
        return dict(np.load(keep))
    x = pcm if seed is None else (pcm * (1 + 1e-7 * np.random.default_rng(seed).standard_normal(len(pcm)))).astype(np.float32)
    t = time.time()
    ref = R.Ref(path, lib_path=R.VARIANTS[var], flash_attn=False, dtw_preset=AHEADS_LARGE_V3)
    ref.tf_set(res["windows"], force=True, open_end=res["windows_open"])
    ret, segs = ref.full(x, n_threads=NT, **PARAMS)
    st = ref.tf_steps()
    ref.tf_set(None)
    ref.close()
    assert ret == res["full"]["ret"]
    flat = [tk[0] for s in segs for tk in s["tokens"]]
    assert flat == [tk[0] for s in res["full"]["segments"] for tk in s["tokens"]], f"{name}: forced run left the tokens"
    print(f"{name}: {len(st['pick'])} steps, {int((st['pick'] != st['teacher']).sum())} flips ({time.time() - t:.0f} s)",
          flush=True)
    np.savez(keep, **st)
    return st


def forced(st):
    """the steps of a recorded run that were teacher-forced (teacher >= 0), in order"""
    keep = st["teacher"] >= 0
    return {k: v[keep] for k, v in st.items()}


def main():
    names = ["v4/p0", "v3"]
    if "--realisations" in sys.argv:
        names = sys.argv[sys.argv.index("--realisations") + 1].split(",")
    for nm in names:  # every library variant must load (a stale build fails hours later otherwise)
        R.lib(R.VARIANTS[REALISATIONS[nm][0]])
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    pcm, name = workload(10)
    meta = json.load(open(os.path.join(OUT, name + ".json")))
    res = meta["results"]
    path = S.ensure_model("large-v3", SEED, cache)
    assert S.file_sha256(path) == meta["model_sha256"]
    # every window of the fixture is open (windows_open): its last step -- the one that ends the window --
    # is the decoder's own, unforced (teacher -1), and no later callback sees it; the GPU check compares the
    # forced steps (tests/parity_util.py StepForcer: len(window) per open window) and the run's final tokens
    base = forced(forced_steps("base", "v4", None, pcm, res, path, cache))
    assert (base["pick"] == base["teacher"]).all(), "the reference's own pick differs from its forced token"
    n = len(base["pick"])
    assert n == sum(len(w) for w in res["windows"]), (n, sum(len(w) for w in res["windows"]))
    rec = {"windows": res["windows"], "open_end": res["windows_open"], "n_steps": int(n), "eot": None,
           "realisations": {}, "fixture": name}
    arrays = {KEY + "/cand": base["cand"].astype(np.int32), KEY + "/cand_logit": base["cand_logit"],
              KEY + "/ts_margin": (base["ts_lse"] - base["text_max"]).astype(np.float32)}
    fl = np.zeros(n, np.float32)
    fl_ts = np.zeros(n, np.float32)
    for nm in names:
        var, seed = REALISATIONS[nm]
        st = forced(forced_steps(nm, var, seed, pcm, res, path, cache))
        assert len(st["pick"]) == n, f"{nm}: {len(st['pick'])} steps vs {n}"
        flips = [[int(i), int(st["pick"][i]), int(st["teacher"][i])] for i in np.nonzero(st["pick"] != st["teacher"])[0]]
        d, dts = floors(base, st)
        fl = np.maximum(fl, d)
        fl_ts = np.maximum(fl_ts, dts)
        rec["realisations"][nm] = {"flips": flips, "max_dlogit": float(d.max()) if n else 0.0}
    arrays[KEY + "/floor"] = fl
    arrays[KEY + "/floor_ts"] = fl_ts
    print(f"{KEY}: {n} steps in {len(res['windows'])} windows; flips "
          f"{ {k: len(v['flips']) for k, v in rec['realisations'].items()} }; floor median {np.median(fl):.2e} "
          f"max {fl.max():.2e}", flush=True)
    np.savez_compressed(os.path.join(OUT, "c4_10m_tf.npz"), **arrays)
    with open(os.path.join(OUT, "c4_10m_tf.json"), "w") as f:
        json.dump({"seed": SEED, "cases": {KEY: rec}}, f, indent=0)


if __name__ == "__main__":
    main()
