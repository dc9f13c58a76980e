"""Teacher-forced decisions of the REFERENCE at every decode step, and the reference's own per-step noise
floor (tf_golden.json / tf_golden.npz), for the greedy whisper_full fixtures whose GPU free run may part
from the reference at a near-tie (tests/parity_util.py).

A free-run comparison stops at the first step where the two runs pick different tokens: after it, the
prefixes differ and nothing later is comparable. The fixtures here let a GPU test compare EVERY step: the
GPU run is teacher-forced onto the reference's decoded tokens (tests/parity_util.decision_check), and its
own greedy pick at each step -- on exactly the reference's prefix -- must be the reference's token. A step
where they differ is accepted only if the reference itself does not decide it: it flips that step in one
of its own realisations below, or its gap between the two tokens is within 2x the largest movement of
those logits across its realisations at that step (the per-step form of the Q5_0 test's floor).

Per case (oracle/ref/ref_probe.cpp ref_tf_set / ref_tf_get; oracle/ref_oracle.py Ref.tf_*):
  1. the golden configuration once more with every step recorded, nothing forced: the per-window decoded
     token lists (each step's pick; a window ends on <|endoftext|>, at the 220-step limit or on a
     timestamp reaching the end of the audio) -- asserted to give the fixture's own result tokens;
  2. the same run teacher-forced onto those lists: at every step the reference's own pick (its
     whisper_process_logits + whisper_sample_token on a copy of the decoder, whisper.cpp:6177-6445,
     6460-6592) must equal the forced token -- the mechanism checks itself; this run's per-step
     candidates (16 largest text / EOT logits at the callback point) and the timestamp rule's two sides
     (timestamp log-mass, best text logit) are the base values;
  3. REALISATIONS: the reference's own ggml CPU path built for x86-64-v3 (AVX2 + F16C + FMA) and for
     baseline x86-64 (SSE; oracle/ref/Makefile `variants`), whose SIMD kernels sum in other orders --
     the same library on another x86 host --, and the AVX-512 build on the input perturbed by 1e-7
     relative noise; each teacher-forced onto the same lists: the steps it flips and, per step, the
     largest |logit - base| over the base candidates it also ranks, and of the timestamp rule's margin.

Usage (container with /root/reference, after make -C oracle/ref all variants):
    python tests/golden/make_golden_tf.py            small models (golden.json + nofa_golden.json cases)
    python tests/golden/make_golden_tf.py large      large-v3 / large-v3-turbo (large_golden.json cases)
    python tests/golden/make_golden_tf.py params     the SDK / CLI parameter cases (params_golden.json; whisper_full
                                                      through ref_full_ext with the case's own parameters)
Cases already in tf_golden.json are kept (delete an entry to regenerate it).
"""
import ctypes as C
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
NT = int(os.environ.get("REF_THREADS", "4"))
NC = R.Ref.TF_NC
MODELS = ["tiny.en", "base.en", "tiny", "l3-mini"]
NOFA_DTW = {"tiny.en": (3, -1), "tiny": (4, -1), "l3-mini": (1, 1)}  # make_golden_nofa.py
LARGE_DTW = {"large-v3": 13, "large-v3-turbo": 14}
CFG = {"greedy": dict(temperature_inc=0.0),
       "fixed_work": dict(no_timestamps=True, max_tokens=40, suppress_eot=True, temperature_inc=0.0),
       "token_ts": dict(temperature_inc=0.0, token_timestamps=True)}
LARGE_CFG = {"greedy": dict(temperature_inc=0.0),
             "fixed_work": dict(no_timestamps=True, max_tokens=219, suppress_eot=True, temperature_inc=0.0)}


def clips():
    return {"jfk": S.read_wav_16k_mono(os.path.join(OUT, "jfk.wav")), "synth30": S.synth_audio(480000, 7),
            "test60": S.read_wav_16k_mono(os.path.join(OUT, "sf_test60.wav"))}


def params_ext(c):
    """ref_full_ext fields of a params_golden.json case (bytes fields stored as hex)"""
    return {k: (bytes.fromhex(v) if k in c["bytes_fields"] else v) for k, v in c["ext"].items()}


def cases(which):
    """(key, model, clip, ref init kwargs, ref.full kwargs, fixture (file, result key))"""
    out = []
    if which == "small":
        for model in MODELS:
            for clip in ("jfk", "synth30"):
                for cfg, kw in CFG.items():
                    k = f"{model}/{clip}/full/{cfg}"
                    out.append((k, model, clip, {}, dict(language="en", **kw), ("golden.json", k)))
            if model in ("tiny", "l3-mini"):
                k = f"{model}/jfk/full/auto_lang"
                out.append((k, model, "jfk", {}, dict(language="auto", temperature_inc=0.0), ("golden.json", k)))
        for model, (preset, n_top) in NOFA_DTW.items():
            for clip in ("jfk", "synth30"):
                k = f"{model}/{clip}/full/greedy_dtw"
                out.append(("nofa/" + k, model, clip, dict(flash_attn=False, dtw_preset=preset, dtw_n_top=n_top),
                            dict(language="en", temperature_inc=0.0, no_timestamps=clip == "synth30"),
                            ("nofa_golden.json", k)))
    elif which == "params":
        pg = json.load(open(os.path.join(OUT, "params_golden.json")))
        for name, c in sorted(pg["cases"].items()):
            out.append(("params/" + name, c["model"], c["clip"], {}, dict(c["params"]), ("params_golden.json", name)))
    else:
        for model in ("large-v3", "large-v3-turbo"):
            for clip in ("jfk", "synth30"):
                for cfg, kw in LARGE_CFG.items():
                    k = f"{model}/{clip}/full/{cfg}"
                    out.append(("large/" + k, model, clip, {}, dict(language="en", **kw), ("large_golden.json", k)))
                k = f"{model}/{clip}/full/greedy_dtw"
                out.append(("large/" + k, model, clip, dict(flash_attn=False, dtw_preset=LARGE_DTW[model]),
                            None, ("large_golden.json", k)))
    return out


def realisations(which):
    """(name, library variant, perturbation seed or None)"""
    r = [("v4/p0", "v4", 0), ("v4/p1", "v4", 1), ("v3", "v3", None), ("v3/p0", "v3", 0)]
    if which in ("small", "params"):
        r.append(("v1", "v1", None))
    return r


def windows_of(steps, eot):
    """per-window decoded token lists from a recorded run: each window's picks in step order; a window
    ending on <|endoftext|> lists the tokens before it (the EOT step is forced as the step after them)"""
    wins = {}
    for w, k, p in zip(steps["window"], steps["step"], steps["pick"]):
        wins.setdefault(int(w), []).append((int(k), int(p)))
    out, open_end = [], []
    for w in range(len(wins)):
        ks = [k for k, _ in wins[w]]
        assert ks == list(range(len(ks))), f"window {w}: steps {ks[:8]}... (one decoder, one call per step)"
        picks = [p for _, p in wins[w]]
        if picks[-1] == eot:
            out.append(picks[:-1])
            open_end.append(False)
        else:
            out.append(picks)
            open_end.append(True)
    return out, open_end


def floors(base, steps):
    """per step: largest |logit - base| over the base candidates this realisation also ranks, and the
    movement of the timestamp rule's margin (ts log-mass - best text logit)"""
    n = len(base["pick"])
    d = np.zeros(n, np.float32)
    dts = np.zeros(n, np.float32)
    for i in range(n):
        m = {int(c): float(v) for c, v in zip(steps["cand"][i], steps["cand_logit"][i]) if c >= 0}
        dd = [abs(m[int(c)] - float(v)) for c, v in zip(base["cand"][i], base["cand_logit"][i]) if c >= 0 and int(c) in m]
        d[i] = max(dd) if dd else 0.0
        a = float(base["ts_lse"][i]) - float(base["text_max"][i])
        b = float(steps["ts_lse"][i]) - float(steps["text_max"][i])
        dts[i] = abs(a - b) if np.isfinite(a) and np.isfinite(b) else 0.0
    return d, dts


def run_case(key, model, clip, init_kw, full_kw, fixture, which, audio, cache, fixtures):
    meta = fixtures[fixture[0]]
    want = meta["results"][fixture[1]] if fixture[0] != "params_golden.json" else meta["cases"][fixture[1]]
    ext = params_ext(want) if fixture[0] == "params_golden.json" else None
    if full_kw is None:  # large DTW fixture: its own no_timestamps flag
        full_kw = dict(language="en", temperature_inc=0.0, no_timestamps=want["no_timestamps"])
    if model in MODELS:
        path = os.path.join(cache, f"synth-{model}-s{SEED}.bin")
        if not os.path.exists(path):
            S.write_model(path, model, SEED)
    else:
        path = S.ensure_model(model, SEED, cache)
    pcm = audio[clip]
    kw = dict(n_threads=NT, **full_kw)

    def full(r, x):
        return r.full(x, **kw) if ext is None else r.full_ex(x, ext, **kw)[:2]
    t0 = time.time()
    ref = R.Ref(path, **init_kw)
    ref.L.whisper_token_eot.argtypes = [C.c_void_p]
    eot = ref.L.whisper_token_eot(ref.ctx)
    ref.tf_set([], force=False)
    ret, segs = full(ref, pcm)
    assert ret == want["ret"]
    flat = [t[0] for s in segs for t in s["tokens"]]
    assert flat == [t[0] for s in want["segments"] for t in s["tokens"]], f"{key}: the recorded run is not the fixture's"
    windows, open_end = windows_of(ref.tf_steps(), eot)
    ref.tf_set(None)
    ref.close()  # a fresh context: no_context = false carries a state's prompt history into its next call
    ref = R.Ref(path, **init_kw)
    ref.tf_set(windows, force=True)
    ret, segs = full(ref, pcm)
    base = ref.tf_steps()
    assert [t[0] for s in segs for t in s["tokens"]] == flat, f"{key}: teacher-forced run left the tokens"
    assert (base["pick"] == base["teacher"]).all(), f"{key}: the reference's own pick differs from its forced token"
    ref.tf_set(None)
    ref.close()
    rec = {"windows": windows, "open_end": open_end, "n_steps": int(len(base["pick"])), "eot": int(eot),
           "realisations": {}}
    arrays = {key + "/cand": base["cand"].astype(np.int32), key + "/cand_logit": base["cand_logit"],
              key + "/ts_margin": (base["ts_lse"] - base["text_max"]).astype(np.float32)}
    fl = np.zeros(len(base["pick"]), np.float32)
    fl_ts = np.zeros(len(base["pick"]), np.float32)
    for name, var, seed in realisations(which):
        x = pcm if seed is None else (pcm * (1 + 1e-7 * np.random.default_rng(seed).standard_normal(len(pcm)))).astype(np.float32)
        r = R.Ref(path, lib_path=R.VARIANTS[var], **init_kw)
        r.tf_set(windows, force=True)
        full(r, x)
        st = r.tf_steps()
        r.tf_set(None)
        r.close()
        assert len(st["pick"]) == len(base["pick"]), f"{key}/{name}: {len(st['pick'])} steps vs {len(base['pick'])}"
        flips = [[int(i), int(st["pick"][i]), int(st["teacher"][i])] for i in np.nonzero(st["pick"] != st["teacher"])[0]]
        d, dts = floors(base, st)
        fl = np.maximum(fl, d)
        fl_ts = np.maximum(fl_ts, dts)
        rec["realisations"][name] = {"flips": flips, "max_dlogit": float(d[np.isfinite(d)].max()) if np.isfinite(d).any() else 0.0}
    arrays[key + "/floor"] = fl
    arrays[key + "/floor_ts"] = fl_ts
    print(f"{key}: {rec['n_steps']} steps in {len(windows)} windows; flips "
          f"{ {n: len(v['flips']) for n, v in rec['realisations'].items()} }; floor median "
          f"{np.median(fl) if len(fl) else 0:.2e} max {fl.max() if len(fl) else 0:.2e} ({time.time() - t0:.0f} s)",
          flush=True)
    return rec, arrays


def main():
    which = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] in ("large", "params") else "small"
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    path_json, path_npz = os.path.join(OUT, "tf_golden.json"), os.path.join(OUT, "tf_golden.npz")
    meta = json.load(open(path_json)) if os.path.exists(path_json) else {"seed": SEED, "cases": {}}
    arrays = dict(np.load(path_npz)) if os.path.exists(path_npz) else {}
    fixtures = {f: json.load(open(os.path.join(OUT, f)))
                for f in ("golden.json", "nofa_golden.json", "large_golden.json", "params_golden.json")}
    audio = clips()
    only = sys.argv[2:] if len(sys.argv) > 2 else None
    for _, var, _ in realisations(which):  # every library variant must load (a stale build fails late otherwise)
        R.lib(R.VARIANTS[var])
    for c in cases(which):
        if c[0] in meta["cases"] or (only and not any(c[0] == o or c[0].endswith("/" + o) for o in only)):
            continue
        rec, arr = run_case(*c, which, audio, cache, fixtures)
        meta["cases"][c[0]] = rec
        arrays.update(arr)
        np.savez_compressed(path_npz, **arrays)
        with open(path_json, "w") as f:
            json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
