"""The reference's own t_dtw noise floor for the configs[4] fixture (c4_golden.json, written by
make_golden_c4.py): the same whisper_full (synthetic large-v3 F16, flash_attn = false, DTW with the
LARGE_V3 alignment heads, 60 s, sequential windows) by the REFERENCE on the audio perturbed by 1e-7
relative noise. DTW picks a path through the alignment heads' attention by strict comparisons
(ref src/whisper.cpp:8837-8998); on near-uniform synthetic attention the path has near-ties, so an
attention difference far below any parity bar moves some tokens' t_dtw by a frame or two. Recorded
under results/"tdtw_floor": the tokens compared (the identical-token prefix of the two runs), how
many t_dtw differ and by how much -- tests/test_gpu_c4.py bounds the GPU's differences by it.

Usage (container with /root/reference; ~15 min per seed on 8 cores, ~55 min at 10 minutes):
    python tests/golden/make_golden_c4_floor.py [--minutes 10] [--forced] [seed ...]      (default: seed 0)
(--minutes 10: the 10-minute fixture c4_10m_golden.json of make_golden_c4.py --minutes 10; the perturbed run
is cached under OWK_MODEL_CACHE, so it may run beside make_golden_c4.py and be compared afterwards)
Seed 0 writes results/"tdtw_floor"; every seed's summary goes to results/"tdtw_floor_seeds" (the
union of decisions a 1e-7 perturbation flips).
--forced: the perturbed reference teacher-forced onto the fixture's traced windows (ref_oracle tf_set, open
window ends left to it), so its tokens stay the fixture's over the whole clip -- the free perturbed run at
10 minutes parts from the unperturbed one at token 1783 of 14 312 and compares t_dtw only before that.
Written to results/"tdtw_floor_tf_seeds"; test_gpu_c4's teacher-forced DTW check reads it beside the free seeds.
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

MINUTES = int(sys.argv[sys.argv.index("--minutes") + 1]) if "--minutes" in sys.argv else 1
FORCED = "--forced" in sys.argv
# --lib v3|v1: the reference built for another x86 SIMD level (oracle/ref/Makefile variants), its input
# unperturbed -- another summation order of the same ggml path (recorded with seed "v3" / "v1")
LIB = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else None


def perturbed_run(seed, name):
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    path = S.ensure_model("large-v3", SEED, cache)
    keep = os.path.join(cache, f"{name}_floor{'_tf' if FORCED else ''}_seed{seed}-{S.file_sha256(path)[:16]}.json")
    if LIB:
        keep = os.path.join(cache, f"{name}_floor{'_tf' if FORCED else ''}_{LIB}-{S.file_sha256(path)[:16]}.json")
    if os.path.exists(keep):
        return json.load(open(keep))["segments"]
    pcm, _ = workload(MINUTES)
    rng = np.random.default_rng(seed)
    pp = pcm if LIB else (pcm * (1 + 1e-7 * rng.standard_normal(len(pcm)))).astype(np.float32)
    ref = R.Ref(path, lib_path=R.VARIANTS[LIB] if LIB else None, flash_attn=False, dtw_preset=AHEADS_LARGE_V3)
    if FORCED:
        res = json.load(open(os.path.join(OUT, name + ".json")))["results"]
        ref.tf_set(res["windows"], force=True, open_end=res["windows_open"])
    t = time.time()
    ret, segs = ref.full(pp, n_threads=NT, **PARAMS)
    ref.close()
    print("perturbed whisper_full", ret, f"{time.time() - t:.0f} s", flush=True)
    with open(keep, "w") as f:
        json.dump({"ret": ret, "segments": segs}, f)
    return segs


def run(seed):
    _, name = workload(MINUTES)
    segs = perturbed_run(seed, name)
    meta = json.load(open(os.path.join(OUT, name + ".json")))
    want = [tk for s in meta["results"]["full"]["segments"] for tk in s["tokens"]]
    got = [tk for s in segs for tk in s["tokens"]]
    n = 0
    while n < min(len(want), len(got)) and want[n][0] == got[n][0]:
        n += 1
    diffs = [(i, int(got[i][8]), int(want[i][8])) for i in range(n) if got[i][8] != want[i][8]]
    shift = max((abs(a - b) for _, a, b in diffs), default=0)
    rec = {"seed": LIB or seed, "compared": n, "n_tokens": len(want), "n_diff": len(diffs), "max_shift": shift,
           "diffs": diffs[:2000]}
    print(f"seed {seed}: identical tokens {n} of {len(want)}; t_dtw differs on {len(diffs)} (max shift {shift} cs)",
          flush=True)
    return rec


def main():
    args = [a for a in sys.argv[1:] if a != "--forced"]
    for opt in ("--minutes", "--lib"):
        if opt in args:
            i = args.index(opt)
            args = args[:i] + args[i + 2:]
    seeds = [int(a) for a in args] or [0]
    if LIB:
        seeds = seeds[:1]
    recs = [run(sd) for sd in seeds]
    path_json = os.path.join(OUT, workload(MINUTES)[1] + ".json")
    meta = json.load(open(path_json))  # re-read: several of these may run side by side
    key = "tdtw_floor_tf_seeds" if FORCED else "tdtw_floor_seeds"
    for rec in recs:
        if rec["seed"] == 0 and not FORCED:
            meta["results"]["tdtw_floor"] = {k: v for k, v in rec.items() if k != "seed"}
        seeds_l = [x for x in meta["results"].get(key, []) if x["seed"] != rec["seed"]]
        meta["results"][key] = sorted(seeds_l + [rec], key=lambda x: str(x["seed"]))
    with open(path_json, "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
