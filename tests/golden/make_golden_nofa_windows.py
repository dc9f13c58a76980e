"""Per-window decoded token sequences of the flash_attn = false + DTW fixtures of make_golden_nofa.py
(merged into nofa_golden.json as "<model>/<clip>/dtw_windows"): the reference's whisper_full is re-run
with every decoder call's token prefix traced (ref_probe record_topk = 2, logits untouched), so
tests/test_gpu_nofa.py can teacher-force the GPU decode onto exactly what the reference decoded
(segment assembly folds timestamp pairs, so the result tokens are not the decoded sequence).

Usage (after make_golden_nofa.py):  python tests/golden/make_golden_nofa_windows.py
"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import ref_oracle as R  # noqa: E402
from make_golden_large_floor import windows_of  # noqa: E402
from make_golden_nofa import DTW, SEED, clips  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    meta = json.load(open(os.path.join(OUT, "nofa_golden.json")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    audio = clips()
    for model, (preset, n_top) in DTW.items():
        ref = R.Ref(S.ensure_model(model, SEED, cache), flash_attn=False, dtw_preset=preset, dtw_n_top=n_top)
        for cname, pcm in audio.items():
            key = f"{model}/{cname}"
            want = meta["results"][key + "/full/greedy_dtw"]
            ret, segs = ref.full(pcm, language="en", temperature_inc=0.0, no_timestamps=want["no_timestamps"],
                                 record_topk=2)
            flat = [t[0] for s in want["segments"] for t in s["tokens"]]
            assert [t[0] for s in segs for t in s["tokens"]] == flat
            wins = windows_of(ref, flat)
            if wins is not None:
                meta["results"][key + "/dtw_windows"] = wins
            print(key, "dtw windows", None if wins is None else [len(w) for w in wins], flush=True)
        ref.close()
    with open(os.path.join(OUT, "nofa_golden.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
