"""Fills the recorded-logit (stochastic) fixtures make_golden.py and make_golden_cli_default.py left out,
produced by the REFERENCE (oracle/_ref/libwhisper_ref.so) and added to golden.json / golden.npz:

  * greedy_fallback and sampled (best_of 5 at t = 0.4) on synth30 for base.en and l3-mini -- the
    128-mel / 51,866-vocab shape with language tokens (make_golden.py:109 skipped them);
  * whisper-cli's literal defaults (beam 5 -> sampled best-of-5 ladder, make_golden_cli_default.py) on the
    multilingual tiny and l3-mini, both clips, language "en" (so the prompt carries <|en|><|transcribe|>).

Same recording as the originals (ref_probe.cpp ref_record_cb truncates each decoder's logits at the
logits_filter_callback point to a recorded top set; tests/golden/recording.py Injector substitutes them on
the GPU), so RNG streams, candidate sorting, KV-cell reordering, the fallback decisions and the best-of choice
are compared bit for bit by tests/test_gpu_parity.py::test_whisper_full. Entries already present are kept.

Usage (container with /root/reference):  python tests/golden/make_golden_fill.py
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
from make_golden import CONFIGS, SEED, clips  # noqa: E402
from make_golden_cli_default import CLI_DEFAULT, attempts  # noqa: E402
from recording import prefix_hash  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
NT = int(os.environ.get("REF_THREADS", "4"))
FILL = [("base.en", "synth30", "greedy_fallback"), ("base.en", "synth30", "sampled"),
        ("l3-mini", "synth30", "greedy_fallback"), ("l3-mini", "synth30", "sampled")]
FILL += [(m, c, "cli_default") for m in ("tiny", "l3-mini") for c in ("jfk", "synth30")]


def main():
    meta = json.load(open(os.path.join(OUT, "golden.json")))
    arrays = dict(np.load(os.path.join(OUT, "golden.npz")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    audio = clips()
    refs = {}
    for model, cname, cfg_name in FILL:
        key = f"{model}/{cname}/full/{cfg_name}"
        if key in meta["results"]:
            continue
        if model not in refs:
            path = os.path.join(cache, f"synth-{model}-s{SEED}.bin")
            if not os.path.exists(path):
                S.write_model(path, model, SEED)
            assert S.file_sha256(path) == meta["models"][model]["sha256"]
            refs[model] = R.Ref(path)
        ref = refs[model]
        cfg = CLI_DEFAULT if cfg_name == "cli_default" else CONFIGS[cfg_name]
        t = time.time()
        ret, segs = ref.full(audio[cname], language="en", record_topk=True, n_threads=NT, **cfg)
        off, prefix, idx, val = ref.recorded()
        rec = {"ret": ret, "segments": segs}
        if cfg_name == "cli_default":
            rec.update(attempts=attempts(off, prefix), params=CLI_DEFAULT)
        meta["results"][key] = rec
        arrays[key + "/rec_hash"] = np.array([prefix_hash(prefix[off[i]:off[i + 1]]) for i in range(len(off) - 1)],
                                             np.uint64)
        arrays[key + "/rec_idx"] = np.where(idx < 0, 65535, idx).astype(np.uint16)
        arrays[key + "/rec_val"] = val
        print(f"{key}: ret {ret}, {len(segs)} segments, {sum(len(s['tokens']) for s in segs)} tokens, "
              f"{len(off) - 1} decoder calls, {attempts(off, prefix)} attempts ({time.time() - t:.0f} s)", flush=True)
        np.savez_compressed(os.path.join(OUT, "golden.npz"), **arrays)
        with open(os.path.join(OUT, "golden.json"), "w") as f:
            json.dump(meta, f, indent=0)
    for r in refs.values():
        r.close()


if __name__ == "__main__":
    main()
