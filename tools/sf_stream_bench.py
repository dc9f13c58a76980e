"""Many live SortFormer streams on one MI355X.

N streams of the 2 s preset, each fed the same wall-clock sequence of 2 s blocks of its own
seeded synthetic audio (synthetic-weight GGUF of tests/golden/make_golden_sf.py):
  sequential : sortformer_stream_feed per stream per block (the reference API, one GPU head
               pass per chunk)
  batched    : owk_sortformer_stream_feed_batch per block round (one head pass over all
               streams' stacked rows)
Reports aggregate real-time factor (audio seconds of all streams / wall seconds) and the
worst per-round latency. Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import sortformer as SF  # noqa: E402
import sortformer_synth as SS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=30.0, help="audio per stream")
    ap.add_argument("--block", type=int, default=32000, help="samples per feed")
    ap.add_argument("--preset", default="2s")
    a = ap.parse_args()
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "sf_golden.json")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
    if not os.path.exists(path):
        assert SS.write_model(path, meta["seed"]) == meta["sha256"]
    sf = SF.Sortformer(path)
    n = int(a.seconds * 16000)
    pcms = [S.synth_audio(n, 50 + i).astype(np.float32) for i in range(a.streams)]
    n_rounds = (n + a.block - 1) // a.block
    res = {"metric": "SortFormer streaming real-time factor, all streams (audio-s/wall-s)", "streams": a.streams,
           "stream_seconds": a.seconds, "block_samples": a.block, "preset": a.preset,
           "data": "synthetic weights (real shapes) and seeded synthetic audio"}
    for mode in ("sequential", "batched"):
        for rep in range(2):  # first repetition warms up allocations
            sts = [sf.stream(a.preset) for _ in range(a.streams)]
            frames = 0
            worst = 0.0
            t0 = time.perf_counter()
            for r in range(n_rounds):
                blk = [p[r * a.block:(r + 1) * a.block] for p in pcms]
                tr = time.perf_counter()
                if mode == "sequential":
                    outs = [st.feed(b) for st, b in zip(sts, blk)]
                else:
                    outs = SF.feed_batch(sts, blk)
                worst = max(worst, time.perf_counter() - tr)
                frames += sum(o.shape[0] for o in outs)
            t = time.perf_counter() - t0
            for st in sts:
                st.close()
        res[mode] = {"wall_s": round(t, 4), "rtf": round(a.streams * a.seconds / t, 1),
                     "worst_round_ms": round(1e3 * worst, 2), "frames": frames}
    res["speedup"] = round(res["sequential"]["wall_s"] / res["batched"]["wall_s"], 2)
    sf.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
