"""SortFormer diarization throughput on the MI355X (libsortformer.so) next to the reference
ggml CPU path (oracle/_ref/libsortformer_ref.so, bounded sample), SURVEY §8 row B / BASELINE
configs[4] (diarization of long audio).

Workload: the synthetic-weight GGUF of tests/golden/make_golden_sf.py (real tensor set and
shapes), a seeded synthetic 16 kHz clip of --minutes minutes, offline sortformer_diarize with
the default parameters (chunk 188 frames, speaker cache 188). Also times the low-latency
streaming preset fed in 0.5 s blocks. Prints one JSON line.

    python tools/sf_bench.py [--minutes 10] [--cpu-seconds 60]
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
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--cpu-seconds", type=float, default=60.0, help="audio seconds for the CPU reference sample")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "sf_golden.json")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
    if not os.path.exists(path):
        assert SS.write_model(path, meta["seed"]) == meta["sha256"]
    n = int(args.minutes * 60 * 16000)
    pcm = S.synth_audio(n, 3)
    sf = SF.Sortformer(path)
    sf.diarize(pcm[:16000 * 30])  # warm-up (code objects, buffers)
    ts = []
    for _ in range(args.reps):
        t = time.perf_counter()
        probs = sf.diarize(pcm)
        ts.append(time.perf_counter() - t)
    wall = min(ts)
    # streaming: low-latency preset, 0.5 s blocks
    st = sf.stream("low")
    blk = 8000
    t = time.perf_counter()
    frames = 0
    for i in range(0, min(n, 16000 * 120), blk):
        frames += st.feed(pcm[i:i + blk]).shape[0]
    frames += st.flush().shape[0]
    swall = time.perf_counter() - t
    st.close()
    sf.close()
    out = {"metric": "SortFormer diarization real-time factor (audio-s/wall-s)", "unit": "audio-s/wall-s",
           "value": round(n / 16000 / wall, 2), "frames": int(probs.shape[0]), "audio_s": n / 16000,
           "wall_s": round(wall, 4), "workload": "offline sortformer_diarize, default params, synthetic GGUF",
           "stream_low_latency": {"audio_s": min(n, 16000 * 120) / 16000, "wall_s": round(swall, 3),
                                  "rtf": round(min(n, 16000 * 120) / 16000 / swall, 2), "frames": frames,
                                  "block_s": blk / 16000}}
    ref = os.path.join(ROOT, "oracle", "_ref", "libsortformer_ref.so")
    if os.path.exists(ref) and args.cpu_seconds > 0:
        nt = len(os.sched_getaffinity(0))
        nt = min(nt, int(os.environ.get("OMP_NUM_THREADS", nt)))
        m = int(args.cpu_seconds * 16000)
        rsf = SF.Sortformer(path, lib=ref, n_threads=nt)
        t = time.perf_counter()
        rsf.diarize(pcm[:m])
        rw = time.perf_counter() - t
        rsf.close()
        out["cpu_baseline"] = {"value": round(m / 16000 / rw, 2), "unit": "audio-s/wall-s", "cores": nt,
                               "kind": "reference", "sample": f"first {args.cpu_seconds:.0f} s of the same clip"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
