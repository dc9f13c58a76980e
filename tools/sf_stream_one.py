"""One SortFormer stream fed in fixed blocks (the configs[4] sequential diarizer: the "2s" preset,
2 s blocks): wall time per block and for the whole clip. Prints one JSON line.

    python tools/sf_stream_one.py [--minutes 10] [--preset 2s] [--block 32000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import sortformer as SF  # noqa: E402
import sortformer_synth as SS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--preset", default="2s")
    ap.add_argument("--block", type=int, default=32000)
    args = ap.parse_args()
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "sf_golden.json")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
    if not os.path.exists(path):
        assert SS.write_model(path, meta["seed"]) == meta["sha256"]
    n = int(args.minutes * 60 * 16000)
    pcm = S.synth_audio(n, 5)
    sf = SF.Sortformer(path)
    warm = sf.stream(args.preset)
    for i in range(0, min(n, 20 * args.block), args.block):
        warm.feed(pcm[i:i + args.block])
    warm.close()
    st = sf.stream(args.preset)
    times, frames = [], 0
    t0 = time.perf_counter()
    for i in range(0, n, args.block):
        t1 = time.perf_counter()
        frames += len(st.feed(pcm[i:i + args.block]))
        times.append(time.perf_counter() - t1)
    frames += len(st.flush())
    wall = time.perf_counter() - t0
    st.close()
    sf.close()
    times.sort()
    print(json.dumps({"metric": "SortFormer streaming wall time", "preset": args.preset, "block_samples": args.block,
                      "audio_s": n / 16000, "wall_s": round(wall, 4), "rtf": round(n / 16000 / wall, 2),
                      "blocks": len(times), "frames": frames,
                      "block_ms_median": round(1e3 * times[len(times) // 2], 3),
                      "block_ms_max": round(1e3 * times[-1], 3)}))


if __name__ == "__main__":
    main()
