"""Where a persistent decode-chain launch spends its time (csrc/k_chain.hip, debug stamps).

Runs whisper_full on full-depth large-v3 (flash_attn = false + DTW, configs[4]'s one-row steps) with the
chain's realtime stamps armed for one decoder layer (owk_debug_dec_chain_trace: eager launches), then prints
per chain launch and stage the times (us, from the launch's first block entry) at which blocks entered the
stage, had their weight DMA issued, saw the previous stage's hand-off, finished the LayerNorm prologue, the
MFMAs and published: median / max over the stage's items.

  python tools/chain_trace.py [--layer 10] [--clip jfk|synth30]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import owk  # noqa: E402
import owk_synth as S  # noqa: E402

NST, NTS = 4, 6
POINTS = ["entry", "weights", "handoff", "layernorm", "mfma", "published"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", type=int, default=10)
    ap.add_argument("--clip", default="jfk")
    args = ap.parse_args()
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "large_golden.json")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    path = S.ensure_model("large-v3", meta["seed"], cache)
    owk.quiet()
    w = owk.Whisper(path, flash_attn=False, dtw_preset=meta["dtw"]["large-v3"])
    L = w.L
    L.owk_debug_dec_chain_trace.argtypes = [C.c_int]
    L.owk_debug_dec_chain_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
    pcm = S.read_wav_16k_mono(os.path.join(ROOT, "tests", "golden", "jfk.wav")) if args.clip == "jfk" \
        else S.synth_audio(480000, 7)
    p = w.params(0, language="en", temperature_inc=0.0)
    st = w.new_state()
    assert w.full(st, pcm, p) == 0  # warm
    L.owk_debug_dec_chain_trace(args.layer)
    try:
        assert w.full(st, pcm, p) == 0
        n = 2 * 256 * NST * NTS
        buf = (C.c_ulonglong * n)()
        got = L.owk_debug_dec_chain_stamps(st, buf, n)
    finally:
        L.owk_debug_dec_chain_trace(-1)
    assert got == n, got
    ts = np.frombuffer(buf, dtype=np.uint64).reshape(2, 256, NST, NTS).astype(np.int64)
    out = {"layer": args.layer, "clip": args.clip, "chains": []}
    for ch, name in enumerate(["A (attn.out -> LN -> cross-Q)", "B (cross_attn.out -> LN -> mlp.0 -> mlp.2 -> LN -> QKV)"]):
        t = ts[ch]
        live = t[:, :, 0] > 0
        t0 = t[:, 0, 0][live[:, 0]].min()
        end = t[:, :, 5][live].max()
        print(f"chain {name}: launch span (first entry -> last publish) {(end - t0) / 100:.2f} us")
        rows = []
        for s in range(NST):
            m = live[:, s]
            if not m.any():
                continue
            rel = (t[m, s, :] - t0) / 100.0  # 100 MHz -> us
            med = np.median(rel, axis=0)
            mx = rel.max(axis=0)
            print(f"  stage {s}: {int(m.sum()):3d} items | " +
                  " | ".join(f"{POINTS[k]} {med[k]:6.2f}/{mx[k]:6.2f}" for k in range(NTS)))
            rows.append({"stage": s, "items": int(m.sum()), "median_us": [round(float(x), 2) for x in med],
                         "max_us": [round(float(x), 2) for x in mx]})
        out["chains"].append({"name": name, "span_us": round(float(end - t0) / 100, 2), "stages": rows})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
