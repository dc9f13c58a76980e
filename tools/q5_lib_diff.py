"""Digest of one greedy whisper_full on synthetic large-v3-q5_0 (2 clips of 30 s, one owk_full_batch call):
every token's id and f32 p / plog, hashed -- run once per library build (OWK_LIB) to tell a bit-identical
kernel change from one that moves the activations.

    OWK_LIB=... python tools/q5_lib_diff.py [--model large-v3-q5_0]
"""
import argparse
import hashlib
import json
import os
import struct
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk  # noqa: E402
import owk_synth as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="large-v3-q5_0")
    a = ap.parse_args()
    model = S.ensure_model(a.model, cache_dir=os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models"))
    owk.quiet()
    w = owk.Whisper(model, flash_attn=True)
    p = w.params(0, language="en", temperature_inc=0.0, no_context=True)
    pcms = [S.synth_audio(480000, 11 + i) for i in range(2)]
    sts = [w.new_state() for _ in pcms]
    ret = w.full_batch(sts, pcms, p)
    h = hashlib.sha256()
    n = 0
    for st in sts:
        for seg in w.segments(st):
            for t in seg["tokens"]:
                h.update(struct.pack("<iff", t[0], t[2], t[3]))
                n += 1
    print(json.dumps({"lib": os.environ.get("OWK_LIB", "in-tree"), "ret": ret, "tokens": n, "digest": h.hexdigest()[:16]}))


if __name__ == "__main__":
    main()
