"""Adds whisper_full_parallel + VAD fixtures to tests/golden/vad_golden.json: the REFERENCE's
whisper_full_parallel(params.vad = true, n_processors = 2) (ref src/whisper.cpp:7801-7929: the VAD
pre-pass of 7812-7824 over the whole clip, the processed audio split into 2 chunks decoded on their
own states, results merged with the chunk offsets, and the segment getters' mapping back to the
original timeline of 7947-8025) on the synthetic tiny.en model and the VAD fixture clips.

Usage (after make_golden_vad.py, in a container that has /root/reference):
    python tests/golden/make_golden_vad_parallel.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden_vad import OUT, SEED, VAD_MODEL, R, S, lib, vad_clips  # noqa: E402


def main():
    path_json = os.path.join(OUT, "vad_golden.json")
    meta = json.load(open(path_json))
    clips = vad_clips()
    L = lib()
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-tiny.en-s{SEED}.bin")
    assert S.write_model(path, "tiny.en", SEED) == meta["full_model_sha256"]
    for cname in ("jfk", "composite"):
        ref = R.Ref(path)
        L.ref_set_vad(VAD_MODEL.encode())
        ret, segs = ref.full(clips[cname], temperature_inc=0.0, n_processors=2)
        ref.close()
        # a second, recorded run (record_topk truncates the logits after recording them, which moves
        # timestamp probabilities, so the fixture's segments come from the plain run above): every
        # decoder call's prefix and top logits -- the two chunks' calls interleave in the shared
        # recorder, a prefix names its call -- so a parting can be shown to be a near-tie
        ref = R.Ref(path)
        ref.full(clips[cname], temperature_inc=0.0, n_processors=2, record_topk=4)
        off, prefix, ids, vals = ref.recorded()
        ref.close()
        calls = [{"prefix": prefix[off[i]:off[i + 1]].tolist(), "top": ids[i][:4].tolist(),
                  "val": [float(v) for v in vals[i][:4]]} for i in range(len(off) - 1)]
        meta["full"][f"{cname}/parallel2"] = {"ret": ret, "calls": calls, "segments": [
            {"t0": s["t0"], "t1": s["t1"], "tokens": [t[0] for t in s["tokens"]]} for s in segs]}
        print(cname, ret, len(segs), "segments", [(s["t0"], s["t1"]) for s in segs][:8])
    L.ref_set_vad(None)
    json.dump(meta, open(path_json, "w"), indent=1)


if __name__ == "__main__":
    main()
