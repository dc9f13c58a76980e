"""Generate the quantized streaming-SortFormer fixtures (sfq_golden.json / sfq_golden.npz) by
running the REFERENCE implementation on the reference's own quantized GGUFs.

The synthetic F16 GGUF of make_golden_sf.py (sortformer_synth.py, SHA-256 pinned) is quantized by
the reference's streaming-sortformer/tools/quantize.cpp, compiled from its sources into
oracle/_ref/sortformer-quantize (oracle/ref/Makefile), to each type that tool writes
(quantize.cpp:101-107: q8_0, q4_k, q5_k; its tensor rule quantize.cpp:16-90). The reference
streaming-sortformer + ggml CPU path (oracle/_ref/libsortformer_ref.so) then runs on each file:
ggml_mul_mat rounds every f32 activation row to the weight's vec_dot_type (Q8_0 / Q8_K) and takes
the block dots. Recorded per type: the layer-0 conformer and the whole 17-layer stack of the staged
API on the 15 s golden pre-encoder input, offline diarization of the first 60 s of test.wav, and
the 2 s streaming preset in 8000-sample blocks -- each with the reference's own noise floor (the
same run on input perturbed by 1e-7 relative noise), since Q8 activation rounding turns ulp-level
differences into whole quantization steps.

Usage (in a container that has /root/reference):  python tests/golden/make_golden_sfq.py
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import sortformer as SF  # noqa: E402
import sortformer_synth as SS  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(ROOT, "oracle", "_ref", "libsortformer_ref.so")
QUANT = os.path.join(ROOT, "oracle", "_ref", "sortformer-quantize")
SEED = 4321
KINDS = ("q8_0", "q4_k", "q5_k")


def quantized_model(kind, cache):
    """(path, sha256) of the reference quantizer's output for the synthetic GGUF"""
    src = os.path.join(cache, f"synth-sortformer-s{SEED}.gguf")
    SS.write_model(src, SEED)
    dst = os.path.join(cache, f"synth-sortformer-s{SEED}-{kind}.gguf")
    subprocess.run([QUANT, src, dst, kind], check=True, capture_output=True)
    return dst, S.file_sha256(dst)


def perturbed(x):
    rng = np.random.default_rng(0)
    return (x * (1 + 1e-7 * rng.standard_normal(x.size).reshape(x.shape))).astype(np.float32)


def main():
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    f16 = json.load(open(os.path.join(OUT, "sf_golden.json")))
    f16a = np.load(os.path.join(OUT, "sf_golden.npz"))
    assert f16["seed"] == SEED
    test60 = S.read_wav_16k_mono(os.path.join(OUT, "sf_test60.wav"))
    pre = f16a["stage/preenc"]
    meta = {"seed": SEED, "models": {}, "results": {}}
    arrays = {}
    for kind in KINDS:
        path, sha = quantized_model(kind, cache)
        meta["models"][kind] = {"sha256": sha}
        sf = SF.Sortformer(path, lib=REF, n_threads=8)

        def record(key, fn, x):
            got = fn(x)
            arrays[key] = got
            d = np.abs(fn(perturbed(x)).astype(np.float64) - got)
            meta["results"]["noise_floor/" + key] = {"max": float(d.max()), "mean": float(d.mean())}
            print(f"{key}: shape {got.shape} floor max {d.max():.3e} mean {d.mean():.3e}", flush=True)

        record(f"{kind}/conf0", lambda x: sf.conformer(x, 0), pre)
        record(f"{kind}/conf16", lambda x: sf.conformer(x, 16), pre)
        record(f"{kind}/trans17", lambda x: sf.transformer(x, 17), f16a["stage/proj"])
        record(f"{kind}/diarize/test60", sf.diarize, test60)

        def stream(x):
            st = sf.stream("2s")
            outs, pos = [], 0
            while pos < len(x):
                outs.append(st.feed(x[pos:pos + 8000]))
                pos += 8000
            outs.append(st.flush())
            st.close()
            return np.concatenate(outs, 0)
        record(f"{kind}/stream/2s_blocks8000", stream, test60)
        meta["results"][f"rttm/{kind}/test60"] = SF.to_rttm(arrays[f"{kind}/diarize/test60"], 0.5, 11, "/x/test60.wav",
                                                            lib=REF)
        sf.close()
    np.savez_compressed(os.path.join(OUT, "sfq_golden.npz"), **arrays)
    with open(os.path.join(OUT, "sfq_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
