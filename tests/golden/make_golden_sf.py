"""Generate the streaming-SortFormer golden fixtures (sf_golden.json / sf_golden.npz) by
running the REFERENCE implementation.

The reference streaming-sortformer/src/sortformer.cpp + its ggml CPU path is compiled from
/root/reference sources by oracle/ref/Makefile into oracle/_ref/libsortformer_ref.so and
driven through the sortformer.h C ABI (open-whisper-kit_amd/python/sortformer.py). Inputs
are deterministic: the synthetic-weight GGUF written by sortformer_synth.py (SHA-256
recorded so the GPU box regenerates the identical file), the first 60 s of the reference's
own streaming-sortformer/test.wav (sf_test60.wav, data) and seeded synthetic clips.

Usage (in a container that has /root/reference):  python tests/golden/make_golden_sf.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import sortformer as SF  # noqa: E402
import sortformer_synth as SS  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(ROOT, "oracle", "_ref", "libsortformer_ref.so")
SEED = 4321

# streaming feeds: (preset, block sizes in samples, cycled)
STREAMS = {
    "2s_blocks8000": ("2s", [8000]),
    "low_ragged": ("low", [3200, 7000, 160, 12345, 999]),
    "5s_blocks16000": ("5s", [16000]),
}


def clips():
    test60 = S.read_wav_16k_mono(os.path.join(OUT, "sf_test60.wav"))
    synth = S.synth_audio(16000 * 45, 11)
    return {"test60": test60, "synth45": synth}


def feed_all(st, pcm, blocks):
    outs, counts, pos, i = [], [], 0, 0
    while pos < len(pcm):
        n = min(blocks[i % len(blocks)], len(pcm) - pos)
        p = st.feed(pcm[pos:pos + n])
        outs.append(p)
        counts.append(int(p.shape[0]))
        pos += n
        i += 1
    fl = st.flush()
    outs.append(fl)
    counts.append(int(fl.shape[0]))
    return np.concatenate(outs, 0), counts


def main():
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-sortformer-s{SEED}.gguf")
    sha = SS.write_model(path, SEED)
    meta = {"seed": SEED, "sha256": sha, "results": {}}
    arrays = {}
    sf = SF.Sortformer(path, lib=REF, n_threads=8)
    audio = clips()

    # staged API on the first 15 s of test60 (one chunk's worth)
    pcm = audio["test60"][:16000 * 15]
    mel, seq = sf.mel(pcm)
    arrays["stage/mel"] = mel
    meta["results"]["stage/seq_len"] = seq
    pre = sf.preenc(mel, seq)
    arrays["stage/preenc"] = pre
    for L in (0, 16):
        arrays[f"stage/conf{L}"] = sf.conformer(pre, L)
    proj = sf.projection(arrays["stage/conf16"])
    arrays["stage/proj"] = proj
    for L in (0, 17):
        arrays[f"stage/trans{L}"] = sf.transformer(proj, L)
    arrays["stage/pred"] = sf.prediction(arrays["stage/trans17"])

    # The reference's own noise floor, per case: the same run on the clip perturbed by 1e-7
    # relative noise (below the f32 ulp of most samples). Re-associated f32 arithmetic cannot
    # be expected to land closer to the golden than this (the synthetic deep stack amplifies
    # ulp-level differences through 35 layers and the speaker-cache feedback);
    # tests/test_sortformer.py bounds the GPU error by it.
    def perturbed(x):
        rng = np.random.default_rng(0)
        return (x * (1 + 1e-7 * rng.standard_normal(len(x)))).astype(np.float32)

    def record(key, fn, x):
        got = fn(x)
        arrays[key] = got
        d = np.abs(fn(perturbed(x)).astype(np.float64) - got)
        meta["results"]["noise_floor/" + key] = {"max": float(d.max()), "mean": float(d.mean())}
        return got

    # offline diarization (default params) + RTTM
    for name, x in audio.items():
        probs = record(f"diarize/{name}", sf.diarize, x)
        meta["results"][f"rttm/{name}"] = SF.to_rttm(probs, 0.5, 11, f"/x/{name}.wav", lib=REF)
    # non-default offline params: FIFO + shorter chunks, more compressions
    sf2 = SF.Sortformer(path, lib=REF, n_threads=8, chunk_len=48, fifo_len=40, spkcache_update_period=64,
                        right_context=2, chunk_left_context=2)
    record("diarize_fifo/test60", sf2.diarize, audio["test60"])
    sf2.close()

    # streaming API
    for name, (preset, blocks) in STREAMS.items():
        def run(x, preset=preset, blocks=blocks, name=name):
            st = sf.stream(preset)
            probs, counts = feed_all(st, x, blocks)
            meta["results"].setdefault(f"stream_counts/{name}", counts)
            st.close()
            return probs
        record(f"stream/{name}", run, audio["test60"])

    sf.close()
    np.savez_compressed(os.path.join(OUT, "sf_golden.npz"), **arrays)
    with open(os.path.join(OUT, "sf_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(arrays), "arrays;", {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
