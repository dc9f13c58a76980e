"""configs[4] golden fixture (c4_golden.json / c4_golden.npz): large-v3 transcription with DTW token
timestamps + streaming SortFormer diarization + the DiarizationAligner, at full large-v3 depth,
produced by the REFERENCE (oracle/_ref/libwhisper_ref.so and libsortformer_ref.so, compiled from
/root/reference sources by oracle/ref/Makefile).

Workload (BASELINE configs[4], restated on the 60 s of real speech the SortFormer fixtures use,
tests/golden/sf_test60.wav = the first 60 s of the reference's streaming-sortformer/test.wav):
  * ONE whisper_full over the 60 s (the sequential 30 s window loop with seek advance and prompt
    carry, ref src/whisper.cpp:7034-7769): synthetic large-v3 F16 (make_golden_large.py's model,
    same seed), flash_attn = false, dtw_token_timestamps with WHISPER_AHEADS_LARGE_V3
    (ref 394, 8837-8998), greedy, temperature_inc = 0, token_timestamps, no_context = false;
    recorded: segments with every token's (id, t0, t1, t_dtw, p), and the per-window DECODED
    token lists (decoder-call prefixes traced, logits untouched; traced_windows below)
    so a GPU run can be teacher-forced onto them;
  * sortformer_stream_feed in 2 s blocks with the "2s" preset, then flush (ref
    streaming-sortformer/src/sortformer.cpp:2776-3265): probabilities, per-feed frame counts, the
    RTTM (threshold 0.5, median 11) and the reference's own 1e-7-perturbation noise floor;
  * the aligner (Swift DiarizationAligner restated in oracle/diarize_align.py) over the reference's
    tokens (Swift WordTiming per token: token text, t0/100, t1/100, p; WhisperContext.swift:126-139)
    and the parsed reference RTTM: words with speakers and utterances.

Usage (container with /root/reference):
    python tests/golden/make_golden_c4.py              -> c4_golden.*      (60 s, ~15 min on 8 cores)
    python tests/golden/make_golden_c4.py --minutes 10 -> c4_10m_golden.*  (round 5: the 10 minutes BASELINE
        configs[4] states, on tools/pipeline_bench.py's own clip owk_synth.synth_audio(600 s, seed 5); about
        20 windows with prompt carry and the AOSC speaker cache well past its first minute)
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import diarize_align as DA  # noqa: E402
import owk_synth as S  # noqa: E402
import ref_oracle as R  # noqa: E402
import sortformer as SF  # noqa: E402
import sortformer_synth as SS  # noqa: E402
from make_golden_large import SEED  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF_SF = os.path.join(ROOT, "oracle", "_ref", "libsortformer_ref.so")
AHEADS_LARGE_V3 = 13
BLOCK = 32000  # 2 s feeds
NT = int(os.environ.get("REF_THREADS", "8"))
PARAMS = dict(language="en", temperature_inc=0.0, token_timestamps=True, no_context=False)


def stream_run(sf, pcm):
    st = sf.stream("2s")
    outs, counts = [], []
    for i in range(0, len(pcm), BLOCK):
        p = st.feed(pcm[i:i + BLOCK])
        outs.append(p)
        counts.append(int(p.shape[0]))
    fl = st.flush()
    outs.append(fl)
    counts.append(int(fl.shape[0]))
    st.close()
    return np.concatenate(outs, 0), counts


def traced_windows(ref, flat):
    """Per-window decoded token prefixes from the traced decoder calls (a window starts where the
    traced prefix is empty again) and, per window, whether its end is OPEN: a window whose longest
    traced prefix is n_max - 1 = 219 tokens stopped at the n_text_ctx/2 - 4 step limit (ref
    whisper.cpp:7219), so its last sampled token follows no traced call. A teacher-forced run
    forces the prefix and leaves that last step to the decoder (tests/parity_util.Forcer); every
    other window ended on <|endoftext|> right after its longest prefix."""
    off, prefix, _, _ = ref.recorded()
    longest = []
    for i in range(len(off) - 1):
        p = prefix[off[i]:off[i + 1]].tolist()
        if not p:
            longest.append([])
        elif len(p) > len(longest[-1]):
            longest[-1] = p
    open_end = [len(w) + 1 >= 220 for w in longest]
    # the last window may also end on a kept token that follows no call: a timestamp reaching the
    # end of the audio (ref 7359-7441) -- the last result token, appended; that window's end is open too
    # (no <|endoftext|> step: its last token is the decoder's, read back from the result)
    if flat and not open_end[-1] and (not longest[-1] or longest[-1][-1] != flat[-1]):
        longest[-1].append(flat[-1])
        open_end[-1] = True
    return longest, open_end


def words_of(L, ctx, segs):
    """Swift WordTiming per token (WhisperContext.swift:126-139): text, t0 / 100, t1 / 100, p."""
    out = []
    for s in segs:
        for t in s["tokens"]:
            txt = L.whisper_token_to_str(ctx, t[0]).decode("utf-8", "replace")
            out.append((txt, float(np.float32(t[6]) / np.float32(100.0)), float(np.float32(t[7]) / np.float32(100.0)),
                        float(t[2])))
    return out


def workload(minutes):
    """(audio, fixture name) of a configs[4] fixture: the 60 s of real speech, or the bench's synthetic clip"""
    if minutes == 1:
        return S.read_wav_16k_mono(os.path.join(OUT, "sf_test60.wav")), "c4_golden"
    return S.synth_audio(int(minutes * 60 * 16000), 5), f"c4_{minutes}m_golden"


def main():
    minutes = int(sys.argv[sys.argv.index("--minutes") + 1]) if "--minutes" in sys.argv else 1
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    pcm, name = workload(minutes)
    meta = {"seed": SEED, "aheads_preset": AHEADS_LARGE_V3, "params": PARAMS, "block": BLOCK, "results": {},
            "minutes": minutes, "audio": "tests/golden/sf_test60.wav" if minutes == 1 else
            f"owk_synth.synth_audio({minutes * 60 * 16000}, 5)"}
    arrays = {}

    # --- transcription + DTW ---
    path = S.ensure_model("large-v3", SEED, cache)
    meta["model_sha256"] = S.file_sha256(path)
    ref = R.Ref(path, flash_attn=False, dtw_preset=AHEADS_LARGE_V3)
    L = ref.L
    L.whisper_token_to_str.restype = C.c_char_p
    L.whisper_token_to_str.argtypes = [C.c_void_p, C.c_int]
    # first window's prefill logits on this soft_max (flash_attn = false) context: the measured-logit-
    # error bound of the free-run comparison (tests/parity_util.LogitError)
    ref.mel(pcm, n_threads=NT)
    ref.encode(0, n_threads=NT)
    L.whisper_token_transcribe.argtypes = [C.c_void_p]
    L.whisper_token_lang.argtypes = [C.c_void_p, C.c_int]
    prompt = [L.whisper_token_sot(ref.ctx), L.whisper_token_lang(ref.ctx, 0), L.whisper_token_transcribe(ref.ctx)]
    lg = ref.decode(prompt, 0, n_threads=NT)
    top = np.argsort(-lg)[:64]
    arrays["prefill_top_idx"] = top.astype(np.int32)
    arrays["prefill_top_val"] = lg[top]
    meta["results"]["prefill_prompt"] = prompt
    t1 = int(lg.argmax())
    lg2 = ref.decode([t1], len(prompt), n_threads=NT)
    top2 = np.argsort(-lg2)[:64]
    arrays["step1_top_idx"] = top2.astype(np.int32)
    arrays["step1_top_val"] = lg2[top2]
    meta["results"]["step1_token"] = t1
    # one whisper_full on a FRESH state (no_context = false: a state carries its prompt history into
    # the next call), decoder-call prefixes traced with the logits untouched (record_topk = 2; the
    # other fixtures assert that tracing changes nothing, make_golden_nofa_windows.py)
    ref.close()
    stage1 = os.path.join(cache, f"c4_stage1-{meta['model_sha256'][:16]}" + ("" if minutes == 1 else f"-{minutes}m") + ".json")  # the 15-min run, kept
    if os.path.exists(stage1):
        st1 = json.load(open(stage1))
    else:
        ref = R.Ref(path, flash_attn=False, dtw_preset=AHEADS_LARGE_V3)
        t = time.time()
        ret, segs = ref.full(pcm, n_threads=NT, record_topk=2, **PARAMS)
        print("whisper_full", ret, len(segs), "segments", sum(len(s["tokens"]) for s in segs), "tokens",
              f"{time.time() - t:.0f} s", flush=True)
        wins, open_end = traced_windows(ref, [t[0] for s in segs for t in s["tokens"]])
        st1 = {"ret": ret, "segments": segs, "windows": wins, "open": open_end, "words": words_of(L, ref.ctx, segs)}
        ref.close()
        with open(stage1, "w") as f:
            json.dump(st1, f)
    segs = st1["segments"]
    assert len(st1["windows"]) >= 2 and segs[-1]["t1"] > 3000, "the transcription must span more than one 30 s window"
    meta["results"]["full"] = {"ret": st1["ret"], "segments": segs}
    meta["results"]["windows"] = st1["windows"]
    meta["results"]["windows_open"] = st1["open"]
    words = [tuple(w) for w in st1["words"]]
    print("windows", [len(w) for w in st1["windows"]], "open", st1["open"], flush=True)

    # --- streaming diarization, 2 s blocks ---
    mm = json.load(open(os.path.join(OUT, "sf_golden.json")))
    sf_path = os.path.join(cache, f"synth-sortformer-s{mm['seed']}.gguf")
    if not os.path.exists(sf_path) or S.file_sha256(sf_path) != mm["sha256"]:
        assert SS.write_model(sf_path, mm["seed"]) == mm["sha256"]
    meta["sortformer_sha256"] = mm["sha256"]
    sf = SF.Sortformer(sf_path, lib=REF_SF, n_threads=NT)
    probs, counts = stream_run(sf, pcm)
    rng = np.random.default_rng(0)
    pp = (pcm * (1 + 1e-7 * rng.standard_normal(len(pcm)))).astype(np.float32)
    probs_p, _ = stream_run(sf, pp)
    sf.close()
    d = np.abs(probs_p.astype(np.float64) - probs)
    arrays["stream_probs"] = probs
    meta["results"]["stream_counts"] = counts
    meta["results"]["noise_floor/stream"] = {"max": float(d.max()), "mean": float(d.mean())}
    rttm = SF.to_rttm(probs, 0.5, 11, "audio", lib=REF_SF)
    meta["results"]["rttm"] = rttm
    print("stream", probs.shape, "frames; floor", meta["results"]["noise_floor/stream"], flush=True)

    # --- aligner over the reference tokens and RTTM ---
    dsegs = DA.rttm_parse(rttm)
    al = DA.align(words, dsegs)
    meta["results"]["words"] = words
    meta["results"]["aligned"] = {"speakers": [w[3] for w in al["words"]],
                                  "utterances": [(u["speaker"], u["words"][0], len(u["words"])) for u in al["segments"]],
                                  "text": al["text"]}
    print("aligned", len(words), "words,", len(al["segments"]), "utterances", flush=True)

    np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
    with open(os.path.join(OUT, name + ".json"), "w") as f:
        json.dump(meta, f, indent=0)
    print(f"wrote {name}.json / .npz")


if __name__ == "__main__":
    main()
