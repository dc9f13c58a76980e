"""BASELINE configs[4] on one MI355X: large-v3 transcription with DTW token timestamps plus
streaming-SortFormer diarization of 10 minutes of audio.

Workload (synthetic data and random-init weights of the real architectures, as bench.py):
  * a seeded 10 min synthetic 16 kHz clip;
  * transcription: large-v3 F16 with flash_attn = false (DTW needs the soft_max path, as in
    the reference) and dtw_aheads_preset = WHISPER_AHEADS_LARGE_V3; the clip is cut into 30 s
    chunks decoded as one owk_full_batch (the whisper_full_parallel split), greedy,
    temperature_inc = 0, timestamps on, token timestamps on;
  * diarization: sortformer_diarize of the whole clip (default parameters);
  * alignment: sortformer_to_rttm -> RTTM parse -> DiarizationAligner.align of every token
    (the Swift SDK's WordTiming per token, WhisperContext.swift:126-139, chunk offsets added),
    all host C++ in libwhisper.so (include/owk_diarize.h).
Reports the wall time of each part and the real-time factor of the whole job; the reference
CPU path (16 threads) is timed on ONE 30 s chunk of the same transcription settings.

--mode sequential runs the job as the Swift SDK does (WhisperContext.swift calls whisper_full over
the whole buffer): ONE whisper_full over the 10 minutes -- the reference's sequential window loop
with seek advance and prompt carry (ref src/whisper.cpp:7034-7769), no_context = false -- plus
sortformer_stream_feed in 2 s blocks (the "2s" preset) on a second host thread and its own HIP
stream beside it (--serial: after it), and the aligner on the absolute token times. The chunk
split above changes results at split points; the sequential mode is the reference's
semantics, the chunked one the batch-throughput form. --mode both reports both.

    python tools/pipeline_bench.py [--minutes 10] [--no-cpu] [--mode both|chunked|sequential]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import owk  # noqa: E402
import owk_synth as S  # noqa: E402
import sortformer as SF  # noqa: E402
import sortformer_synth as SS  # noqa: E402

AHEADS_LARGE_V3 = 13
CHUNK = 30 * 16000


def words_of(w, states, offsets):
    words = []
    for off, st_ in zip(offsets, states):
        for s in w.segments(st_):
            for t in s["tokens"]:
                txt = w.L.whisper_token_to_str(w.ctx, t[0]).decode("utf-8", "replace")
                words.append((txt, off + t[6] / 100.0, off + t[7] / 100.0, t[2]))
    return words


def run_chunked(args, w, sf, pcm, n):
    chunks = [pcm[i:i + CHUNK] for i in range(0, n, CHUNK)]
    p = w.params(0, language="en", temperature_inc=0.0, token_timestamps=True)
    # warm-up (code objects, buffers, graphs) on one chunk
    st = [w.new_state()]
    w.full_batch(st, chunks[:1], p)
    sf.diarize(pcm[:CHUNK])

    states = [w.new_state() for _ in chunks]
    if args.prof:
        w.L.owk_prof_enable(w.ctx, 1)
        w.L.owk_prof_reset(w.ctx)
    t0 = time.perf_counter()
    ret = w.full_batch(states, chunks, p)
    t_asr = time.perf_counter() - t0
    assert ret == 0, ret
    if args.prof:
        tot = {c: w.prof(c) for c in w.prof_classes()}
        for c, v in sorted(tot.items(), key=lambda kv: -kv[1]["ms"]):
            print(f"[prof] {c:20s} {v['ms']:10.2f} ms  launches {v['launches']:8d}", file=sys.stderr, flush=True)
        w.L.owk_prof_enable(w.ctx, 0)
    n_tok = sum(len(s["tokens"]) for st_ in states for s in w.segments(st_))
    n_dtw = sum(1 for st_ in states for s in w.segments(st_) for t in s["tokens"] if t[8] >= 0)
    t0 = time.perf_counter()
    probs = sf.diarize(pcm)
    t_diar = time.perf_counter() - t0
    t0 = time.perf_counter()
    segs = owk.rttm_parse(SF.to_rttm(probs))
    aligned = owk.align(words_of(w, states, [ci * CHUNK / 16000.0 for ci in range(len(chunks))]), segs)
    t_align = time.perf_counter() - t0
    for st_ in states + st:
        w.free_state(st_)
    return {"value": round(n / 16000 / (t_asr + t_diar + t_align), 2),
            "asr_wall_s": round(t_asr, 3), "diarize_wall_s": round(t_diar, 4), "align_wall_s": round(t_align, 4),
            "rttm_segments": len(segs), "aligned_words": len(aligned["words"]),
            "utterances": len(aligned["segments"]), "chunks": len(chunks),
            "tokens": n_tok, "tokens_with_t_dtw": n_dtw, "diarize_frames": int(probs.shape[0]),
            "workload": "large-v3 F16 flash_attn=false + DTW (LARGE_V3 heads), 30 s chunks in one batch, greedy; "
                        "SortFormer offline, synthetic weights and audio"}


def run_sequential(args, w, sf, pcm, n):
    p = w.params(0, language="en", temperature_inc=0.0, token_timestamps=True, no_context=False)
    warm = w.new_state()
    w.full(warm, pcm[:CHUNK], p)  # warm-up: code objects, buffers, batch-1 graphs
    w.free_state(warm)
    st = w.new_state()
    if args.prof:
        w.L.owk_prof_enable(w.ctx, 1)
        w.L.owk_prof_reset(w.ctx)
    # the diarizer streams its 2 s blocks on its own context / HIP stream from a second host thread
    # while whisper_full runs (the two parts are independent until the aligner; ctypes releases the
    # GIL for both), so the job's wall time is the longer of the two plus the aligner
    diar = {}

    def diarize():
        stream = sf.stream("2s")
        t1 = time.perf_counter()
        blocks = [stream.feed(pcm[i:i + 32000]) for i in range(0, n, 32000)]
        blocks.append(stream.flush())
        diar["wall"] = time.perf_counter() - t1
        diar["end"] = time.perf_counter()
        stream.close()
        diar["blocks"] = blocks
    import threading
    th = threading.Thread(target=diarize) if args.concurrent else None
    t0 = time.perf_counter()
    if th:
        th.start()
    ret = w.full(st, pcm, p)
    t_asr = time.perf_counter() - t0
    if th:
        th.join()
    t_both = max(t_asr, diar.get("end", t0) - t0) if th else None
    assert ret == 0, ret
    if args.prof:
        tot = {c: w.prof(c) for c in w.prof_classes()}
        for c, v in sorted(tot.items(), key=lambda kv: -kv[1]["ms"]):
            print(f"[prof] {c:20s} {v['ms']:10.2f} ms  launches {v['launches']:8d}", file=sys.stderr, flush=True)
        w.L.owk_prof_enable(w.ctx, 0)
    segs_w = w.segments(st)
    n_tok = sum(len(s["tokens"]) for s in segs_w)
    n_dtw = sum(1 for s in segs_w for t in s["tokens"] if t[8] >= 0)
    # streaming diarization: 2 s blocks as a live feed would deliver them (after the ASR unless concurrent)
    if not th:
        diarize()
    blocks, t_diar = diar["blocks"], diar["wall"]
    probs = np.concatenate([b for b in blocks if len(b)], axis=0) if any(len(b) for b in blocks) \
        else np.zeros((0, 4), np.float32)
    t0 = time.perf_counter()
    segs = owk.rttm_parse(SF.to_rttm(probs))
    aligned = owk.align(words_of(w, [st], [0.0]), segs)  # token times are absolute in one whisper_full
    t_align = time.perf_counter() - t0
    w.free_state(st)
    wall = (t_both if th else t_asr + t_diar) + t_align
    return {"value": round(n / 16000 / wall, 2), "wall_s": round(wall, 3),
            "diarize_concurrent": bool(th), "serial_value": round(n / 16000 / (t_asr + t_diar + t_align), 2),
            "asr_wall_s": round(t_asr, 3), "diarize_wall_s": round(t_diar, 4), "align_wall_s": round(t_align, 4),
            "segments": len(segs_w), "rttm_segments": len(segs), "aligned_words": len(aligned["words"]),
            "utterances": len(aligned["segments"]), "tokens": n_tok, "tokens_with_t_dtw": n_dtw,
            "diarize_frames": int(probs.shape[0]),
            "workload": "large-v3 F16 flash_attn=false + DTW (LARGE_V3 heads), ONE whisper_full over the whole "
                        "buffer (sequential windows, prompt carry), greedy; SortFormer streamed in 2 s blocks; "
                        "synthetic weights and audio"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--prof", action="store_true", help="per-kernel-class HIP-event timing of the ASR part (eager)")
    ap.add_argument("--mode", choices=["both", "chunked", "sequential"], default="both")
    ap.add_argument("--serial", dest="concurrent", action="store_false",
                    help="sequential mode: diarize after the transcription instead of beside it")
    ap.add_argument("--whole-k-rows", type=int, default=None,
                    help="A/B: decode passes of at most this many rows take the whole-K chain (engine default if unset)")
    args = ap.parse_args()
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    model = S.ensure_model("large-v3", cache_dir=cache)
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "sf_golden.json")))
    sf_path = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
    if not os.path.exists(sf_path):
        assert SS.write_model(sf_path, meta["seed"]) == meta["sha256"]
    n = int(args.minutes * 60 * 16000)
    pcm = S.synth_audio(n, 5)

    owk.quiet()
    if args.whole_k_rows is not None:
        import ctypes as C
        owk.load().owk_debug_set_whole_k_rows.argtypes = [C.c_int]
        owk.load().owk_debug_set_whole_k_rows(args.whole_k_rows)
    w = owk.Whisper(model, flash_attn=False, dtw_preset=AHEADS_LARGE_V3)
    sf = SF.Sortformer(sf_path)
    import ctypes as C
    w.L.whisper_token_to_str.restype = C.c_char_p
    w.L.whisper_token_to_str.argtypes = [C.c_void_p, C.c_int]
    out = {"metric": "transcribe + DTW + diarize + align real-time factor (audio-s/wall-s), configs[4]",
           "unit": "audio-s/wall-s", "audio_s": n / 16000}
    if args.mode in ("both", "chunked"):
        out["chunked"] = run_chunked(args, w, sf, pcm, n)
        out["value"] = out["chunked"]["value"]
    if args.mode in ("both", "sequential"):
        out["sequential"] = run_sequential(args, w, sf, pcm, n)
        out.setdefault("value", out["sequential"]["value"])
    sf.close()
    if not args.no_cpu:
        import ref_oracle as R
        if R.available():
            nt = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "1000")))
            ref = R.Ref(model, flash_attn=False, dtw_preset=AHEADS_LARGE_V3)
            t0 = time.perf_counter()
            r, segs = ref.full(pcm[:CHUNK], n_threads=nt, language="en", temperature_inc=0.0, token_timestamps=True)
            rw = time.perf_counter() - t0
            ref.close()
            out["cpu_baseline_asr"] = {"value": round(30.0 / rw, 3), "unit": "audio-s/wall-s", "cores": nt,
                                       "kind": "reference", "sample": f"one 30 s chunk, same settings, ret={r}, "
                                       f"{sum(len(s['tokens']) for s in segs)} tokens, wall {rw:.1f} s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
