"""whisper-cli's literal decoding defaults as an injected golden (added to golden.json / golden.npz under
"<model>/<clip>/full/cli_default"), produced by the REFERENCE (oracle/_ref/libwhisper_ref.so).

whisper-cli (ref examples/cli/cli.cpp:44-54, 79, 1168-1212) decodes with beam search (beam_size 5 > 1
selects WHISPER_SAMPLING_BEAM_SEARCH), greedy.best_of 5, temperature 0, temperature_inc 0.2 (the
fallback ladder), entropy_thold 2.4, logprob_thold -1, no_speech_thold 0.6, flash_attn. A window whose
beam result fails the thresholds is decoded again at t = 0.2, 0.4, ... by best_of sampled decoders
(ref src/whisper.cpp:7130-7557). Beam candidates and samples are mt19937 draws
(ref src/whisper.cpp:6577-6580), so the run records and truncates each decoder's logits at the
logits_filter_callback point (ref_probe.cpp ref_record_cb) and the GPU test substitutes them
(tests/golden/recording.py Injector): RNG streams, candidate sorting, KV-cell reordering, the
fallback decisions and the best-of choice must then match bit for bit (tests/test_gpu_parity.py,
config "cli_default").

The fixture is kept only if the beam -> sampled best-of switch actually runs: the recorded calls must
show more decoding attempts than windows (each attempt starts with every decoder's empty prefix).

Usage (container with /root/reference):  python tests/golden/make_golden_cli_default.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import ref_oracle as R  # noqa: E402
from make_golden import SEED, clips  # noqa: E402
from recording import prefix_hash  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
CLI_DEFAULT = dict(strategy=1, beam_size=5, best_of=5, temperature=0.0, temperature_inc=0.2)
MODELS = ("tiny.en", "base.en")


def attempts(off, prefix):
    """decoding attempts of a recorded run: runs of consecutive empty-prefix calls (one per decoder)"""
    n, prev_empty = 0, False
    for i in range(len(off) - 1):
        empty = off[i + 1] == off[i]
        if empty and not prev_empty:
            n += 1
        prev_empty = empty
    return n


def main():
    meta = json.load(open(os.path.join(OUT, "golden.json")))
    arrays = dict(np.load(os.path.join(OUT, "golden.npz")))
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    audio = clips()
    for model in MODELS:
        path = os.path.join(cache, f"synth-{model}-s{SEED}.bin")
        if not os.path.exists(path):
            S.write_model(path, model, SEED)
        assert S.file_sha256(path) == meta["models"][model]["sha256"]
        ref = R.Ref(path)
        for cname, pcm in audio.items():
            key = f"{model}/{cname}/full/cli_default"
            ret, segs = ref.full(pcm, language="en", record_topk=True, n_threads=int(os.environ.get("REF_THREADS", "4")),
                                 **CLI_DEFAULT)
            off, prefix, idx, val = ref.recorded()
            n_att = attempts(off, prefix)
            n_win = len({(s["t0"]) for s in segs}) if segs else 0
            print(f"{key}: ret {ret}, {len(segs)} segments, {sum(len(s['tokens']) for s in segs)} tokens, "
                  f"{len(off) - 1} decoder calls, {n_att} decoding attempts", flush=True)
            meta["results"][key] = {"ret": ret, "segments": segs, "attempts": n_att, "params": CLI_DEFAULT}
            arrays[key + "/rec_hash"] = np.array([prefix_hash(prefix[off[i]:off[i + 1]]) for i in range(len(off) - 1)],
                                                 np.uint64)
            arrays[key + "/rec_idx"] = np.where(idx < 0, 65535, idx).astype(np.uint16)
            arrays[key + "/rec_val"] = val
            del n_win
        ref.close()
    np.savez_compressed(os.path.join(OUT, "golden.npz"), **arrays)
    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
