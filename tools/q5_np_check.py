"""CPU check: numpy restatement of the Q5_0 encoder (q5 weights x q8_0 activations) against
the reference golden encoder rows (tests/golden/q5_golden.npz). Debug tool, not a test."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402
import whisper_np as W  # noqa: E402

f32 = np.float32
Q5 = {}
MODE = sys.argv[2] if len(sys.argv) > 2 else "q8"


def q8(a):
    b = a.reshape(a.shape[0], -1, 32)
    am = np.abs(b).max(-1)
    d = (am / f32(127)).astype(f32)
    with np.errstate(divide="ignore"):
        idv = np.where(am != 0, f32(127) / am, f32(0)).astype(f32)
    q = np.rint((b * idv[..., None]).astype(f32))
    return (q * d.astype(np.float16).astype(f32)[..., None]).reshape(a.shape)


def mm(a, w):
    a = np.asarray(a, f32)
    if id(w) in Q5:
        if MODE == "q8":
            return (q8(a).astype(np.float64) @ Q5[id(w)].astype(np.float64).T).astype(f32)
        if MODE == "f32":
            return (a.astype(np.float64) @ Q5[id(w)].astype(np.float64).T).astype(f32)
    return (a.astype(np.float16).astype(f32) @ np.asarray(w, f32).T).astype(f32)


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "tiny.en"
    path = S.ensure_model(model)
    hp, filters, t = W.read_model(path)
    for name, w in list(t.items()):
        if w.ndim == 2 and name not in ("encoder.positional_embedding", "decoder.positional_embedding",
                                       "encoder.conv1.bias", "encoder.conv2.bias"):
            blocks = S.q5_0_blocks(w.astype(f32))
            bl = np.frombuffer(blocks, np.uint8).reshape(-1, 22)
            d = bl[:, 0:2].copy().view("<f2")[:, 0].astype(f32)
            qh = bl[:, 2:6].copy().view("<u4")[:, 0]
            qs = bl[:, 6:22]
            lo = np.concatenate([qs & 15, qs >> 4], axis=-1).astype(np.int32)
            hb = ((qh[:, None] >> np.arange(32)) & 1).astype(np.int32)
            v = (((lo | (hb << 4)) - 16) * d[:, None]).astype(f32).reshape(w.shape)
            t[name] = v
            Q5[id(v)] = v
    W.mm = mm
    pcm = S.read_wav_16k_mono(os.path.join(ROOT, "tests", "golden", "jfk.wav"))
    mel, _ = W.log_mel(pcm, filters)
    enc = W.encoder(hp, t, mel)
    rows = np.concatenate([enc[:16], enc[740:756], enc[1484:]])
    gold = np.load(os.path.join(ROOT, "tests", "golden", "q5_golden.npz"))[f"{model}/jfk/enc_rows"]
    e = np.abs(rows - gold)
    print(model, MODE, "max", e.max(), "mean", e.mean())


if __name__ == "__main__":
    main()
