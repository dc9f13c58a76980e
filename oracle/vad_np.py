"""TEST INFRASTRUCTURE -- numpy restatement of the reference's Silero VAD (CPU oracle).

Only tests/ may import this module; the product path is csrc/vad.cpp + csrc/k_vad.hip.
Pinned against the reference's own outputs (tests/golden/vad_golden.*, made by
tests/golden/make_golden_vad.py from the compiled reference) by tests/test_vad.py.

Restates (ref = /root/reference):
  * model file parse            ref/src/whisper.cpp:4761-5076
  * per-chunk graph             ref/src/whisper.cpp:4519-4653 (stft 4519, encoder 4542, lstm 4567)
  * chunk loop / state reset    ref/src/whisper.cpp:5086-5188
  * segments_from_probs         ref/src/whisper.cpp:5210-5444
  * whisper_vad audio filter    ref/src/whisper.cpp:6643-6826
  * processed->original time    ref/src/whisper.cpp:7947-8025
ggml numerics reproduced: ggml_conv_1d = im2col into F16 (both operands F16, f32
accumulation, ggml.c ggml_conv_1d); the LSTM matmuls are F32 x F32; sigmoid 1/(1+exp(-x)).
"""
from __future__ import annotations

import struct

import numpy as np

SR = 16000


def load_model(path: str) -> dict:
    b = open(path, "rb").read()
    o = 0

    def i32():
        nonlocal o
        v = struct.unpack_from("<i", b, o)[0]
        o += 4
        return v

    assert struct.unpack_from("<I", b, 0)[0] == 0x67676D6C
    o = 4
    n = i32()
    mtype = b[o:o + n].decode()
    o += n
    version = (i32(), i32(), i32())
    n_window, n_context = i32(), i32()
    nl = i32()
    layers = [(i32(), i32(), i32()) for _ in range(nl)]
    lstm_in, lstm_hidden, fin, fout = i32(), i32(), i32(), i32()
    t = {}
    while o < len(b):
        nd, ln, tt = i32(), i32(), i32()
        ne = [i32() for _ in range(nd)]
        name = b[o:o + ln].decode()
        o += ln
        cnt = int(np.prod(ne)) if ne else 1
        dt = np.float16 if tt == 1 else np.float32
        t[name] = np.frombuffer(b, dt, cnt, o).astype(np.float32).reshape(list(reversed(ne)) or [1])
        o += cnt * (2 if tt == 1 else 4)
    return dict(type=mtype, version=version, n_window=n_window, n_context=n_context, layers=layers,
                lstm_in=lstm_in, hidden=lstm_hidden, t=t)


def f16(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def _conv1d(w, x, stride, pad):
    """ggml_conv_1d: w [OC][IC][K] (f16 values), x [B][IC][L] f32 -> [B][OC][OL]; im2col in F16."""
    oc, ic, k = w.shape
    B, _, L = x.shape
    xp = np.zeros((B, ic, L + 2 * pad), np.float32)
    xp[:, :, pad:pad + L] = f16(x)
    ol = (L + 2 * pad - k) // stride + 1
    cols = np.stack([xp[:, :, t * stride:t * stride + k] for t in range(ol)], axis=1)  # [B][OL][IC][K]
    return np.einsum("btik,oik->bot", cols.astype(np.float64), w.astype(np.float64)).astype(np.float32)


def encode_chunks(m: dict, frames: np.ndarray) -> np.ndarray:
    """frames [B][512] -> LSTM input projection W_ih x + b_ih, [B][512] (ref 4519-4576)."""
    t = m["t"]
    B = frames.shape[0]
    padded = np.concatenate([frames[:, 64:0:-1], frames, frames[:, -2:-66:-1]], axis=1)  # reflect 64/64
    basis = t["_model.stft.forward_basis_buffer"].reshape(258, 1, 256)
    st = _conv1d(basis, padded[:, None, :], 128, 0)  # [B][258][4]
    re, im = st[:, :129], st[:, 129:]
    cur = np.sqrt((re * re + im * im).astype(np.float32))
    for i, (s, p) in enumerate(((1, 1), (2, 1), (2, 1), (1, 1))):
        w = t[f"_model.encoder.{i}.reparam_conv.weight"]
        cur = _conv1d(w, cur, s, p) + t[f"_model.encoder.{i}.reparam_conv.bias"][None, :, None]
        cur = np.maximum(cur.astype(np.float32), 0.0)
    x = cur[:, :, 0]
    W = t["_model.decoder.rnn.weight_ih"]  # [512][128]
    return ((x.astype(np.float64) @ W.T.astype(np.float64)).astype(np.float32)
            + t["_model.decoder.rnn.bias_ih"][None, :]).astype(np.float32)


def sigmoid(x):
    return (1.0 / (1.0 + np.exp(-x.astype(np.float32)))).astype(np.float32)


def lstm_and_head(m: dict, ig: np.ndarray, h: np.ndarray, c: np.ndarray):
    """Sequential LSTM over chunks + ReLU + final 1x1 conv + sigmoid (ref 4567-4650)."""
    t = m["t"]
    Whh = t["_model.decoder.rnn.weight_hh"].astype(np.float64)
    bhh = t["_model.decoder.rnn.bias_hh"]
    wf = f16(t["_model.decoder.decoder.2.weight"].reshape(-1)).astype(np.float64)
    bf = np.float32(t["_model.decoder.decoder.2.bias"].reshape(-1)[0])
    H = m["hidden"]
    probs = np.zeros(ig.shape[0], np.float32)
    for i in range(ig.shape[0]):
        hg = (Whh @ h.astype(np.float64)).astype(np.float32) + bhh
        g = (ig[i] + hg).astype(np.float32)
        it, ft, gt, ot = sigmoid(g[:H]), sigmoid(g[H:2 * H]), np.tanh(g[2 * H:3 * H]), sigmoid(g[3 * H:])
        c = (ft * c + it * gt).astype(np.float32)
        h = (ot * np.tanh(c)).astype(np.float32)
        z = np.float32(f16(np.maximum(h, 0)).astype(np.float64) @ wf) + bf
        probs[i] = sigmoid(np.array([z]))[0]
    return probs, h, c


class Vad:
    def __init__(self, path):
        self.m = load_model(path)
        self.reset()

    def reset(self):
        H = self.m["hidden"]
        self.h = np.zeros(H, np.float32)
        self.c = np.zeros(H, np.float32)

    def detect(self, pcm, reset=True):
        """whisper_vad_detect_speech(_stateful): one prob per 512-sample chunk (ref 5086-5165)."""
        if reset:
            self.reset()
        nw = self.m["n_window"]
        n = len(pcm)
        nch = (n + nw - 1) // nw
        fr = np.zeros(nch * nw, np.float32)
        fr[:n] = pcm
        ig = encode_chunks(self.m, fr.reshape(nch, nw))
        p, self.h, self.c = lstm_and_head(self.m, ig, self.h, self.c)
        return p


def samples_to_cs(s):
    return int((s / float(SR)) * 100.0 + 0.5)


def cs_to_samples(cs):
    return int((cs / 100.0) * SR + 0.5)


def segments_from_probs(probs, n_window=512, threshold=0.5, min_speech_duration_ms=250,
                        min_silence_duration_ms=100, max_speech_duration_s=3.4028235e38, speech_pad_ms=30):
    """ref/src/whisper.cpp:5210-5444; returns [(start_cs, end_cs)]."""
    f32 = np.float32
    threshold = f32(threshold)
    n = len(probs)
    min_sil = SR * min_silence_duration_ms // 1000
    audio_len = n * n_window
    min_speech = SR * min_speech_duration_ms // 1000
    pad = SR * speech_pad_ms // 1000
    if f32(max_speech_duration_s) > f32(100000.0):
        max_speech = 2147483647 // 2
    else:
        tmp = SR * int(f32(max_speech_duration_s)) - n_window - 2 * pad
        max_speech = 2147483647 // 2 if (tmp > 2147483647 or tmp < 0) else tmp
    min_sil_at_max = SR * 98 // 1000
    neg = f32(threshold - f32(0.15))
    if neg < f32(0.01):
        neg = f32(0.01)
    sp = []
    is_sp = False
    temp_end = prev_end = next_start = cur_start = 0
    has_cur = False
    for i in range(n):
        p = f32(probs[i])
        cs = n_window * i
        if p >= threshold and temp_end:
            temp_end = 0
            if next_start < prev_end:
                next_start = cs
        if p >= threshold and not is_sp:
            is_sp, cur_start, has_cur = True, cs, True
            continue
        if is_sp and (cs - cur_start) > max_speech:
            if prev_end:
                sp.append([cur_start, prev_end])
                has_cur = True
                if next_start < prev_end:
                    is_sp = has_cur = False
                else:
                    cur_start = next_start
                prev_end = next_start = temp_end = 0
            else:
                sp.append([cur_start, cs])
                prev_end = next_start = temp_end = 0
                is_sp = has_cur = False
                continue
        if p < neg and is_sp:
            if not temp_end:
                temp_end = cs
            if (cs - temp_end) > min_sil_at_max:
                prev_end = temp_end
            if (cs - temp_end) < min_sil:
                continue
            if (temp_end - cur_start) > min_speech:
                sp.append([cur_start, temp_end])
            prev_end = next_start = temp_end = 0
            is_sp = has_cur = False
            continue
    if has_cur and (audio_len - cur_start) > min_speech:
        sp.append([cur_start, audio_len])
    i = 0
    while len(sp) > 1 and i < len(sp) - 1:
        if sp[i + 1][0] - sp[i][1] < SR * 200 // 1000:
            sp[i][1] = sp[i + 1][1]
            del sp[i + 1]
        else:
            i += 1
    sp = [s for s in sp if not (s[1] - s[0] < min_speech)]
    out = []
    for i in range(len(sp)):
        if i == 0:
            sp[i][0] = sp[i][0] - pad if sp[i][0] > pad else 0
        if i < len(sp) - 1:
            sil = sp[i + 1][0] - sp[i][1]
            if sil < 2 * pad:
                sp[i][1] += sil // 2
                sp[i + 1][0] = sp[i + 1][0] - sil // 2 if sp[i + 1][0] > sil // 2 else 0
            else:
                sp[i][1] = sp[i][1] + pad if sp[i][1] + pad < audio_len else audio_len
                sp[i + 1][0] = sp[i + 1][0] - pad if sp[i + 1][0] > pad else 0
        else:
            sp[i][1] = sp[i][1] + pad if sp[i][1] + pad < audio_len else audio_len
        out.append((samples_to_cs(sp[i][0]), samples_to_cs(sp[i][1])))
    return out
