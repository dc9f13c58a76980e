"""TEST INFRASTRUCTURE -- numpy restatement of the reference Whisper numerics.

A plain CPU re-statement of the reference algorithm for the hot path, used only by
tests/ as an independent checker (it is pinned against the golden vectors that the
compiled reference produced, tests/test_oracle_pin.py). Never imported by the product.

Each function cites the reference code it restates (paths relative to /root/reference):
  read_model        src/whisper.cpp:1485-1956       ggml-bin loader
  log_mel           src/whisper.cpp:3104-3260       STFT -> mel -> log10 -> clamp/normalise
  gelu_table        ggml/src/ggml-cpu/vec.h:975-1009  F16 GELU lookup table
  layer_norm        ggml/src/ggml-cpu/ops.cpp:3578-3623 + whisper.cpp:2103-2108
  mul_mat_f16       ggml-cpu.c:1227 (activation rounded to F16, f32 accumulate)
  encoder           src/whisper.cpp:1976-2269 (conv stack + FA encoder, 36 zero pad keys)
  cross_kv          src/whisper.cpp:2272-2346
  decode            src/whisper.cpp:2458-2978; FA one_chunk ops.cpp:8140-8233 (F16 V accumulator)
"""
from __future__ import annotations

import struct

import numpy as np

f16 = np.float16
f32 = np.float32


def read_model(path):
    b = open(path, "rb").read()
    hp = struct.unpack_from("<11i", b, 4)
    off = 48
    n_mel, n_fft = struct.unpack_from("<ii", b, off)
    off += 8
    filters = np.frombuffer(b, "<f4", n_mel * n_fft, off).reshape(n_mel, n_fft)
    off += n_mel * n_fft * 4
    n_vocab, = struct.unpack_from("<i", b, off)
    off += 4
    for _ in range(n_vocab):
        ln, = struct.unpack_from("<I", b, off)
        off += 4 + ln
    t = {}
    while off < len(b):
        nd, nl, tt = struct.unpack_from("<iii", b, off)
        off += 12
        ne = struct.unpack_from("<%di" % nd, b, off)
        off += 4 * nd
        name = b[off:off + nl].decode()
        off += nl
        n = int(np.prod(ne))
        dt = "<f2" if tt == 1 else "<f4"
        t[name] = np.frombuffer(b, dt, n, off).reshape(tuple(reversed(ne)))
        off += n * (2 if tt == 1 else 4)
    keys = ["n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer", "n_text_ctx",
            "n_text_state", "n_text_head", "n_text_layer", "n_mels", "ftype"]
    return dict(zip(keys, hp)), filters, t


# ------------------------------------------------------------------------------------
def log_mel(pcm, filters):
    """(mel[n_mel][n_len], n_len_org) -- reflect pad 200, zero pad 30 s, periodic Hann,
    |FFT|^2 of 201 bins, mel projection, log10(max(.,1e-10)), max-8 clamp, (x+4)/4."""
    pcm = np.asarray(pcm, f32)
    n = len(pcm)
    padded = np.zeros(n + 480000 + 400, f32)
    padded[200:200 + n] = pcm
    padded[:200] = pcm[1:201][::-1]
    n_len = (len(padded) - 400) // 160
    n_len_org = 1 + (n + 200 - 400) // 160
    i = np.arange(400)
    hann = (0.5 * (1.0 - np.cos((2.0 * np.pi * i / 400).astype(f32)).astype(np.float64))).astype(f32)
    n_w = n + 200
    n_compute = min(n_w // 160 + 1, n_len)
    idx = np.arange(n_compute)[:, None] * 160 + i[None, :]
    frames = padded[idx].copy()
    frames[idx >= n_w] = 0.0
    frames = (frames * hann[None, :]).astype(np.float64)
    spec = np.fft.rfft(frames, axis=1)
    power = spec.real ** 2 + spec.imag ** 2
    mel = np.full((filters.shape[0], n_len), -10.0, np.float64)
    mel[:, :n_compute] = np.log10(np.maximum(filters.astype(np.float64) @ power.T, 1e-10))
    mel = mel.astype(f32)
    mmax = float(mel.max()) - 8.0
    mel = np.where(mel.astype(np.float64) < mmax, f32(mmax), mel)
    return ((mel.astype(np.float64) + 4.0) / 4.0).astype(f32), n_len_org


# ------------------------------------------------------------------------------------
def _tanhf(x):
    """The C library's tanhf (what the reference calls); numpy's float32 tanh differs in
    the last ulp for some inputs, which flips f16 table entries."""
    import ctypes

    libm = ctypes.CDLL("libm.so.6")
    libm.tanhf.restype = ctypes.c_float
    libm.tanhf.argtypes = [ctypes.c_float]
    return np.array([libm.tanhf(float(v)) for v in np.asarray(x, f32)], f32)


def gelu_table():
    x = np.arange(65536, dtype=np.uint16).view(f16).astype(f32)
    a = f32(0.044715)
    c = f32(0.79788456080286535587989211986876)
    with np.errstate(all="ignore"):
        inner = (((a * x).astype(np.float64) * x.astype(np.float64)) + 1.0).astype(f32)  # fma(a*x, x, 1)
        g = (f32(0.5) * x * (f32(1.0) + _tanhf(c * x * inner))).astype(f32)
    return g.astype(f16).view(np.uint16)


_GT = None


def gelu(x):
    global _GT
    if _GT is None:
        _GT = gelu_table().view(f16).astype(f32)
    x = np.asarray(x, f32)
    y = _GT[x.astype(f16).view(np.uint16)]
    y = np.where(x >= 10.0, x, y)
    return np.where(x <= -10.0, f32(0.0), y).astype(f32)


def layer_norm(x, w, b, eps=1e-5):
    x = np.asarray(x, f32)
    s = x.astype(np.float64).sum(axis=-1, keepdims=True)
    mean = (s.astype(f32) / f32(x.shape[-1])).astype(f32)
    y = (x - mean).astype(f32)
    var = ((y.astype(np.float64) ** 2).sum(axis=-1, keepdims=True) / x.shape[-1]).astype(f32)
    scale = (f32(1.0) / np.sqrt(var + f32(eps))).astype(f32)
    return ((y * scale).astype(f32) * w + b).astype(f32)


def mm(a, w):
    """ggml_mul_mat with an F16 weight: activation rounded to f16, f32 accumulation."""
    return (np.asarray(a, f32).astype(f16).astype(f32) @ np.asarray(w, f32).T).astype(f32)


# ------------------------------------------------------------------------------------
def _flash_tiled(q, k, v, scale, n_zero_pad):
    """F32-accumulated attention (tiled path): softmax over T real keys + n_zero_pad keys
    with score 0 and value 0. q,k,v: [H][T][64] (q/k/v already f16-representable)."""
    s = np.einsum("htd,hsd->hts", q.astype(f32), k.astype(f32)) * f32(scale)
    m = np.maximum(s.max(axis=-1, keepdims=True), 0.0 if n_zero_pad else -np.inf)
    p = np.exp((s - m).astype(np.float64))
    den = p.sum(axis=-1, keepdims=True) + n_zero_pad * np.exp(-m.astype(np.float64))
    return (np.einsum("hts,hsd->htd", p, v.astype(np.float64)) / den).astype(f32)


def encoder(hp, t, mel, offset=0):
    d, H, L, nm = hp["n_audio_state"], hp["n_audio_head"], hp["n_audio_layer"], hp["n_mels"]
    T = hp["n_audio_ctx"]
    win = np.zeros((nm, 2 * T), f32)
    i1 = min(offset + 2 * T, mel.shape[1])
    if i1 > offset:
        win[:, : i1 - offset] = mel[:, offset:i1]

    def conv(x, w, bias, stride):  # x [C][Tin]; w [O][C][3]
        tin = x.shape[1]
        xp = np.pad(x, ((0, 0), (1, 1)))
        tout = tin // stride
        cols = np.stack([xp[:, k: k + stride * tout: stride] for k in range(3)], axis=-1)  # [C][Tout][3]
        A = cols.transpose(1, 0, 2).reshape(tout, -1)
        return mm(A, w.reshape(w.shape[0], -1)) + bias.reshape(1, -1)

    x1 = gelu(conv(win, t["encoder.conv1.weight"], t["encoder.conv1.bias"], 1))  # [3000][d]
    x2 = gelu(conv(x1.T, t["encoder.conv2.weight"], t["encoder.conv2.bias"], 2))  # [1500][d]
    x = (t["encoder.positional_embedding"] + x2).astype(f32)
    n_pad = (T + 255) // 256 * 256 - T
    for l in range(L):
        p = f"encoder.blocks.{l}."
        h = layer_norm(x, t[p + "attn_ln.weight"], t[p + "attn_ln.bias"])
        q = (mm(h, t[p + "attn.query.weight"]) + t[p + "attn.query.bias"]).astype(f16)
        k = mm(h, t[p + "attn.key.weight"]).astype(f16)
        v = (mm(h, t[p + "attn.value.weight"]) + t[p + "attn.value.bias"]).astype(f16)
        sh = lambda z: z.reshape(T, H, 64).transpose(1, 0, 2)  # noqa: E731
        a = _flash_tiled(sh(q), sh(k), sh(v), 1.0 / np.sqrt(64.0), n_pad)
        a = a.transpose(1, 0, 2).reshape(T, d)
        x = (x + (mm(a, t[p + "attn.out.weight"]) + t[p + "attn.out.bias"])).astype(f32)
        h = layer_norm(x, t[p + "mlp_ln.weight"], t[p + "mlp_ln.bias"])
        h = gelu(mm(h, t[p + "mlp.0.weight"]) + t[p + "mlp.0.bias"])
        x = (x + (mm(h, t[p + "mlp.2.weight"]) + t[p + "mlp.2.bias"])).astype(f32)
    return layer_norm(x, t["encoder.ln_post.weight"], t["encoder.ln_post.bias"])


def cross_kv(hp, t, enc):
    s = f32(64.0 ** -0.25)
    out = []
    for l in range(hp["n_text_layer"]):
        p = f"decoder.blocks.{l}.cross_attn."
        k = (mm(enc, t[p + "key.weight"]) * s).astype(f16)
        v = (mm(enc, t[p + "value.weight"]) + t[p + "value.bias"]).astype(f16)
        out.append((k, v))
    return out


def _one_chunk(qh, K, V, scale, n_zero_pad):
    """ggml one_chunk flash attention for one query row: per key, F16 V accumulator
    rounded after every update (ops.cpp:8168-8233). qh [H][64] f16, K,V [N][H][64] f16."""
    H = qh.shape[0]
    s_all = (np.einsum("hd,nhd->nh", qh.astype(f32), K.astype(f32)) * f32(scale)).astype(f32)
    M = np.full(H, -np.inf, f32)
    S = np.zeros(H, f32)
    acc = np.zeros((H, 64), f16)
    N = K.shape[0]
    with np.errstate(over="ignore", invalid="ignore"):
        for i in range(N + n_zero_pad):
            s = s_all[i] if i < N else np.zeros(H, f32)
            vv = V[i].astype(f32) if i < N else np.zeros((H, 64), f32)
            newmax = s > M
            ms = np.where(newmax, np.exp((M - s).astype(f32)), f32(1.0)).astype(f32)
            vs = np.where(newmax, f32(1.0), np.exp((s - M).astype(f32))).astype(f32)
            M = np.where(newmax, s, M)
            acc = np.where(newmax[:, None], (acc.astype(f32) * ms[:, None]).astype(f16), acc)
            acc = (acc.astype(np.float64) + vv.astype(np.float64) * vs[:, None].astype(np.float64)).astype(f32).astype(f16)
            S = (S.astype(np.float64) * ms + vs).astype(f32)
    inv = np.where(S == 0, f32(0.0), f32(1.0) / S).astype(f32)
    return (acc.astype(f32) * inv[:, None]).astype(f32)


class Decoder:
    """Greedy-call decoder over one sequence (cells in position order)."""

    def __init__(self, hp, t, cross):
        self.hp, self.t, self.cross = hp, t, cross
        self.k = [[] for _ in range(hp["n_text_layer"])]
        self.v = [[] for _ in range(hp["n_text_layer"])]

    def step(self, tokens, n_past):
        hp, t = self.hp, self.t
        d, H = hp["n_text_state"], hp["n_text_head"]
        s = f32(64.0 ** -0.25)
        n = len(tokens)
        x = (t["decoder.token_embedding.weight"][tokens].astype(f32) +
             t["decoder.positional_embedding"][n_past:n_past + n]).astype(f32)
        n_pad = (hp["n_audio_ctx"] + 255) // 256 * 256 - hp["n_audio_ctx"]
        tiled = n >= 32
        for l in range(hp["n_text_layer"]):
            p = f"decoder.blocks.{l}."
            h = layer_norm(x, t[p + "attn_ln.weight"], t[p + "attn_ln.bias"])
            q = ((mm(h, t[p + "attn.query.weight"]) + t[p + "attn.query.bias"]) * s).astype(f16)
            kk = (mm(h, t[p + "attn.key.weight"]) * s).astype(f16)
            vv = (mm(h, t[p + "attn.value.weight"]) + t[p + "attn.value.bias"]).astype(f16)
            self.k[l] += list(kk)
            self.v[l] += list(vv)
            K = np.stack(self.k[l]).reshape(-1, H, 64)
            V = np.stack(self.v[l]).reshape(-1, H, 64)
            a = np.zeros((n, d), f32)
            for r in range(n):
                nk = n_past + r + 1
                if tiled and K.shape[0] % 16 == 0:
                    a[r] = _flash_tiled(q[r].reshape(H, 1, 64), K[:nk].transpose(1, 0, 2),
                                        V[:nk].transpose(1, 0, 2), 1.0, 0).reshape(d)
                else:
                    a[r] = _one_chunk(q[r].reshape(H, 64), K[:nk], V[:nk], 1.0, 0).reshape(d)
            x = (x + (mm(a, t[p + "attn.out.weight"]) + t[p + "attn.out.bias"])).astype(f32)
            h = layer_norm(x, t[p + "cross_attn_ln.weight"], t[p + "cross_attn_ln.bias"])
            q = (mm(h, t[p + "cross_attn.query.weight"]) + t[p + "cross_attn.query.bias"]).astype(f16)
            Kc, Vc = self.cross[l]
            Kc = Kc.reshape(-1, H, 64)
            Vc = Vc.reshape(-1, H, 64)
            for r in range(n):
                if tiled:
                    a[r] = _flash_tiled(q[r].reshape(H, 1, 64), Kc.transpose(1, 0, 2), Vc.transpose(1, 0, 2), s,
                                        n_pad).reshape(d)
                else:
                    a[r] = _one_chunk(q[r].reshape(H, 64), Kc, Vc, s, n_pad).reshape(d)
            x = (x + (mm(a, t[p + "cross_attn.out.weight"]) + t[p + "cross_attn.out.bias"])).astype(f32)
            h = layer_norm(x, t[p + "mlp_ln.weight"], t[p + "mlp_ln.bias"])
            h = gelu(mm(h, t[p + "mlp.0.weight"]) + t[p + "mlp.0.bias"])
            x = (x + (mm(h, t[p + "mlp.2.weight"]) + t[p + "mlp.2.bias"])).astype(f32)
        h = layer_norm(x[-1:], t["decoder.ln.weight"], t["decoder.ln.bias"])
        return mm(h, t["decoder.token_embedding.weight"])[0]
