"""Synthetic-weight Whisper models in the reference's ggml-bin file format.

No real Whisper weights exist offline, so parity and throughput are measured on
deterministic synthetic weights written in exactly the format the reference loader
reads (whisper_model_load, /root/reference src/whisper.cpp:1485-1956; tensor naming
src/whisper-arch.h:42-106; dtype rules models/convert-pt-to-ggml.py:300-315:
>=2-D tensors F16 except conv biases and positional embeddings, which are F32).

The mel filterbank (80 bins) and tokenizer vocab are the reference's own test-model
data (assets/, extracted by tools/extract_assets.py); the 128-bin filterbank for the
large-v3 family is generated here with the Slaney mel formula and validated against
the 80-bin one (tests/test_synth.py).

Same seed => byte-identical file on any machine (numpy PCG64), so the GPU box
regenerates exactly the models the golden fixtures were produced from (the fixtures
record each file's SHA-256).
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import struct

import numpy as np

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "assets")

# hparams: n_vocab, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer,
#          n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels
MODELS = {
    "tiny.en":        (51864, 1500, 384, 6, 4, 448, 384, 6, 4, 80),
    "tiny":           (51865, 1500, 384, 6, 4, 448, 384, 6, 4, 80),
    "base.en":        (51864, 1500, 512, 8, 6, 448, 512, 8, 6, 80),
    "small.en":       (51864, 1500, 768, 12, 12, 448, 768, 12, 12, 80),
    "large-v3":       (51866, 1500, 1280, 20, 32, 448, 1280, 20, 32, 128),
    "large-v3-turbo": (51866, 1500, 1280, 20, 32, 448, 1280, 20, 4, 128),
    # reduced-depth shapes with the large-v3 width / vocab / 128 mels, for fast tests
    "l3-mini":        (51866, 1500, 1280, 20, 2, 448, 1280, 20, 2, 128),
}

GGML_FILE_MAGIC = 0x67676D6C


def slaney_mel_filters(n_mels: int, sr: int = 16000, n_fft: int = 400) -> np.ndarray:
    """Slaney-normalised triangular mel filterbank [n_mels, 1 + n_fft/2] (float32)."""
    fft_freqs = np.linspace(0.0, sr / 2.0, 1 + n_fft // 2)

    f_sp = 200.0 / 3.0
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0

    def hz_to_mel(f):
        f = np.asanyarray(f, dtype=np.float64)
        m = f / f_sp
        return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, m)

    def mel_to_hz(m):
        m = np.asanyarray(m, dtype=np.float64)
        f = f_sp * m
        return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f)

    mel_pts = mel_to_hz(np.linspace(hz_to_mel(0.0), hz_to_mel(sr / 2.0), n_mels + 2))
    fdiff = np.diff(mel_pts)
    ramps = mel_pts[:, None] - fft_freqs[None, :]
    w = np.zeros((n_mels, len(fft_freqs)))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0.0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_pts[2:n_mels + 2] - mel_pts[:n_mels])
    w *= enorm[:, None]
    return w.astype(np.float32)


def mel_filters(n_mels: int) -> np.ndarray:
    if n_mels == 80:
        return np.load(os.path.join(ASSETS, "mel_filters_80.npy"))
    return slaney_mel_filters(n_mels)


def vocab_bytes(multilingual: bool) -> bytes:
    name = "vocab_multilingual.bin.gz" if multilingual else "vocab_en.bin.gz"
    with gzip.open(os.path.join(ASSETS, name), "rb") as f:
        return f.read()


def tensor_list(hp):
    """(name, shape-in-numpy-order, is_f16) in the order convert-pt-to-ggml writes them."""
    n_vocab, n_actx, d, _, n_alayer, n_tctx, dt, _, n_tlayer, n_mels = hp
    out = [("encoder.positional_embedding", (n_actx, d), False),
           ("encoder.conv1.weight", (d, n_mels, 3), True),
           ("encoder.conv1.bias", (d, 1), False),
           ("encoder.conv2.weight", (d, d, 3), True),
           ("encoder.conv2.bias", (d, 1), False)]
    for i in range(n_alayer):
        p = f"encoder.blocks.{i}."
        out += [(p + "attn.query.weight", (d, d), True), (p + "attn.query.bias", (d,), False),
                (p + "attn.key.weight", (d, d), True),
                (p + "attn.value.weight", (d, d), True), (p + "attn.value.bias", (d,), False),
                (p + "attn.out.weight", (d, d), True), (p + "attn.out.bias", (d,), False),
                (p + "attn_ln.weight", (d,), False), (p + "attn_ln.bias", (d,), False),
                (p + "mlp.0.weight", (4 * d, d), True), (p + "mlp.0.bias", (4 * d,), False),
                (p + "mlp.2.weight", (d, 4 * d), True), (p + "mlp.2.bias", (d,), False),
                (p + "mlp_ln.weight", (d,), False), (p + "mlp_ln.bias", (d,), False)]
    out += [("encoder.ln_post.weight", (d,), False), ("encoder.ln_post.bias", (d,), False),
            ("decoder.positional_embedding", (n_tctx, dt), False),
            ("decoder.token_embedding.weight", (n_vocab, dt), True)]
    for i in range(n_tlayer):
        p = f"decoder.blocks.{i}."
        for a in ("attn", "cross_attn"):
            out += [(p + a + ".query.weight", (dt, dt), True), (p + a + ".query.bias", (dt,), False),
                    (p + a + ".key.weight", (dt, dt), True),
                    (p + a + ".value.weight", (dt, dt), True), (p + a + ".value.bias", (dt,), False),
                    (p + a + ".out.weight", (dt, dt), True), (p + a + ".out.bias", (dt,), False),
                    (p + a + "_ln.weight", (dt,), False), (p + a + "_ln.bias", (dt,), False)]
        out += [(p + "mlp.0.weight", (4 * dt, dt), True), (p + "mlp.0.bias", (4 * dt,), False),
                (p + "mlp.2.weight", (dt, 4 * dt), True), (p + "mlp.2.bias", (dt,), False),
                (p + "mlp_ln.weight", (dt,), False), (p + "mlp_ln.bias", (dt,), False)]
    out += [("decoder.ln.weight", (dt,), False), ("decoder.ln.bias", (dt,), False)]
    return out


def _sinusoids(length, channels, max_timescale=10000.0):
    inc = np.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2))
    t = np.arange(length)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


def _tensor_values(name, shape, rng, hp):
    """Scales chosen so activations stay O(1) (unit-variance linears, LN gains ~1) and
    greedy decoding is non-degenerate: the tied token embedding is small (0.1) so the
    fed-back token does not dominate its own logit, positions are strong (1.0), the
    decoder's residual branches are damped (0.5) except the last MLP (4.0), and the
    final LayerNorm gain 30/sqrt(d) gives logits std ~3 -- varied text tokens,
    timestamps, several segments and multi-window seeks (tuned against the reference)."""
    d = hp[2]
    n_text_layer = hp[8]
    if name == "encoder.positional_embedding":
        return _sinusoids(shape[0], shape[1])
    if name == "decoder.ln.weight":
        return (30.0 / np.sqrt(d) * (1.0 + 0.1 * rng.standard_normal(shape, dtype=np.float32))).astype(np.float32)
    if name.endswith("_ln.weight") or name == "encoder.ln_post.weight":
        return (1.0 + 0.1 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if name == "decoder.token_embedding.weight":
        return rng.standard_normal(shape, dtype=np.float32) * np.float32(0.1)
    if name == "decoder.positional_embedding":
        return rng.standard_normal(shape, dtype=np.float32) * np.float32(1.0)
    if name.endswith(".weight"):
        fan_in = int(np.prod(shape[1:]))
        gain = 1.0
        if name.startswith("decoder.") and (name.endswith("attn.out.weight") or name.endswith("mlp.2.weight")):
            gain = 4.0 if name == f"decoder.blocks.{n_text_layer - 1}.mlp.2.weight" else 0.5
        return rng.standard_normal(shape, dtype=np.float32) * np.float32(gain / np.sqrt(fan_in))
    # biases
    return rng.standard_normal(shape, dtype=np.float32) * np.float32(0.02)


def write_model(path: str, model: str, seed: int = 1234) -> str:
    """Write a synthetic ggml-bin model; returns its SHA-256 hex digest."""
    hp = MODELS[model]
    n_vocab = hp[0]
    multilingual = n_vocab >= 51865
    rng = np.random.default_rng(seed)
    h = hashlib.sha256()
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        def w(b):
            f.write(b)
            h.update(b)
        w(struct.pack("<I", GGML_FILE_MAGIC))
        w(struct.pack("<11i", *hp, 1))  # ftype 1 = mostly F16
        filt = mel_filters(hp[9])
        w(struct.pack("<ii", *filt.shape))
        w(np.ascontiguousarray(filt, dtype="<f4").tobytes())
        w(vocab_bytes(multilingual))
        for name, shape, f16 in tensor_list(hp):
            vals = _tensor_values(name, shape, rng, hp)
            arr = vals.astype(np.float16 if f16 else np.float32)
            nb = name.encode()
            w(struct.pack("<iii", len(shape), len(nb), 1 if f16 else 0))
            w(struct.pack("<%di" % len(shape), *reversed(shape)))
            w(nb)
            w(arr.tobytes())
    os.replace(tmp, path)
    return h.hexdigest()


def q5_0_blocks(x: np.ndarray) -> bytes:
    """ggml Q5_0 blocks (22 B per 32 weights) of a row-major f32 tensor, restating
    quantize_row_q5_0_ref (/root/reference ggml/src/ggml-quants.c:110-152): d = max / -16 with
    max the first largest-magnitude value, q = min(31, (int8)(x / d + 16.5)), 4 low bits packed
    in nibbles (element j low, j + 16 high), 5th bits in a little-endian u32."""
    b = np.ascontiguousarray(x, np.float32).reshape(-1, 32)
    am = np.argmax(np.abs(b), axis=1)
    mx = b[np.arange(len(b)), am]
    d = (mx / np.float32(-16.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1.0) / d, np.float32(0.0)).astype(np.float32)
    # x * id + 16.5f is one fused multiply-add in the reference build (gcc contracts it on
    # FMA targets): the product is exact in double, so a single rounding to f32 follows
    xs = (b.astype(np.float64) * idv.astype(np.float64)[:, None] + 16.5).astype(np.float32)
    xi = np.minimum(31, np.trunc(xs).astype(np.int64).astype(np.int8).astype(np.int64) & 0xFF).astype(np.uint8)
    qs = (xi[:, :16] & 0x0F) | ((xi[:, 16:] & 0x0F) << 4)
    bits = ((xi >> 4) & 1).astype(np.uint32)
    qh = (bits << np.arange(32, dtype=np.uint32)[None, :]).sum(axis=1, dtype=np.uint64).astype("<u4")
    out = np.zeros((len(b), 22), np.uint8)
    out[:, 0:2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 2:6] = qh.view(np.uint8).reshape(-1, 4)
    out[:, 6:22] = qs
    return out.tobytes()


def q4_0_blocks(x: np.ndarray) -> bytes:
    """ggml Q4_0 blocks (18 B per 32 weights), restating quantize_row_q4_0_ref
    (/root/reference ggml/src/ggml-quants.c:36-71): d = max / -8 with max the first
    largest-magnitude value, q = min(15, (int8)(x / d + 8.5)) (the multiply-add contracted to
    one FMA as in q5_0_blocks), element j low nibble, j + 16 high nibble of byte j."""
    b = np.ascontiguousarray(x, np.float32).reshape(-1, 32)
    am = np.argmax(np.abs(b), axis=1)
    mx = b[np.arange(len(b)), am]
    d = (mx / np.float32(-8.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1.0) / d, np.float32(0.0)).astype(np.float32)
    xs = (b.astype(np.float64) * idv.astype(np.float64)[:, None] + 8.5).astype(np.float32)
    xi = np.minimum(15, np.trunc(xs).astype(np.int64).astype(np.int8).astype(np.int64) & 0xFF).astype(np.uint8)
    qs = (xi[:, :16] & 0x0F) | ((xi[:, 16:] & 0x0F) << 4)
    out = np.zeros((len(b), 18), np.uint8)
    out[:, 0:2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 2:18] = qs
    return out.tobytes()


def _minmax_blocks(x: np.ndarray, nbits: int):
    """Shared part of quantize_row_q4_1_ref / quantize_row_q5_1_ref (ref ggml/src/ggml-quants.c:
    73-108, 154-196): d = (max - min) / (2^nbits - 1), id = 1/d, x' = (x - min) * id, and
    x' + 0.5f -- the multiply and add contracted to one FMA by gcc (as for Q5_0), so the
    quantized value is trunc(f32(f64(x - min) * id + 0.5))."""
    b = np.ascontiguousarray(x, np.float32).reshape(-1, 32)
    mn = b.min(axis=1)
    mx = b.max(axis=1)
    d = ((mx - mn) / np.float32((1 << nbits) - 1)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1.0) / d, np.float32(0.0)).astype(np.float32)
    t = (b - mn[:, None]).astype(np.float32)
    xs = (t.astype(np.float64) * idv.astype(np.float64)[:, None] + 0.5).astype(np.float32)
    return b, d, mn, xs


def q4_1_blocks(x: np.ndarray) -> bytes:
    """ggml Q4_1 blocks (20 B per 32 weights: d f16, m f16, qs[16]), restating
    quantize_row_q4_1_ref (ref ggml/src/ggml-quants.c:73-108): q = min(15, (int8)(x' + 0.5)),
    element j low nibble, j + 16 high nibble of byte j."""
    b, d, mn, xs = _minmax_blocks(x, 4)
    xi = np.minimum(15, np.trunc(xs).astype(np.int64).astype(np.int8).astype(np.int64) & 0xFF).astype(np.uint8)
    qs = (xi[:, :16] & 0x0F) | ((xi[:, 16:] & 0x0F) << 4)
    out = np.zeros((len(b), 20), np.uint8)
    out[:, 0:2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = mn.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 4:20] = qs
    return out.tobytes()


def q5_1_blocks(x: np.ndarray) -> bytes:
    """ggml Q5_1 blocks (24 B per 32 weights: d f16, m f16, qh u32, qs[16]), restating
    quantize_row_q5_1_ref (ref ggml/src/ggml-quants.c:154-196): q = (uint8)(x' + 0.5), 4 low
    bits in nibbles, 5th bits in a little-endian u32."""
    b, d, mn, xs = _minmax_blocks(x, 5)
    xi = (np.trunc(xs).astype(np.int64) & 0xFF).astype(np.uint8)
    qs = (xi[:, :16] & 0x0F) | ((xi[:, 16:] & 0x0F) << 4)
    bits = ((xi >> 4) & 1).astype(np.uint32)
    qh = (bits << np.arange(32, dtype=np.uint32)[None, :]).sum(axis=1, dtype=np.uint64).astype("<u4")
    out = np.zeros((len(b), 24), np.uint8)
    out[:, 0:2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = mn.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 4:8] = qh.view(np.uint8).reshape(-1, 4)
    out[:, 8:24] = qs
    return out.tobytes()


def q8_0_blocks(x: np.ndarray) -> bytes:
    """block_q8_0 rows of f32 values: quantize_row_q8_0_ref (ref ggml/src/ggml-quants.c:199-222):
    d = amax / 127 (stored f16), q = roundf(x * (1/d)) (round half away from zero)."""
    b = x.astype(np.float32).reshape(-1, 32)
    amax = np.abs(b).max(axis=1)
    d = (amax / np.float32(127.0)).astype(np.float32)
    idv = np.where(d != 0, np.float32(1.0) / np.where(d != 0, d, np.float32(1.0)), np.float32(0.0)).astype(np.float32)
    x0 = (b * idv[:, None]).astype(np.float32)
    q = (np.sign(x0) * np.floor(np.abs(x0) + np.float32(0.5))).astype(np.int8)
    out = np.zeros((b.shape[0], 34), np.uint8)
    out[:, 0:2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    out[:, 2:34] = q.view(np.uint8)
    return out.tobytes()


def quantize_q8_0(src: str, dst: str) -> str:
    """Q8_0 copy of an F16 ggml-bin model as whisper-quantize writes it (same tensor rule as
    quantize_q5_0; ttype 8, ftype 2007 = GGML_QNT_VERSION 2 * 1000 + MOSTLY_Q8_0 7)."""
    return quantize_q5_0(src, dst, kind="q8_0")


def quantize_q4_0(src: str, dst: str) -> str:
    """Q4_0 copy (ttype 2, ftype 2002 = GGML_QNT_VERSION 2 * 1000 + MOSTLY_Q4_0 2)."""
    return quantize_q5_0(src, dst, kind="q4_0")


def quantize_q4_1(src: str, dst: str) -> str:
    """Q4_1 copy (ttype 3, ftype 2003 = GGML_QNT_VERSION 2 * 1000 + MOSTLY_Q4_1 3)."""
    return quantize_q5_0(src, dst, kind="q4_1")


def quantize_q5_1(src: str, dst: str) -> str:
    """Q5_1 copy (ttype 7, ftype 2009 = GGML_QNT_VERSION 2 * 1000 + MOSTLY_Q5_1 9)."""
    return quantize_q5_0(src, dst, kind="q5_1")


_QKIND = {"q5_0": (8, 6, q5_0_blocks), "q8_0": (7, 8, q8_0_blocks), "q4_0": (2, 2, q4_0_blocks),
          "q4_1": (3, 3, q4_1_blocks), "q5_1": (9, 7, q5_1_blocks)}  # ftype, ttype


def quantize_q5_0(src: str, dst: str, kind: str = "q5_0") -> str:
    """Q5_0 copy of an F16 ggml-bin model, as whisper-quantize writes it
    (/root/reference examples/quantize/quantize.cpp:159-168, examples/common-ggml.cpp:97-230):
    every 2-D tensor except the positional embeddings becomes Q5_0 (ttype 6), ftype becomes
    2008 (GGML_QNT_VERSION 2 * 1000 + MOSTLY_Q5_0 8). Returns the SHA-256."""
    skip = {"encoder.conv1.bias", "encoder.conv2.bias", "encoder.positional_embedding", "decoder.positional_embedding"}
    raw = open(src, "rb").read()
    off = 0

    def take(n):
        nonlocal off
        v = raw[off:off + n]
        off += n
        return v
    h = hashlib.sha256()
    tmp = f"{dst}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        def w(b):
            f.write(b)
            h.update(b)
        w(take(4))
        hp = list(struct.unpack("<11i", take(44)))
        hp[10] = 2000 + _QKIND[kind][0]
        w(struct.pack("<11i", *hp))
        n_mel, n_fft = struct.unpack("<ii", take(8))
        w(struct.pack("<ii", n_mel, n_fft))
        w(take(n_mel * n_fft * 4))
        n_vocab = struct.unpack("<i", raw[off:off + 4])[0]
        vstart = off
        off += 4
        for _ in range(n_vocab):
            ln = struct.unpack("<I", raw[off:off + 4])[0]
            off += 4 + ln
        w(raw[vstart:off])
        while off < len(raw):
            n_dims, name_len, ttype = struct.unpack("<iii", take(12))
            ne = struct.unpack("<%di" % n_dims, take(4 * n_dims))
            name = take(name_len)
            nel = int(np.prod(ne))
            data = take(nel * (2 if ttype == 1 else 4))
            quant = n_dims == 2 and name.decode() not in skip
            w(struct.pack("<iii", n_dims, name_len, _QKIND[kind][1] if quant else ttype))
            w(struct.pack("<%di" % n_dims, *ne))
            w(name)
            if quant:
                x = np.frombuffer(data, "<f2" if ttype == 1 else "<f4").astype(np.float32)
                w(_QKIND[kind][2](x))
            else:
                w(data)
    os.replace(tmp, dst)
    return h.hexdigest()


def _stamp_path(path: str) -> str:
    return path + ".stamp"


def _cached_ok(path: str) -> bool:
    """A cache file is reused only if the stamp written after its generation completed exists
    and records the file's current size (a file left by a killed or concurrent writer is not)."""
    try:
        with open(_stamp_path(path)) as f:
            st = json.load(f)
        return os.path.getsize(path) == st["size"]
    except (OSError, ValueError, KeyError):
        return False


def _stamp(path: str, sha: str) -> None:
    with open(_stamp_path(path) + f".tmp{os.getpid()}", "w") as f:
        json.dump({"size": os.path.getsize(path), "sha256": sha}, f)
    os.replace(_stamp_path(path) + f".tmp{os.getpid()}", _stamp_path(path))


def file_sha256(path: str) -> str:
    """SHA-256 of a model file (from its generation stamp when valid, else computed)."""
    if _cached_ok(path):
        with open(_stamp_path(path)) as f:
            return json.load(f)["sha256"]
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def ensure_model(model: str, seed: int = 1234, cache_dir: str | None = None) -> str:
    """Path to a cached synthetic model (generated on first use; regenerated when its
    generation stamp is missing or does not match the file)."""
    cache_dir = cache_dir or os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache_dir, exist_ok=True)
    kind = next((k for k in ("q5_0", "q8_0", "q4_0", "q4_1", "q5_1") if model.endswith("-" + k)), None)
    base = model[:-5] if kind else model
    path = os.path.join(cache_dir, f"synth-{base}-s{seed}.bin")
    if not _cached_ok(path):
        _stamp(path, write_model(path, base, seed))
    if kind:
        qpath = os.path.join(cache_dir, f"synth-{base}-{kind}-s{seed}.bin")
        if not _cached_ok(qpath):
            _stamp(qpath, quantize_q5_0(path, qpath, kind=kind))
        return qpath
    return path


def synth_audio(n_samples: int, seed: int) -> np.ndarray:
    """Speech-like synthetic 16 kHz mono clip: band-limited noise x syllabic AM envelope,
    with voiced harmonic bursts; peak <= 0.5."""
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples) / 16000.0
    noise = rng.standard_normal(n_samples)
    # crude band-limit: moving-average difference (~300-3400 Hz emphasis)
    k1 = np.ones(3) / 3.0
    k2 = np.ones(24) / 24.0
    bl = np.convolve(noise, k1, "same") - np.convolve(noise, k2, "same")
    f0 = 110.0 + 40.0 * np.sin(2 * np.pi * 0.3 * t + rng.uniform(0, 6.28))
    phase = 2 * np.pi * np.cumsum(f0) / 16000.0
    voiced = sum(np.sin(k * phase) / k for k in range(1, 8))
    env = np.clip(np.sin(2 * np.pi * 3.5 * t + rng.uniform(0, 6.28)), 0, None) ** 2
    env *= (np.sin(2 * np.pi * 0.2 * t + rng.uniform(0, 6.28)) > -0.3)
    x = env * (0.6 * voiced + 0.8 * bl)
    x = x / (np.max(np.abs(x)) + 1e-9) * 0.5
    return x.astype(np.float32)


def read_wav_16k_mono(path: str) -> np.ndarray:
    """Minimal PCM16 WAV reader (16 kHz mono) -> float32 in [-1, 1)."""
    b = open(path, "rb").read()
    assert b[:4] == b"RIFF" and b[8:12] == b"WAVE"
    off = 12
    fmt = None
    while off < len(b):
        cid, sz = b[off:off + 4], struct.unpack_from("<I", b, off + 4)[0]
        if cid == b"fmt ":
            fmt = struct.unpack_from("<HHIIHH", b, off + 8)
        elif cid == b"data":
            assert fmt is not None and fmt[0] == 1 and fmt[1] == 1 and fmt[2] == 16000 and fmt[5] == 16
            return (np.frombuffer(b, dtype="<i2", count=sz // 2, offset=off + 8) / 32768.0).astype(np.float32)
        off += 8 + sz + (sz & 1)
    raise ValueError("no data chunk")
