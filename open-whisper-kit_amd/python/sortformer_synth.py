"""Synthetic-weight streaming-SortFormer models in the reference's GGUF v3 format.

No real SortFormer weights exist offline, so parity and throughput run on
deterministic synthetic weights written in exactly the layout the reference loader reads
(sortformer_init, /root/reference streaming-sortformer/src/sortformer.cpp:287-626):

* metadata keys and values of the reference converter (scripts/convert_to_gguf.py:251-280);
* tensor names of sortformer.cpp:425-572, PyTorch shapes (GGUF stores ne reversed);
* dtypes per the converter: preprocessor.featurizer.fb / .window F32, everything else F16
  (the depthwise conv already BatchNorm-fused, convert_to_gguf.py:177-207).

The 128 x 257 filterbank is the Slaney-normalised librosa mel basis NeMo uses
(n_fft 512, sr 16 kHz, fmin 0, fmax 8 kHz), the window a symmetric 400-point Hann.
Same seed => byte-identical file on any machine (numpy PCG64); the golden fixtures
record the SHA-256.
"""
from __future__ import annotations

import hashlib
import os
import struct

import numpy as np

from owk_synth import slaney_mel_filters

GGUF_TYPE_UINT32 = 4
GGUF_TYPE_FLOAT32 = 6
GGUF_TYPE_STRING = 8
GGML_TYPE_F32 = 0
GGML_TYPE_F16 = 1
ALIGN = 32

N_CONF, D, H, DFF, KCONV = 17, 512, 8, 2048, 9
N_TRANS, TD, TFF = 18, 192, 768
C_SUB = 256


def tensor_list(n_conf: int = N_CONF, n_trans: int = N_TRANS):
    """(name, numpy shape) in the order they are written."""
    out = [("preprocessor.featurizer.fb", (128, 257)),
           ("preprocessor.featurizer.window", (400,)),
           ("encoder.pre_encode.conv.0.weight", (C_SUB, 1, 3, 3)), ("encoder.pre_encode.conv.0.bias", (C_SUB,)),
           ("encoder.pre_encode.conv.2.weight", (C_SUB, 1, 3, 3)), ("encoder.pre_encode.conv.2.bias", (C_SUB,)),
           ("encoder.pre_encode.conv.3.weight", (C_SUB, C_SUB, 1, 1)), ("encoder.pre_encode.conv.3.bias", (C_SUB,)),
           ("encoder.pre_encode.conv.5.weight", (C_SUB, 1, 3, 3)), ("encoder.pre_encode.conv.5.bias", (C_SUB,)),
           ("encoder.pre_encode.conv.6.weight", (C_SUB, C_SUB, 1, 1)), ("encoder.pre_encode.conv.6.bias", (C_SUB,)),
           ("encoder.pre_encode.out.weight", (D, C_SUB * 16)), ("encoder.pre_encode.out.bias", (D,))]
    for i in range(n_conf):
        p = f"encoder.layers.{i}."
        for ff in ("feed_forward1", "feed_forward2"):
            n = "norm_" + ff
            out += [(p + n + ".weight", (D,)), (p + n + ".bias", (D,)),
                    (p + ff + ".linear1.weight", (DFF, D)), (p + ff + ".linear1.bias", (DFF,)),
                    (p + ff + ".linear2.weight", (D, DFF)), (p + ff + ".linear2.bias", (D,))]
        out += [(p + "norm_self_att.weight", (D,)), (p + "norm_self_att.bias", (D,))]
        for lin in ("linear_q", "linear_k", "linear_v", "linear_out"):
            out += [(p + f"self_attn.{lin}.weight", (D, D)), (p + f"self_attn.{lin}.bias", (D,))]
        out += [(p + "self_attn.linear_pos.weight", (D, D)),
                (p + "self_attn.pos_bias_u", (H, D // H)), (p + "self_attn.pos_bias_v", (H, D // H)),
                (p + "norm_conv.weight", (D,)), (p + "norm_conv.bias", (D,)),
                (p + "conv.pointwise_conv1.weight", (2 * D, D, 1)), (p + "conv.pointwise_conv1.bias", (2 * D,)),
                (p + "conv.depthwise_conv.weight", (D, 1, KCONV)), (p + "conv.depthwise_conv.bias", (D,)),
                (p + "conv.pointwise_conv2.weight", (D, D, 1)), (p + "conv.pointwise_conv2.bias", (D,)),
                (p + "norm_out.weight", (D,)), (p + "norm_out.bias", (D,))]
    out += [("sortformer_modules.encoder_proj.weight", (TD, D)), ("sortformer_modules.encoder_proj.bias", (TD,))]
    for i in range(n_trans):
        p = f"transformer_encoder.layers.{i}."
        for lin in ("query_net", "key_net", "value_net", "out_projection"):
            out += [(p + f"first_sub_layer.{lin}.weight", (TD, TD)), (p + f"first_sub_layer.{lin}.bias", (TD,))]
        out += [(p + "layer_norm_1.weight", (TD,)), (p + "layer_norm_1.bias", (TD,)),
                (p + "second_sub_layer.dense_in.weight", (TFF, TD)), (p + "second_sub_layer.dense_in.bias", (TFF,)),
                (p + "second_sub_layer.dense_out.weight", (TD, TFF)), (p + "second_sub_layer.dense_out.bias", (TD,)),
                (p + "layer_norm_2.weight", (TD,)), (p + "layer_norm_2.bias", (TD,))]
    out += [("sortformer_modules.first_hidden_to_hidden.weight", (TD, TD)),
            ("sortformer_modules.first_hidden_to_hidden.bias", (TD,)),
            ("sortformer_modules.single_hidden_to_spks.weight", (4, TD)),
            ("sortformer_modules.single_hidden_to_spks.bias", (4,))]
    return out


# residual-branch output projections: damped so the identity path carries the per-frame
# variation of the input through 17 + 18 layers (random-init deep stacks otherwise wash it out)
BRANCH_OUT = ("linear2.weight", "self_attn.linear_out.weight", "conv.pointwise_conv2.weight",
              "first_sub_layer.out_projection.weight", "second_sub_layer.dense_out.weight")
BRANCH_GAIN = 0.1
SPK_GAIN = 30.0
SPK_BIAS = (-4.9, -10.1, 0.56, 3.84)  # centred on test.wav (sortformer diarize, reference)


def _values(name: str, shape, rng) -> np.ndarray:
    """Unit-variance linears, LayerNorm gains ~1, small biases; the speaker head is scaled so
    the four sigmoid outputs spread over (0, 1) and cross the 0.5 / silence thresholds, which
    exercises every AOSC branch (speaker-cache compression, silence profile, top-k boosts)."""
    if name == "preprocessor.featurizer.fb":
        return slaney_mel_filters(128, sr=16000, n_fft=512)
    if name == "preprocessor.featurizer.window":
        n = np.arange(400, dtype=np.float64)
        return (0.5 - 0.5 * np.cos(2.0 * np.pi * n / 399.0)).astype(np.float32)
    if "norm" in name or "layer_norm" in name:
        if name.endswith(".weight"):
            return (1.0 + 0.1 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
        return (0.05 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if name.endswith("pos_bias_u") or name.endswith("pos_bias_v"):
        return (0.1 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if name.endswith(".weight"):
        fan_in = int(np.prod(shape[1:]))
        gain = 1.0
        if name.startswith("encoder.pre_encode.conv.0"):
            gain = 0.25   # log-mel inputs are O(10)
        if name == "sortformer_modules.single_hidden_to_spks.weight":
            gain = SPK_GAIN
        if any(name.endswith(x) for x in BRANCH_OUT):
            gain = BRANCH_GAIN
        return (rng.standard_normal(shape, dtype=np.float32) * np.float32(gain / np.sqrt(fan_in))).astype(np.float32)
    if name == "sortformer_modules.single_hidden_to_spks.bias":
        return np.array(SPK_BIAS, np.float32)
    return (0.02 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)


def _gguf_str(s: str) -> bytes:
    b = s.encode()
    return struct.pack("<Q", len(b)) + b


def write_model(path: str, seed: int = 4321, n_conf: int = N_CONF, n_trans: int = N_TRANS) -> str:
    """Write a synthetic SortFormer GGUF; returns its SHA-256 hex digest."""
    rng = np.random.default_rng(seed)
    kv = [("general.architecture", GGUF_TYPE_STRING, "sortformer"),
          ("sortformer.mel.n_mels", GGUF_TYPE_UINT32, 128),
          ("sortformer.mel.n_fft", GGUF_TYPE_UINT32, 512),
          ("sortformer.mel.hop_length", GGUF_TYPE_UINT32, 160),
          ("sortformer.mel.win_length", GGUF_TYPE_UINT32, 400),
          ("sortformer.mel.sample_rate", GGUF_TYPE_UINT32, 16000),
          ("sortformer.mel.dither", GGUF_TYPE_FLOAT32, 1e-5),
          ("sortformer.encoder.n_layers", GGUF_TYPE_UINT32, n_conf),
          ("sortformer.encoder.d_model", GGUF_TYPE_UINT32, D),
          ("sortformer.encoder.n_heads", GGUF_TYPE_UINT32, H),
          ("sortformer.encoder.conv_kernel_size", GGUF_TYPE_UINT32, KCONV),
          ("sortformer.encoder.ff_expansion", GGUF_TYPE_UINT32, 4),
          ("sortformer.encoder.subsampling_factor", GGUF_TYPE_UINT32, 8),
          ("sortformer.encoder.subsampling_conv_channels", GGUF_TYPE_UINT32, C_SUB),
          ("sortformer.encoder.pos_emb_max_len", GGUF_TYPE_UINT32, 5000),
          ("sortformer.transformer.n_layers", GGUF_TYPE_UINT32, n_trans),
          ("sortformer.transformer.d_model", GGUF_TYPE_UINT32, TD),
          ("sortformer.transformer.n_heads", GGUF_TYPE_UINT32, 8),
          ("sortformer.transformer.ff_inner", GGUF_TYPE_UINT32, TFF),
          ("sortformer.n_speakers", GGUF_TYPE_UINT32, 4)]
    tensors = []
    for name, shape in tensor_list(n_conf, n_trans):
        v = _values(name, shape, rng)
        f32 = name.startswith("preprocessor.featurizer.")
        tensors.append((name, shape, np.ascontiguousarray(v.astype(np.float32 if f32 else np.float16))))

    head = bytearray()
    head += b"GGUF" + struct.pack("<IQQ", 3, len(tensors), len(kv))
    for k, t, v in kv:
        head += _gguf_str(k) + struct.pack("<i", t)
        if t == GGUF_TYPE_STRING:
            head += _gguf_str(v)
        elif t == GGUF_TYPE_UINT32:
            head += struct.pack("<I", v)
        else:
            head += struct.pack("<f", v)
    off = 0
    for name, shape, arr in tensors:
        head += _gguf_str(name) + struct.pack("<I", len(shape))
        head += struct.pack("<%dQ" % len(shape), *reversed(shape))
        head += struct.pack("<iQ", GGML_TYPE_F32 if arr.dtype == np.float32 else GGML_TYPE_F16, off)
        off += (arr.nbytes + ALIGN - 1) // ALIGN * ALIGN
    head += b"\0" * ((-len(head)) % ALIGN)

    h = hashlib.sha256()
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(head)
        h.update(head)
        for _, _, arr in tensors:
            b = arr.tobytes() + b"\0" * ((-arr.nbytes) % ALIGN)
            f.write(b)
            h.update(b)
    os.replace(tmp, path)
    return h.hexdigest()


def ensure_model(seed: int = 4321, cache_dir: str | None = None) -> str:
    cache_dir = cache_dir or os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache_dir, exist_ok=True)
    path = os.path.join(cache_dir, f"synth-sortformer-s{seed}.gguf")
    if not os.path.exists(path):
        write_model(path, seed)
    return path
