"""Large (encoder / cross-KV) GEMM on the GPU: correctness of the 256x256 ring kernel against a
float64 numpy product of the same f16 operands, then device time of both large-GEMM kernels on
the encoder shapes of large-v3 at 32 clips (random operands, interleaved rounds in one process).

    python tools/gemm_big_check.py            -> JSON lines on stdout
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk  # noqa: E402

EPI = {"f32": 7, "resid": 2, "gelu": 1, "f16": 0}  # kernels.h EPI_* (EPI_F32 = 7, EPI_RESID_F32 = 2, EPI_GELU_F16 = 1)
SHAPES = {  # name: (M, N, K, epilogue) -- large-v3 encoder at 32 clips x 1500 positions
    "qkv": (48000, 3840, 1280, "f32"),
    "o_proj": (48000, 1280, 1280, "resid"),
    "mlp0": (48000, 5120, 1280, "f32"),
    "mlp0_gelu": (48000, 5120, 1280, "gelu"),
    "mlp0_f16": (48000, 5120, 1280, "f16"),
    "mlp1": (48000, 1280, 5120, "resid"),
    "cross_kv": (48000, 2560, 1280, "f32"),
    "conv2": (48000, 1280, 3840, "f32"),
}


def main():
    L = owk.load()
    L.owk_debug_gemm_bench.restype = C.c_double
    L.owk_debug_gemm_bench.argtypes = [C.c_int] * 6
    L.owk_debug_gemm.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_uint16)] * 2 + [C.POINTER(C.c_float)]
    rng = np.random.default_rng(0)
    for M, N, K in [(4100, 1280, 1280), (3000, 2560, 640), (2048, 1024, 128), (6000, 1536, 5120)]:
        a = rng.uniform(-1, 1, (M, K)).astype(np.float16)
        w = rng.uniform(-1, 1, (N, K)).astype(np.float16)
        out = np.zeros((M, N), np.float32)
        P = lambda x: x.view(np.uint16).ctypes.data_as(C.POINTER(C.c_uint16))
        rc = L.owk_debug_gemm(0, M, N, K, P(a), P(w), out.ctypes.data_as(C.POINTER(C.c_float)))
        ref = a.astype(np.float64) @ w.astype(np.float64).T
        err = float(np.abs(out - ref).max())
        print(json.dumps({"check": [M, N, K], "rc": rc, "max_abs_err": err, "ok": bool(rc == 0 and err < 1e-3 * np.sqrt(K))}),
              flush=True)
    res = {}
    for rnd in range(3):
        for name, (M, N, K, epi) in SHAPES.items():
            for kern, flag in (("256", 0), ("8phase", 0x800), ("128", 0x100)):
                mode = EPI[epi] | 0x200 | max(flag, 0) if flag >= 0 else EPI[epi]
                us = L.owk_debug_gemm_bench(0, mode, M, N, K, 10)
                res.setdefault((name, kern), []).append(us)
    for (name, kern), v in res.items():
        M, N, K, _ = SHAPES[name]
        us = float(np.median(v))
        print(json.dumps({"gemm": name, "kernel": kern, "M": M, "N": N, "K": K, "us": round(us, 1),
                          "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
