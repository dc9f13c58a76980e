"""Encoder-shaped k_gemm_8p launches over K: per-tile fixed cost vs main-loop cost (owk_debug_gemm_bench)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
L = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "open-whisper-kit_amd/lib/libwhisper.so"))
L.owk_debug_gemm_bench.restype = C.c_double
L.owk_debug_gemm_bench.argtypes = [C.c_int] * 6
M = 48000
MODES = ((7, "F32"), (0, "F16"), (2, "RESID_F32"), (1, "GELU_F16"))
if len(sys.argv) > 1:
    MODES = tuple(m for m in MODES if m[1] in sys.argv[1:])
for mode, name in MODES:
    for N in (1280, 5120):
        pts = []
        for K in (256, 640, 1280, 2560, 5120):
            us = min(L.owk_debug_gemm_bench(0, mode | 0x200, M, N, K, 10) for _ in range(2))
            tiles = ((M + 255) // 256) * ((N + 255) // 256)
            rounds = tiles / 256
            pts.append((K, us / rounds))
            print(f"{name:10s} N={N:5d} K={K:5d} {us:9.1f} us  {2*M*N*K/us/1e6:7.1f} TFLOP/s  {us/rounds:7.2f} us per tile-round", flush=True)
        n = len(pts)
        mk = sum(k for k, _ in pts) / n
        mt = sum(t for _, t in pts) / n
        b = sum((k - mk) * (t - mt) for k, t in pts) / sum((k - mk) ** 2 for k, _ in pts)
        print(f"  fit: per tile-round {mt - b * mk:.2f} us fixed + {b * 64:.3f} us per 64-deep K step", flush=True)
