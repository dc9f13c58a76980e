"""Encoder GEMM epilogue modes at the encoder's shape (M = 32 clips x 1500 rows, K = 1280): device time per
launch of k_gemm_8p for QKV_ENC / KV_CROSS (head-major outputs) against the plain F16 epilogue of the same N."""
import ctypes as C
import os

L = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "open-whisper-kit_amd/lib/libwhisper.so"))
L.owk_debug_gemm_bench.restype = C.c_double
L.owk_debug_gemm_bench.argtypes = [C.c_int] * 6
M, K = 48000, 1280
for mode, name, N in ((4, "QKV_ENC", 3840), (0, "F16", 3840), (5, "KV_CROSS", 2560), (0, "F16", 2560), (2, "RESID_F32", 1280)):
    us = min(L.owk_debug_gemm_bench(0, mode | 0x200, M, N, K, 10) for _ in range(3))
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    print(f"{name:9s} N={N:5d} {us:8.1f} us {2 * M * N * K / us / 1e6:7.1f} TFLOP/s  {us / -(-tiles // 256):6.2f} us per tile round", flush=True)
