"""Device us per launch of the decode-row GEMM shapes of large-v3 (32 rows) through the engine dispatch;
run under OWK_ROWS_NT / OWK_ROWS_NT_MIN_N to compare column tiles per block."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "open-whisper-kit_amd", "python"))
import owk  # noqa: E402

L = owk.load()
L.owk_debug_gemm_bench.restype = C.c_double
L.owk_debug_gemm_bench.argtypes = [C.c_int] * 6
tag = f"NT={os.environ.get('OWK_ROWS_NT', '0')} min_n={os.environ.get('OWK_ROWS_NT_MIN_N', '16384')}"
for mode, N, K, name in ((1, 5120, 1280, "mlp0+gelu"), (6, 3840, 1280, "qkv"), (0, 1280, 1280, "cross-q"),
                         (7, 51866, 1280, "logits")):
    t = min(L.owk_debug_gemm_bench(0, mode | 0x200, 32, N, K, 100) for _ in range(3))
    print(f"{tag} {name} N={N} K={K}: {t:.2f} us")
