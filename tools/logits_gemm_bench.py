"""Device us per launch of the logits-shaped decode GEMM (M rows x 51866 x 1280, EPI_F32) through the
engine dispatch: `OWK_ROWS_NT=<n> python tools/logits_gemm_bench.py` (the env picks the column tiles
per block)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "open-whisper-kit_amd", "python"))
import owk  # noqa: E402

L = owk.load()
L.owk_debug_gemm_bench.restype = C.c_double
L.owk_debug_gemm_bench.argtypes = [C.c_int] * 6
for M in (32, 8):
    t = min(L.owk_debug_gemm_bench(0, 7 | 0x200, M, 51866, 1280, 50) for _ in range(3))
    print(f"NT={os.environ.get('OWK_ROWS_NT', '0')} M={M}: {t:.2f} us ({51866 * 1280 * 2 / t / 1e3:.0f} GB/s of weights)")
