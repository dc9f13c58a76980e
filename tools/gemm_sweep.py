"""Decode-row GEMM tuning sweep on the GPU (one process per J/KS setting, env overrides).
    python tools/gemm_sweep.py            -> table on stdout
"""
import ctypes as C
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SHAPES = [(16, 32), (1280, 1280), (3840, 1280), (5120, 1280), (1280, 5120), (51866, 1280)]


def child(mode):
    sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
    import owk
    L = owk.load()
    L.owk_debug_gemm_bench.restype = C.c_double
    L.owk_debug_gemm_bench.argtypes = [C.c_int] * 6
    out = {}
    for N, K in SHAPES:
        out[f"{N}x{K}"] = L.owk_debug_gemm_bench(0, mode, 32, N, K, 200)
    print(json.dumps(out))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(int(sys.argv[2]))
        return
    for mode, j, ks in itertools.product([0, 8], [0, 2, 4, 8], [0, 2, 4]):
        env = dict(os.environ, OWK_GR_J=str(j), OWK_GR_KS=str(ks))
        r = subprocess.run([sys.executable, __file__, "child", str(mode)], env=env, capture_output=True, text=True,
                           timeout=120)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
        print(f"mode={mode} J={j} KS={ks} {line}", flush=True)


if __name__ == "__main__":
    main()
