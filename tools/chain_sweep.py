"""Decoder matmul/LayerNorm chain (no attention) of a large-v3-shaped model on the GPU, per variant:
owk_debug_decode_chain (R rows, 32 layers of distinct weights, one captured hipGraph) in one child
process per environment setting (the launchers read their OWK_GR_* overrides once).
    python tools/chain_sweep.py [R] > table
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
VARIANTS = [{}]


def child(R):
    sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
    import owk
    L = owk.load()
    L.owk_debug_decode_chain.restype = C.c_double
    L.owk_debug_decode_chain.argtypes = [C.c_int] * 4
    print(json.dumps({"us_per_layer": min(L.owk_debug_decode_chain(0, R, 32, 20) for _ in range(3))}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(int(sys.argv[2]))
        return
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    for v in VARIANTS + [json.loads(a) for a in sys.argv[2:]]:
        env = dict(os.environ, **v)
        r = subprocess.run([sys.executable, __file__, "child", str(R)], env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
        print(f"R={R} {json.dumps(v)} {line}", flush=True)


if __name__ == "__main__":
    main()
