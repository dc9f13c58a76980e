"""OWK_BACKTRACE=1 crash handler of libwhisper.so (whisper_api.cpp): a child process that loads the library
and faults prints the fault, one line per frame (mapped file + file offset) and the mappings around the
fault address, with async-signal-safe calls only, then dies of the same signal. An abort (SIGABRT) prints
the frames without the maps dump. CPU only: loading the library needs no GPU."""
import os
import signal
import subprocess
import sys

import pytest

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "open-whisper-kit_amd", "lib",
                   "libwhisper.so")

CHILD = r"""
import ctypes, os, sys
ctypes.CDLL(sys.argv[1])
if sys.argv[2] == "segv":
    ctypes.string_at(16)
else:
    os.abort()
"""


@pytest.mark.parametrize("kind,sig", [("segv", signal.SIGSEGV), ("abort", signal.SIGABRT)])
def test_crash_handler_prints_frames(kind, sig):
    if not os.path.exists(LIB):
        pytest.skip("libwhisper.so not built")
    env = dict(os.environ, OWK_BACKTRACE="1")
    r = subprocess.run([sys.executable, "-c", CHILD, LIB, kind], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == -sig, (r.returncode, r.stderr[-2000:])
    err = r.stderr
    assert f"[owk] fatal signal {hex(int(sig))}" in err, err[-2000:]
    assert "[owk] native backtrace (mapped file + file offset):" in err
    frames = [ln for ln in err.splitlines() if ln.startswith("  0x")]
    assert len(frames) >= 3 and any("libwhisper.so+0x" in ln or "python" in ln for ln in frames), frames[:8]
    assert ("/proc/self/maps around the fault address" in err) == (kind == "segv")
