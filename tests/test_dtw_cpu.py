"""CPU: the DTW token-timestamp algorithm of the engine (owk_debug_dtw -> timestamps.cpp
dtw_time_indices: ggml_norm over tokens, width-7 reflect median filter, mean over heads,
DTW + backtrace, per-token placement) fed with the REFERENCE's own captured alignment-head
attention (state->aheads_cross_QKs_data of its DTW re-decode, make_golden_nofa.py)
reproduces the reference's t_dtw exactly. No GPU needed: this pins the algorithm; the GPU
test (test_gpu_nofa.py) then compares end to end."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import owk

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("model", ["tiny.en", "tiny", "l3-mini"])
def test_dtw_matches_reference(model):
    meta = json.load(open(os.path.join(GOLDEN, "nofa_golden.json")))
    arr = np.load(os.path.join(GOLDEN, "nofa_golden.npz"))
    key = f"{model}/jfk"
    din = meta["results"][key + "/dtw_in"]
    cap = np.ascontiguousarray(arr[key + "/dtw_cap"], np.float32)
    segs = meta["results"][key + "/full/greedy_dtw"]["segments"]
    n_frames = din["n_frames"]  # min(3000, best decoder seek_delta, seek_end) (ref whisper.cpp:7748)
    L = owk.load()
    L.owk_debug_dtw.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.POINTER(C.c_int), C.c_int]
    out = np.zeros(4096, np.int32)
    n = L.owk_debug_dtw(cap.ctypes.data_as(C.POINTER(C.c_float)), din["n_ah"], 1500, din["n_tok"], din["sot_len"],
                        n_frames, 7, out.ctypes.data_as(C.POINTER(C.c_int)), len(out))
    assert n >= 0
    eot = 50256 if model.endswith(".en") else 50257
    want = [t[8] for s in segs for t in s["tokens"] if t[0] < eot]
    got = [2 * int(x) for x in out[:n]][: len(want)]  # seek = 0
    assert got == want
