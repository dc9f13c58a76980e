"""Host-side bookkeeping the GPU never touches, driven through the product libraries' host-only hooks
and pinned to the REFERENCE compiled in place (oracle/_ref, oracle/ref/ref_probe.cpp ref_kv_script and
oracle/ref/sf_probe.cpp ref_sf_aosc). tools/sanitize_tests.sh runs this file (with the tokenizer,
grammar, aligner, RTTM, DTW, k-quant and VAD CPU tests) against the ASan + UBSan build of both
libraries (make sanitize).

* KV cells (csrc/kv_cells.h; ref src/whisper.cpp:1019-1137): scripted find_slot / seq_rm / seq_cp /
  cell_max sequences shaped like whisper_full's -- a prompt in sequence 0, copies to the beam / best-of
  decoders, one token per decoder per step, decoders dropped and re-copied, a new window -- plus random
  scripts; every result, the head and every cell's (position, sequences) equal the reference's.
* AOSC (csrc/sortformer.cpp compress_spkcache / update_silence_profile; ref
  streaming-sortformer/src/sortformer.cpp:1729-1920): random speaker caches with predictions on a
  coarse grid (ties for the nth_element selections, values exactly at the 0.5 threshold) and silent
  popped frames; the compressed embeddings / predictions and the silence profile are bit-identical.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import owk

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF_SF = os.path.join(ROOT, "oracle", "_ref", "libsortformer_ref.so")
P = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
F = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))


def _kv_product(n_ctx, ops):
    L = owk.load()
    L.owk_debug_kv_cells.argtypes = [C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int), C.c_int]
    ops = np.ascontiguousarray(ops, np.int32).reshape(-1, 5)
    out = np.zeros(len(ops) + 1 + 2 * n_ctx, np.int32)
    assert L.owk_debug_kv_cells(n_ctx, P(ops), len(ops), P(out), len(out)) == len(out)
    return out


def _kv_reference(n_ctx, ops):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_oracle as R

    if not R.available():
        return None
    L = R.lib()
    L.ref_kv_script.argtypes = [C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int), C.c_int]
    ops = np.ascontiguousarray(ops, np.int32).reshape(-1, 5)
    out = np.zeros(len(ops) + 1 + 2 * n_ctx, np.int32)
    assert L.ref_kv_script(n_ctx, P(ops), len(ops), P(out), len(out)) == len(out)
    return out


def whisper_like_script(rng, n_dec):
    """the allocator calls of whisper_full_with_state for one clip (ref whisper.cpp:7157-7557): per window
    a prompt batch in sequence 0, seq_cp 0 -> j for the decoders, then per step one token per live
    decoder; beam search re-copies sequences between the decoders' KV (seq_rm + seq_cp through the
    spare sequences n_dec .. 2 n_dec - 1); completed decoders stop; a new window clears"""
    ops = []
    for _ in range(rng.integers(1, 3)):
        ops.append([4, 0, 0, 0, 0])
        n_prompt = int(rng.integers(1, 40))
        ops.append([0, n_prompt, 0, 0, 0])
        for j in range(1, n_dec):
            ops.append([1, j, -1, -1, 0])
            ops.append([2, 0, j, -1, -1])
        live = list(range(n_dec))
        pos = n_prompt
        for _ in range(rng.integers(5, 60)):
            for j in live:
                ops.append([0, 1, j, pos, 0])
            if n_dec > 1 and rng.random() < 0.5:  # beam reorder: decoder j takes decoder k's sequence
                j, k = rng.choice(live, 2) if len(live) > 1 else (live[0], live[0])
                tmp = n_dec + int(j)
                ops.append([1, tmp, -1, -1, 0])
                ops.append([2, int(k), tmp, -1, -1])
                ops.append([1, int(j), -1, -1, 0])
                ops.append([2, tmp, int(j), -1, -1])
                ops.append([1, tmp, -1, -1, 0])
            if len(live) > 1 and rng.random() < 0.05:
                live.remove(int(rng.choice(live)))
            ops.append([3, 0, 0, 0, 0])
            pos += 1
    return ops


def random_script(rng, n_ctx):
    ops = []
    for _ in range(200):
        k = rng.integers(0, 4)
        if k == 0:
            ops.append([0, int(rng.integers(1, 12)), int(rng.integers(0, 6)), int(rng.integers(-2, 40)), 0])
        elif k == 1:
            ops.append([1, int(rng.integers(-1, 6)), int(rng.integers(-1, 40)), int(rng.integers(-1, 60)), 0])
        elif k == 2:
            ops.append([2, int(rng.integers(0, 6)), int(rng.integers(0, 6)), int(rng.integers(-1, 40)),
                        int(rng.integers(-1, 60))])
        else:
            ops.append([3, 0, 0, 0, 0])
    return ops


def test_kv_cells_whisper_like_scripts_match_reference():
    rng = np.random.default_rng(5)
    have_ref = None
    for case in range(40):
        n_dec = int(rng.choice([1, 2, 5, 8]))
        n_ctx = 448 * (n_dec + 2 if n_dec > 1 else 1)  # ref whisper.cpp:7157-7175
        ops = whisper_like_script(rng, n_dec)
        got = _kv_product(n_ctx, ops)
        # invariants: every find_slot found a slot; no cell holds a sequence beyond 2 n_dec
        res = got[:len(ops)]
        assert all(r >= 0 for r, o in zip(res, ops) if o[0] == 0), case
        want = _kv_reference(n_ctx, ops)
        have_ref = want is not None
        if have_ref:
            np.testing.assert_array_equal(got, want, err_msg=f"case {case}")
    if not have_ref:
        pytest.skip("reference oracle not built: product invariants only")


def test_kv_cells_random_scripts_match_reference():
    rng = np.random.default_rng(11)
    for case in range(60):
        n_ctx = int(rng.choice([16, 40, 64]))
        ops = random_script(rng, n_ctx)
        got = _kv_product(n_ctx, ops)
        want = _kv_reference(n_ctx, ops)
        if want is None:
            pytest.skip("reference oracle not built")
        np.testing.assert_array_equal(got, want, err_msg=f"case {case}")


def test_kv_cells_rejects_invalid_records():
    L = owk.load()
    L.owk_debug_kv_cells.argtypes = [C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int), C.c_int]
    out = np.zeros(64, np.int32)
    for bad in ([9, 0, 0, 0, 0], [0, 1, 40, 0, 0], [2, 0, 33, 0, 0]):
        ops = np.array(bad, np.int32)
        assert L.owk_debug_kv_cells(8, P(ops), 1, P(out), len(out)) == -2
    ops = np.array([3, 0, 0, 0, 0], np.int32)
    assert L.owk_debug_kv_cells(8, P(ops), 1, P(out), 4) == -1


def _aosc(lib, name, d, embs, preds, mean_sil, n_sil, pop_e, pop_p, target, sil):
    fn = getattr(lib, name)
    fn.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int,
                   C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int, C.c_int,
                   C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    oe = np.zeros((target, d), np.float32)
    op = np.zeros((target, 4), np.float32)
    om = np.zeros(d, np.float32)
    r = fn(d, len(preds), F(embs), F(preds), F(mean_sil), n_sil, len(pop_p), F(pop_e), F(pop_p), target, sil,
           F(oe), F(op), F(om))
    return r, oe, op, om


def test_aosc_matches_reference():
    import sortformer as SF

    prod = SF.load()
    ref = C.CDLL(REF_SF) if os.path.exists(REF_SF) else None
    rng = np.random.default_rng(3)
    grid = np.array([0.0, 0.05, 0.1, 0.25, 0.3, 0.5, 0.5, 0.51, 0.7, 0.75, 0.9, 1.0], np.float32)
    n_cmp = 0
    for case in range(60):
        d = int(rng.choice([8, 32, 512]))
        target = int(rng.choice([16, 40, 188]))
        sil = int(rng.choice([0, 1, 3]))
        if target < (1 + sil) * 4:
            continue
        n = int(rng.integers(target - 2, 3 * target))
        # predictions on a coarse grid (nth_element ties, the 0.5 threshold) with some speakers mostly silent
        preds = grid[rng.integers(0, len(grid), (n, 4))]
        preds[:, int(rng.integers(0, 4))] *= rng.random() < 0.5
        embs = rng.standard_normal((n, d)).astype(np.float32)
        mean_sil = rng.standard_normal(d).astype(np.float32) * 0.1
        n_pop = int(rng.integers(0, 30))
        pop_p = grid[rng.integers(0, 4, (n_pop, 4))]  # mostly below the 0.2 silence threshold in sum
        pop_e = rng.standard_normal((n_pop, d)).astype(np.float32)
        args = (d, np.ascontiguousarray(embs), np.ascontiguousarray(preds), mean_sil, int(rng.integers(0, 50)),
                np.ascontiguousarray(pop_e), np.ascontiguousarray(pop_p), target, sil)
        got = _aosc(prod, "owk_sortformer_debug_aosc", *args)
        assert got[0] == (target if n > target else -1), case
        if ref is None:
            continue
        devnull = os.open(os.devnull, os.O_WRONLY)  # the reference logs each compression to stderr
        saved = os.dup(2)
        os.dup2(devnull, 2)
        try:
            want = _aosc(ref, "ref_sf_aosc", *args)
        finally:
            os.dup2(saved, 2)
            os.close(saved)
            os.close(devnull)
        assert got[0] == want[0], case
        for g, w in zip(got[1:], want[1:]):
            np.testing.assert_array_equal(g, w, err_msg=f"case {case}")
        n_cmp += 1
    if ref is None:
        pytest.skip("reference SortFormer oracle not built: product hook exercised only")
    assert n_cmp >= 30


def test_sanitized_build_is_instrumented():
    """when the libraries under test are the sanitizer build (tools/sanitize_tests.sh), they carry the
    ASan / UBSan runtime calls: the run is not silently against the plain build"""
    path = os.environ.get("OWK_LIB", "")
    if "/san/" not in path:
        pytest.skip("not the sanitizer run")
    syms = open(path, "rb").read()
    assert b"__asan_report_load" in syms and b"__ubsan_handle" in syms
