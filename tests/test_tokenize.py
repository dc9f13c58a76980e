"""whisper_tokenize parity (CPU, no device): the product tokenizer (csrc/model.cpp tokenize_text
over the vocabulary the product loader parses, through the host-only hook owk_debug_tokenize)
against the REFERENCE whisper_tokenize (ref src/whisper.cpp:3272-3320, 3957-3973).

* golden: tests/golden/tokenize_golden.json (make_golden_tokenize.py; 1,200 strings x the English
  and multilingual vocabularies, token ids bit-exact);
* live: when the compiled reference is present (oracle/_ref), a differential run on 1,000 fresh
  strings of another seed.
whisper_full's initial_prompt path (ref 6944-6979) uses exactly this function; its end-to-end
pins are in tests/test_gpu_params.py.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import owk

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "tokenize_golden.json")


def _tok(L, path, text: bytes):
    L.owk_debug_tokenize.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.c_int]
    n = L.owk_debug_tokenize(path.encode(), text, None, 0)
    assert n != -(2 ** 31), "owk_debug_tokenize could not parse the model"
    n = -n if n < 0 else n
    buf = (C.c_int * max(n, 1))()
    m = L.owk_debug_tokenize(path.encode(), text, buf, n)
    assert m == n
    return list(buf[:n])


@pytest.fixture(scope="module")
def tok_golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("model", ["tiny.en", "tiny"])
def test_tokenize_matches_reference_golden(tok_golden, model_path, model):
    L = owk.load()
    owk.quiet()
    path = model_path(model)
    import owk_synth as S

    assert S.file_sha256(path) == tok_golden["models"][model]["sha256"]
    bad = []
    n_tok = 0
    for c in tok_golden["cases"]:
        text = bytes.fromhex(c["text_hex"])
        got = _tok(L, path, text)
        n_tok += len(got)
        if got != c[model]:
            bad.append((text[:60], got[:12], c[model][:12]))
    print(f"{model}: {len(tok_golden['cases'])} strings, {n_tok} tokens")
    assert not bad, f"{len(bad)} strings tokenized differently, first: {bad[:3]}"
    # the golden set covers the whisper_full resize branch (> 1024 tokens) and the empty string
    assert max(len(c[model]) for c in tok_golden["cases"]) > 1024
    assert any(c["text_hex"] == "" for c in tok_golden["cases"])


def test_tokenize_live_differential(model_path):
    import ref_oracle as R

    if not R.available():
        pytest.skip("compiled reference (oracle/_ref) not present")
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_golden_tokenize as G

    L = owk.load()
    owk.quiet()
    rng = np.random.default_rng(98765)
    strings = G.gen_strings(rng, G.vocab_words(False) + G.vocab_words(True)[-2000:])[:1000]
    for model in ("tiny.en", "tiny"):
        path = model_path(model)
        ref = R.Ref(path)
        try:
            for s in strings:
                assert _tok(L, path, s) == ref.tokenize(s), s[:80]
        finally:
            ref.close()


def test_token_count_and_errors(model_path):
    L = owk.load()
    L.owk_debug_tokenize.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.c_int]
    path = model_path("tiny.en")
    # a too-small buffer reports -count (whisper_tokenize / whisper_token_count contract, ref 3957-3973)
    n = L.owk_debug_tokenize(path.encode(), b"Hello world, again and again.", None, 0)
    assert n < 0
    buf = (C.c_int * 2)()
    assert L.owk_debug_tokenize(path.encode(), b"Hello world, again and again.", buf, 2) == n
    assert L.owk_debug_tokenize(b"/nonexistent/model.bin", b"x", buf, 2) == -(2 ** 31)
