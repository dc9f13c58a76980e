"""GBNF grammar-constrained decoding: the host constraint engine of libwhisper.so (csrc/grammar.cpp)
against the reference's own (whisper_grammar_init / whisper_grammar_accept_token /
whisper_suppress_invalid_grammar, ref src/whisper.cpp:5498-5905, driven through
oracle/ref/ref_probe.cpp), on grammars parsed by the reference's examples/grammar-parser.cpp.

For every grammar, every state reached by accepting a token sequence (walks through allowed tokens,
plus a disallowed token that empties the stacks, plus byte tokens that leave a partial UTF-8 code
point) must penalise exactly the same vocabulary ids. CPU only (no device); the end-to-end GPU
parity is tests/test_callers.py's grammar cases (the reference whisper-cli's --grammar output).
"""
import ctypes as C
import os

import numpy as np
import pytest

import owk

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

GRAMMARS = {
    "words": 'root ::= (" " word ",")+ " " word "."\nword ::= "red" | "green" | "blue" | "yellow" | "purple"\n',
    "moves": 'root ::= move (" " move)* [^a-z0-9 ]\nmove ::= " "? [a-h] [1-8] | " castle"\n',
    "nested": 'root ::= item ("," item)* | "none"\nitem ::= " "? ([0-9]+ ("." [0-9]+)? | "(" root ")")\n',
    "utf8": 'root ::= " " ("日本" | "café" | [à-ÿ]+ | [^\\x00-\\x7f])+ "."\n',
}


class GE(C.Structure):
    _fields_ = [("type", C.c_int), ("value", C.c_uint32)]


@pytest.fixture(scope="module")
def ref_ctx():
    import owk_synth as S
    import ref_oracle as R

    if not R.available():
        pytest.skip("reference oracle not built")
    path = S.ensure_model("tiny.en", 1234, os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models"))
    ref = R.Ref(path)
    L = ref.L
    L.whisper_token_to_str.restype = C.c_char_p
    L.whisper_token_to_str.argtypes = [C.c_void_p, C.c_int]
    L.whisper_token_eot.argtypes = [C.c_void_p]
    L.ref_grammar_parse.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_uint32), C.c_int,
                                    C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.ref_grammar_rejects.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.c_int,
                                      C.POINTER(C.c_int), C.c_int]
    vocab = [L.whisper_token_to_str(ref.ctx, i) for i in range(ref.n_vocab)]
    yield ref, vocab, L.whisper_token_eot(ref.ctx)
    ref.close()


def _parse(L, text):
    cap, capr = 4096, 256
    types = (C.c_int * cap)()
    vals = (C.c_uint32 * cap)()
    off = (C.c_int * capr)()
    nr, st = C.c_int(), C.c_int()
    n = L.ref_grammar_parse(text.encode(), b"root", types, vals, cap, off, capr, C.byref(nr), C.byref(st))
    assert 0 < n <= cap and nr.value < capr, n
    rules = []
    for r in range(nr.value):
        a, b = off[r], off[r + 1]
        rules.append((GE * (b - a))(*[GE(types[i], vals[i]) for i in range(a, b)]))
    return rules, st.value


def _ours(rules, start, vocab, eot, accept):
    Lw = owk.load()
    Lw.owk_debug_grammar_rejects.argtypes = [C.POINTER(C.POINTER(GE)), C.c_size_t, C.c_size_t, C.POINTER(C.c_char_p),
                                             C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int), C.c_int]
    ptrs = (C.POINTER(GE) * len(rules))(*[C.cast(r, C.POINTER(GE)) for r in rules])
    voc = (C.c_char_p * len(vocab))(*vocab)
    acc = (C.c_int * max(1, len(accept)))(*accept)
    out = (C.c_int * len(vocab))()
    n = Lw.owk_debug_grammar_rejects(ptrs, len(rules), start, voc, len(vocab), eot, acc, len(accept), out, len(vocab))
    assert n >= 0
    return set(out[:n])


def _refs(ref, text, accept, n_vocab):
    acc = (C.c_int * max(1, len(accept)))(*accept)
    out = (C.c_int * n_vocab)()
    n = ref.L.ref_grammar_rejects(ref.ctx, text.encode(), b"root", acc, len(accept), out, n_vocab)
    assert n >= 0
    return set(out[:n])


@pytest.mark.parametrize("name", sorted(GRAMMARS))
def test_grammar_rejects_match_reference(ref_ctx, name):
    ref, vocab, eot = ref_ctx
    text = GRAMMARS[name]
    rules, start = _parse(ref.L, text)
    rng = np.random.default_rng(len(name))
    seqs = [[]]
    # walks through tokens the grammar allows, 6 steps each
    for _ in range(3):
        seq = []
        for _ in range(6):
            rej = _refs(ref, text, seq, len(vocab))
            allowed = [i for i in range(eot) if vocab[i] and i not in rej]
            if not allowed:
                break
            seq.append(int(rng.choice(allowed)))
            seqs.append(list(seq))
    # a disallowed token (empties every stack) and single UTF-8 bytes (partial code points)
    rej0 = sorted(_refs(ref, text, [], len(vocab)))
    seqs.append([rej0[len(rej0) // 2]])
    bytes_tok = [i for i in range(eot) if len(vocab[i]) == 1 and vocab[i][0] >= 0xC3][:2]
    for b in bytes_tok:
        seqs.append([b])
    checked = 0
    for seq in seqs:
        want = _refs(ref, text, seq, len(vocab))
        got = _ours(rules, start, vocab, eot, seq)
        assert got == want, (name, seq, sorted(got ^ want)[:10])
        checked += 1
    print(f"[grammar] {name}: {checked} states, penalised sets identical to the reference's")
