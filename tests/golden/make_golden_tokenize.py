"""Golden whisper_tokenize vectors (tokenize_golden.json): the REFERENCE whisper_tokenize
(ref src/whisper.cpp:3272-3320, 3957-3973; oracle/_ref/libwhisper_ref.so via ref_oracle.py) on
both vocabularies the synthetic models carry -- the reference's own English (tiny.en) and
multilingual (tiny) vocabularies -- over 1,200 seeded strings: vocabulary-word compositions,
contractions, whitespace runs, digits, Latin / Greek / Cyrillic / CJK / emoji / combining / RTL
UTF-8, control characters, bytes that are not UTF-8 at all, the empty string, and prompts longer
than 1,024 tokens (the resize branch of whisper_full's initial-prompt tokenization, ref 6948-6957).

Strings are stored as hex of their bytes (no NUL: the API takes a C string).

Usage (container with /root/reference):  python tests/golden/make_golden_tokenize.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 1234
N_RANDOM = 1200

UNICODE_POOLS = [
    "àáâãäåæçèéêëìíîïñòóôõöøùúûüýÿÀÉÎÕÜßœŒ",
    "αβγδεζηθικλμνξοπρστυφχψωΑΒΓΔΘΛΞΠΣΦΨΩ",
    "абвгдеёжзийклмнопрстуфхцчшщъыьэюяАБВГДЕЖЗ",
    "日本語のテキスト中文字符한국어文章東京大阪",
    "😀😃😄😁🎉🚀👍🏽❤️🇺🇸",
    "éàöñ",  # combining marks
    "مرحبا بالعالم שלום עולם",
    "—–‘’“”…•€£¥©®™°±×÷",
]
CONTRACTIONS = ["'s", "'t", "'re", "'ve", "'m", "'ll", "'d", "'S", "'T", "'RE", "n't", "'", "''"]
WS = [" ", "  ", "\t", "\n", "\r\n", " \n ", "   ", " ", "　"]


def vocab_words(multilingual):
    """The vocabulary's token strings (bytes), as owk_synth writes them into the model file."""
    import struct

    raw = S.vocab_bytes(multilingual)
    n = struct.unpack_from("<i", raw, 0)[0]
    off, words = 4, []
    for _ in range(n):
        ln = struct.unpack_from("<I", raw, off)[0]
        words.append(raw[off + 4: off + 4 + ln])
        off += 4 + ln
    return [w for w in words if w and b"\0" not in w]


def gen_strings(rng, words):
    out = [b"", b" ", b"a", b"Hello world", b"Hello world.", b" Hello world.", b"I'm here, you're there; it's fine.",
           b"1234567890", b"3.14159 and 1,000,000", b"\xff\xfe\xfd", b"\x01\x02\x03 ctrl", b"tab\tsep\tvalues",
           b"trailing   ", b"   leading", b"multi\n\nline\ntext\n", "Ça va? 日本語 naïve 😀".encode(),
           b"[_BEG_] [_TT_1] <|endoftext|>", b"\xc3\x28 invalid utf8 \xa0\xa1", b"'s't're've'm'll'd",
           b"ALL CAPS SHOUTING!!!", b"mIxEd CaSe WoRdS", b"emoji\xf0\x9f\x98\x80end"]
    long_txt = b" ".join(words[int(i)] .strip() for i in rng.integers(0, len(words), 1500))
    out += [long_txt, b"x" * 3000, (" ".join(["prompt"] * 1100)).encode()]
    while len(out) < N_RANDOM:
        kind = int(rng.integers(0, 8))
        parts = []
        for _ in range(int(rng.integers(1, 12))):
            c = int(rng.integers(0, 7)) if kind == 7 else kind
            if c == 0:
                parts.append(words[int(rng.integers(0, len(words)))])
            elif c == 1:
                parts.append(bytes(int(x) for x in rng.integers(32, 127, int(rng.integers(1, 12)))))
            elif c == 2:
                parts.append(CONTRACTIONS[int(rng.integers(0, len(CONTRACTIONS)))].encode())
            elif c == 3:
                parts.append(WS[int(rng.integers(0, len(WS)))].encode())
            elif c == 4:
                parts.append(str(int(rng.integers(0, 10 ** int(rng.integers(1, 12))))).encode())
            elif c == 5:
                pool = UNICODE_POOLS[int(rng.integers(0, len(UNICODE_POOLS)))]
                k = int(rng.integers(1, 8))
                parts.append("".join(pool[int(i)] for i in rng.integers(0, len(pool), k)).encode())
            else:
                parts.append(bytes(int(x) for x in rng.integers(1, 256, int(rng.integers(1, 6)))))
        s = b"".join(parts).replace(b"\0", b"")
        out.append(s)
    return out


def main():
    import ref_oracle as R

    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    rng = np.random.default_rng(SEED)
    strings = gen_strings(rng, vocab_words(False) + vocab_words(True)[-2000:])
    meta = {"seed": SEED, "models": {}, "cases": [{"text_hex": s.hex()} for s in strings]}
    for model in ("tiny.en", "tiny"):
        path = S.ensure_model(model, SEED, cache)
        meta["models"][model] = {"sha256": S.file_sha256(path)}
        ref = R.Ref(path)
        for c, s in zip(meta["cases"], strings):
            c[model] = ref.tokenize(s)
        ref.close()
        print(model, sum(len(c[model]) for c in meta["cases"]), "tokens", flush=True)
    with open(os.path.join(OUT, "tokenize_golden.json"), "w") as f:
        json.dump(meta, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
