"""Speaker attribution (include/owk_diarize.h, csrc/diarize_align.cpp) on the CPU.

The known answers are the reference SDK's own Swift unit tests, restated case by case:
  ref tests/OpenWhisperKitTests/DiarizationAlignerTests.swift (line of each test cited)
  ref tests/OpenWhisperKitTests/RTTMParserTests.swift
plus a randomized differential test against oracle/diarize_align.py (a restatement of
ref Sources/OpenWhisperKit/DiarizationAligner.swift in Python with f32 arithmetic).
"""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import owk  # noqa: E402
import diarize_align as ref  # noqa: E402


def W(t, s, e, p=0.9):
    return (t, s, e, p)


def spk(res):
    return [w[3] for w in res["words"]]


def test_basic_alignment():  # DiarizationAlignerTests.swift:14
    r = owk.align([W("hello", 0.1, 0.5), W("world", 0.6, 1.0)], [("speaker_0", 0.0, 2.0)])
    assert spk(r) == ["speaker_0", "speaker_0"]


def test_boundary_spanning():  # :26
    r = owk.align([W("crossing", 0.8, 1.4)], [("speaker_0", 0.0, 1.0), ("speaker_1", 1.0, 2.0)])
    assert spk(r) == ["speaker_1"]


def test_zero_duration_word():  # :37
    assert spk(owk.align([W(",", 1.5, 1.5)], [("speaker_0", 0.0, 2.0)])) == ["speaker_0"]


def test_no_matching_segment():  # :45
    assert spk(owk.align([W("orphan", 5.0, 6.0)], [("speaker_0", 0.0, 2.0)], fill_nearest=False)) == [None]


def test_fill_nearest():  # :57
    r = owk.align([W("gap", 3.0, 4.0)], [("speaker_0", 0.0, 2.0), ("speaker_1", 5.0, 7.0)], fill_nearest=True)
    assert spk(r) == ["speaker_0"]


def test_empty_words():  # :72
    r = owk.align([], [("s0", 0, 1)])
    assert r == {"words": [], "segments": [], "text": ""}


def test_empty_diarization_segments():  # :83
    assert spk(owk.align([W("alone", 0, 1)], [])) == [None]


def test_sentence_smoothing():  # :89
    words = [W("Hello", 0.0, 0.5), W("world,", 0.5, 1.0), W("how", 1.0, 1.5), W("are", 1.5, 2.0), W("you?", 2.0, 2.5)]
    segs = [("speaker_0", 0.0, 1.0), ("speaker_1", 1.0, 2.0), ("speaker_0", 2.0, 3.0)]
    r = owk.align(words, segs, sentence_smoothing=True)
    assert len({s for s in spk(r) if s is not None}) == 1


def test_sentence_smoothing_disabled():  # :113
    r = owk.align([W("Hello", 0.0, 0.5), W("world", 0.5, 1.0)], [("speaker_0", 0.0, 0.6), ("speaker_1", 0.6, 1.5)],
                  sentence_smoothing=False)
    assert spk(r) == ["speaker_0", "speaker_1"]


def test_utterance_grouping_and_text():  # :133, :153
    r = owk.align([W("Hello.", 0.0, 1.0), W("Hi.", 1.0, 2.0)], [("speaker_0", 0.0, 1.0), ("speaker_1", 1.0, 2.0)],
                  sentence_smoothing=False)
    assert [u["speaker"] for u in r["segments"]] == ["speaker_0", "speaker_1"]
    assert r["text"] == "[speaker_0]: Hello.\n[speaker_1]: Hi."


def test_tie_breaking_uses_earlier_speaker_order():  # :173
    r = owk.align([W("equal", 0.5, 1.5)], [("speaker_0", 0.0, 1.0), ("speaker_1", 1.0, 2.0)])
    assert spk(r) == ["speaker_0"]


def test_max_words_in_sentence_validation():  # :184
    with pytest.raises(owk.AlignmentFailed, match="maxWordsInSentence"):
        owk.align([W("hello", 0, 1)], [("speaker_0", 0, 2)], max_words_in_sentence=0)


def test_unknown_speaker_text():
    r = owk.align([W("a", 0, 1), W("b", 5, 6)], [("s0", 0, 2)], sentence_smoothing=False)
    assert r["text"] == "[s0]: a\n[unknown]: b"


# --- RTTMParserTests.swift ---------------------------------------------------------------
def test_rttm_parse_empty():  # RTTMParserTests.swift:6
    assert owk.rttm_parse("") == []


def test_rttm_parse_single_line():  # :11
    s = owk.rttm_parse("SPEAKER file 1 0.500 1.200 <NA> <NA> speaker_0 <NA> <NA>")
    assert len(s) == 1 and s[0][0] == "speaker_0"
    assert abs(s[0][1] - 0.5) < 1e-3 and abs(s[0][2] - 1.7) < 1e-3


def test_rttm_parse_multi_line_sorted():  # :21, :81
    s = owk.rttm_parse("SPEAKER file 1 1.000 0.500 <NA> <NA> speaker_1 <NA> <NA>\n"
                       "SPEAKER file 1 0.000 1.000 <NA> <NA> speaker_0 <NA> <NA>")
    assert [x[0] for x in s] == ["speaker_0", "speaker_1"]
    s = owk.rttm_parse("\n".join(f"SPEAKER file 1 {t:.3f} 0.500 <NA> <NA> speaker_{k} <NA> <NA>"
                                 for t, k in [(2.0, 2), (0.0, 0), (1.0, 1)]))
    assert [x[0] for x in s] == ["speaker_0", "speaker_1", "speaker_2"]


def test_rttm_parse_malformed():  # :33, :39
    assert owk.rttm_parse("SPEAKER file 1 bad 1.000 <NA> <NA> speaker_0 <NA> <NA>") == []
    s = owk.rttm_parse("SPEAKER file 1 0.000 1.000 <NA> <NA> speaker_0 <NA> <NA>\n"
                       "SPEAKER file 1 BAD 0.500 <NA> <NA> speaker_bad <NA> <NA>\n"
                       "SPEAKER file 1 1.200 0.800 <NA> <NA> speaker_1 <NA> <NA>")
    assert [x[0] for x in s] == ["speaker_0", "speaker_1"]
    assert owk.rttm_parse("SPEAKER file 1 0.0 1.0 <NA> <NA>") == []  # fewer than 8 fields


def test_rttm_generate():  # :51
    txt = owk.rttm_generate([("speaker_0", 0.0, 1.25), ("speaker_1", 1.25, 2.0)], "audio")
    assert "SPEAKER audio 1 0.00 1.25 <NA> <NA> speaker_0 <NA> <NA>" in txt
    assert "SPEAKER audio 1 1.25 0.75 <NA> <NA> speaker_1 <NA> <NA>" in txt
    assert not txt.endswith("\n")


def test_rttm_round_trip():  # :62
    inp = [("speaker_0", 0.0, 1.2), ("speaker_1", 1.2, 2.35)]
    out = owk.rttm_parse(owk.rttm_generate(inp, "sample"))
    assert [o[0] for o in out] == [i[0] for i in inp]
    for o, i in zip(out, inp):
        assert abs(o[1] - i[1]) < 0.01 and abs(o[2] - i[2]) < 0.01


def test_rttm_from_sortformer_format():
    # lines as sortformer_to_rttm writes them (ref streaming-sortformer/src/sortformer.cpp:2593-2669)
    txt = "SPEAKER audio 1 0.08 1.20 <NA> <NA> speaker_1 <NA> <NA>\nSPEAKER audio 1 0.00 0.40 <NA> <NA> speaker_0 <NA> <NA>\n"
    assert [x[0] for x in owk.rttm_parse(txt)] == ["speaker_0", "speaker_1"]


# --- randomized differential test against the Python restatement -----------------------
PUNCT = ["", "", "", ",", ".", "?", "!", ". ", " "]


@pytest.mark.parametrize("seed", range(40))
def test_align_matches_restatement(seed):
    rng = random.Random(seed)
    grid = lambda: round(rng.uniform(0, 20) * 4) / 4 if rng.random() < 0.5 else rng.uniform(0, 20)  # noqa: E731
    words = []
    for i in range(rng.randint(1, 60)):
        a, b = grid(), grid()
        if rng.random() < 0.1:
            b = a
        words.append((f"w{i}{rng.choice(PUNCT)}", a, b, 0.5))
    segs = []
    for _ in range(rng.randint(0, 12)):
        a = grid()
        segs.append((f"speaker_{rng.randint(0, 3)}", a, a + rng.choice([0.25, 0.5, 1.0, rng.uniform(0, 3)])))
    opts = dict(fill_nearest=rng.random() < 0.5, sentence_smoothing=rng.random() < 0.7,
                max_words_in_sentence=rng.choice([1, 2, 3, 5, 50]))
    got = owk.align(words, segs, **opts)
    exp = ref.align(words, segs, **opts)
    assert spk(got) == spk(exp)
    assert [(u["speaker"], u["text"], u["words"]) for u in got["segments"]] == \
           [(u["speaker"], u["text"], u["words"]) for u in exp["segments"]]
    assert got["text"] == exp["text"]
    segs_sorted = sorted(segs, key=lambda s: s[1])
    assert owk.rttm_generate(segs_sorted, "f") == ref.rttm_generate(segs_sorted, "f")


# --- the configs[4] pipeline's own input: 3,453 words x the reference's 3-speaker stream RTTM ------
@pytest.mark.parametrize("variant", ["default", "nosmooth", "fill", "smooth5"])
def test_align_c4_reference_pipeline(variant):
    """libwhisper.so's aligner on the reference configs[4] pipeline's words and 2 s-stream RTTM
    (tests/golden/c4_golden.json; make_golden_c4.py / make_golden_c4_align.py) with each AlignmentOptions
    variant: word speakers, utterances and text identical to the reference pipeline's."""
    import json
    import os

    meta = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c4_golden.json")))
    words = [tuple(w) for w in meta["results"]["words"]]
    segs = owk.rttm_parse(meta["results"]["rttm"])
    if variant == "default":
        opt, exp = {}, meta["results"]["aligned"]
    else:
        v = meta["results"]["aligned_variants"][variant]
        opt, exp = v["options"], v
    got = owk.align(words, segs, **opt)
    assert spk(got) == exp["speakers"]
    assert [(u["speaker"], u["words"][0], len(u["words"])) for u in got["segments"]] == [tuple(u) for u in exp["utterances"]]
    assert got["text"] == exp["text"]
    if variant in ("nosmooth", "fill"):
        assert len({s for s in exp["speakers"] if s}) >= 3 and len(exp["utterances"]) >= 10
