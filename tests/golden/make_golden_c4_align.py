"""configs[4] aligner variants (adds results/aligned_variants to c4_golden.json).

The reference pipeline's words (its whisper_full tokens as Swift WordTiming, make_golden_c4.py) and
its 2 s-stream RTTM (three speakers: speaker_0 / 1 / 2) through the DiarizationAligner
(ref Sources/OpenWhisperKit/DiarizationAligner.swift:21-309, restated in oracle/diarize_align.py,
which tests/test_diarize_align.py pins to the Swift unit tests) with AlignmentOptions other than
the default. The default options (sentenceSmoothing, maxWordsInSentence 50) smooth the synthetic
model's words -- which almost never end a sentence -- into one speaker_0 utterance; these variants
keep the speaker turns:
  * nosmooth: sentenceSmoothing = false (per-word overlap assignment, unassigned words stay nil);
  * fill:     sentenceSmoothing = false, fillNearest = true (nil words take the nearest segment);
  * smooth5:  sentenceSmoothing = true, maxWordsInSentence = 5 (majority over short windows).

Usage:  python tests/golden/make_golden_c4_align.py [c4_10m_golden]  (after make_golden_c4.py [--minutes 10])
"""
import collections
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import diarize_align as DA  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
VARIANTS = {
    "nosmooth": dict(sentence_smoothing=False),
    "fill": dict(sentence_smoothing=False, fill_nearest=True),
    "smooth5": dict(sentence_smoothing=True, max_words_in_sentence=5),
}


def main():
    path = os.path.join(OUT, (sys.argv[1] if len(sys.argv) > 1 else "c4_golden") + ".json")
    meta = json.load(open(path))
    words = [tuple(w) for w in meta["results"]["words"]]
    dsegs = DA.rttm_parse(meta["results"]["rttm"])
    out = {}
    for name, opt in VARIANTS.items():
        al = DA.align(words, dsegs, **opt)
        out[name] = {"options": opt, "speakers": [w[3] for w in al["words"]],
                     "utterances": [(u["speaker"], u["words"][0], len(u["words"])) for u in al["segments"]],
                     "text": al["text"]}
        print(name, dict(collections.Counter(w[3] for w in al["words"])), len(al["segments"]), "utterances")
    meta["results"]["aligned_variants"] = out
    with open(path, "w") as f:
        json.dump(meta, f, indent=0)


if __name__ == "__main__":
    main()
