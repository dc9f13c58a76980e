/*
 * owk_diarize.h -- C ABI of the speaker-attribution layer that sits between
 * whisper_full() word timings and SortFormer diarization segments.
 *
 * The reference ships these as Swift-only utilities of its SDK:
 *   DiarizationAligner.align(words:diarizationSegments:options:)
 *       ref Sources/OpenWhisperKit/DiarizationAligner.swift:21-75
 *   RTTMParser.parse / RTTMParser.generate
 *       ref Sources/OpenWhisperKit/RTTMParser.swift:13-64
 * Here they are C++ inside libwhisper.so so that the end-to-end pipeline of BASELINE
 * configs[4] (transcribe + diarize + align) runs on Linux hosts without Swift. Results,
 * tie-breaking and error behaviour follow the Swift code line for line (cited in
 * csrc/diarize_align.cpp); times are seconds in f32 like the Swift `Float` fields.
 */
#ifndef OWK_DIARIZE_H
#define OWK_DIARIZE_H

#include "whisper.h"

#ifdef __cplusplus
extern "C" {
#endif

/* WordTiming (ref Sources/OpenWhisperKit/Models.swift): one transcribed word/token */
struct owk_word {
    const char * word;
    float start;
    float end;
    float probability;
};

/* DiarizationSegment (ref Sources/OpenWhisperKit/DiarizationModels.swift:36-60) */
struct owk_dseg {
    const char * speaker;
    float start;
    float end;
};

/* DiarizationAligner.AlignmentOptions (ref DiarizationAligner.swift:5-19) */
struct owk_align_options {
    int fill_nearest;          /* default 0 */
    int sentence_smoothing;    /* default 1 */
    int max_words_in_sentence; /* default 50; must be > 0 */
};

WHISPER_API struct owk_align_options owk_align_default_options(void);

/* DiarizedTranscription: per-word speakers, utterances (runs of one speaker) and the
 * "[speaker]: text" lines. Opaque; owned by the caller, freed by owk_alignment_free. */
struct owk_alignment;

/* Returns NULL if max_words_in_sentence <= 0 (the Swift code throws
 * DiarizationError.alignmentFailed) or on bad arguments. Word/segment strings are
 * copied. n_segs may be 0 (every speaker is then NULL). */
WHISPER_API struct owk_alignment * owk_align(const struct owk_word * words, int n_words, const struct owk_dseg * segs,
                                             int n_segs, struct owk_align_options options);
WHISPER_API void owk_alignment_free(struct owk_alignment * a);

WHISPER_API int owk_alignment_n_words(const struct owk_alignment * a);
/* speaker of word i, or NULL when no segment was attributed (Swift nil) */
WHISPER_API const char * owk_alignment_word_speaker(const struct owk_alignment * a, int i);

WHISPER_API int owk_alignment_n_utterances(const struct owk_alignment * a);
/* utterance i: speaker (NULL = nil), text (words joined by ' '), start/end, and its
 * first word index and word count. Returns 0, or -1 if i is out of range. */
WHISPER_API int owk_alignment_utterance(const struct owk_alignment * a, int i, const char ** speaker, const char ** text,
                                        float * start, float * end, int * first_word, int * n_words);
/* "[speaker]: text" per utterance joined by '\n' ("unknown" for nil speakers) */
WHISPER_API const char * owk_alignment_text(const struct owk_alignment * a);

/* RTTMParser.parse: one segment per "SPEAKER <file> <chan> <start> <dur> <NA> <NA> <spk> ..."
 * line (>= 8 space-separated fields, start/duration parseable as floats), sorted by start. */
struct owk_rttm;
WHISPER_API struct owk_rttm * owk_rttm_parse(const char * text);
WHISPER_API int owk_rttm_n_segments(const struct owk_rttm * r);
WHISPER_API int owk_rttm_segment(const struct owk_rttm * r, int i, const char ** speaker, float * start, float * end);
WHISPER_API void owk_rttm_free(struct owk_rttm * r);

/* RTTMParser.generate: lines "SPEAKER <filename> 1 %.2f %.2f <NA> <NA> <speaker> <NA> <NA>"
 * joined by '\n' (no trailing newline). Writes at most cap bytes including the NUL and
 * returns the full length (excluding the NUL), like snprintf. */
WHISPER_API int owk_rttm_generate(const struct owk_dseg * segs, int n_segs, const char * filename, char * out, int cap);

#ifdef __cplusplus
}
#endif

#endif /* OWK_DIARIZE_H */
