// Speaker attribution of word timings (include/owk_diarize.h): a C++ restatement of the
// reference SDK's Swift DiarizationAligner and RTTMParser. Host-only -- O(words x segments)
// bookkeeping next to the GPU transcription and diarization passes.
//
//   ref Sources/OpenWhisperKit/DiarizationAligner.swift  (cited per function below)
//   ref Sources/OpenWhisperKit/RTTMParser.swift
//
// Swift semantics kept: Float (f32) arithmetic for overlaps and distances; Sequence.max(by:)
// keeps the first maximal element and replaces it only when a later one compares strictly
// greater (min(by:) symmetric); the tie-break comparators make every choice independent of
// Dictionary iteration order; `sorted` is stable.
#include "owk_diarize.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <optional>
#include <string>
#include <vector>

namespace {

using Speaker = std::optional<std::string>;

struct Seg {
    std::string speaker;
    float start, end;
};

struct Word {
    std::string word;
    float start, end, probability;
    Speaker speaker;
};

struct Utterance {
    Speaker speaker;
    std::string text;
    float start, end;
    int first, count;
};

// endsSentence (DiarizationAligner.swift:268-274): last character of the text trimmed of
// whitespace and newlines is one of . ? !
bool is_space_at(const std::string & s, size_t end, size_t & len) {
    // trailing whitespace / newline code point ending at byte `end` (exclusive)
    const unsigned char c = (unsigned char) s[end - 1];
    if (c == ' ' || (c >= 0x09 && c <= 0x0d)) { len = 1; return true; }
    if (end >= 2) {
        const unsigned char a = (unsigned char) s[end - 2];
        if ((a == 0xc2 && (c == 0x85 || c == 0xa0))) { len = 2; return true; }  // U+0085, U+00A0
    }
    if (end >= 3) {
        const unsigned char a = (unsigned char) s[end - 3], b = (unsigned char) s[end - 2];
        if (a == 0xe2 && b == 0x80 && ((c >= 0x80 && c <= 0x8a) || c == 0xa8 || c == 0xa9 || c == 0xaf)) { len = 3; return true; }
        if (a == 0xe2 && b == 0x81 && c == 0x9f) { len = 3; return true; }  // U+205F
        if (a == 0xe3 && b == 0x80 && c == 0x80) { len = 3; return true; }  // U+3000
        if (a == 0xe1 && b == 0x9a && c == 0x80) { len = 3; return true; }  // U+1680
    }
    return false;
}

bool ends_sentence(const std::string & text) {
    size_t end = text.size(), len = 0;
    while (end > 0 && is_space_at(text, end, len)) end -= len;
    if (end == 0) return false;
    const char last = text[end - 1];
    return last == '.' || last == '?' || last == '!';
}

// contains (DiarizationAligner.swift:276-278)
bool contains(float t, const Seg & s) { return t >= s.start && t <= s.end; }

// distanceBetween (DiarizationAligner.swift:295-303)
float distance_between(float ws, float we, const Seg & s) {
    if (we < s.start) return s.start - we;
    if (s.end < ws) return ws - s.end;
    return 0.0f;
}

// nearestSpeaker (DiarizationAligner.swift:280-293): min(by:) over segments, ties by start
Speaker nearest_speaker(float ws, float we, const std::vector<Seg> & segs) {
    if (segs.empty()) return std::nullopt;
    size_t best = 0;
    for (size_t i = 1; i < segs.size(); ++i) {
        const float di = distance_between(ws, we, segs[i]), db = distance_between(ws, we, segs[best]);
        const bool less = di == db ? segs[i].start < segs[best].start : di < db;
        if (less) best = i;
    }
    return segs[best].speaker;
}

// assignSpeaker (DiarizationAligner.swift:77-126)
Speaker assign_speaker(const Word & w, const std::vector<Seg> & segs, const std::map<std::string, int> & order,
                       bool fill_nearest) {
    if (segs.empty()) return std::nullopt;
    const float ws = std::min(w.start, w.end), we = std::max(w.start, w.end);
    if (ws == we) {
        for (const Seg & s : segs)
            if (contains(ws, s)) return s.speaker;
        if (fill_nearest) return nearest_speaker(ws, we, segs);
        return std::nullopt;
    }
    // overlap per speaker, accumulated in segment order (f32)
    std::vector<std::pair<std::string, float>> overlap;
    for (const Seg & s : segs) {
        const float inter = std::min(s.end, we) - std::max(s.start, ws);
        if (inter > 0) {
            auto it = std::find_if(overlap.begin(), overlap.end(), [&](const auto & p) { return p.first == s.speaker; });
            if (it == overlap.end()) overlap.emplace_back(s.speaker, 0.0f + inter);
            else it->second += inter;
        }
    }
    if (!overlap.empty()) {
        // max(by:): lhs < rhs if lhs.value < rhs.value, or equal values and lhs's speaker
        // order is later. Every speaker here has a distinct order, so the maximum is unique.
        auto ord = [&](const std::string & k) {
            auto it = order.find(k);
            return it == order.end() ? INT32_MAX : it->second;
        };
        size_t best = 0;
        for (size_t i = 1; i < overlap.size(); ++i) {
            const auto & b = overlap[best];
            const auto & e = overlap[i];
            const bool less = b.second == e.second ? ord(b.first) > ord(e.first) : b.second < e.second;
            if (less) best = i;
        }
        return overlap[best].first;
    }
    if (fill_nearest) return nearest_speaker(ws, we, segs);
    return std::nullopt;
}

// sentenceStartIndex (DiarizationAligner.swift:166-186)
int sentence_start(const std::vector<Word> & w, int change, int max_words) {
    int start = std::max(0, change - 1), cursor = change - 1, steps = 0;
    while (cursor >= 0 && steps < max_words) {
        if (ends_sentence(w[cursor].word)) return std::min(change - 1, cursor + 1);
        start = cursor;
        cursor -= 1;
        steps += 1;
    }
    return start;
}

// sentenceEndIndex (DiarizationAligner.swift:188-208)
int sentence_end(const std::vector<Word> & w, int change, int max_words) {
    int end = std::min((int) w.size() - 1, change), cursor = change, steps = 0;
    while (cursor < (int) w.size() && steps < max_words) {
        end = cursor;
        if (ends_sentence(w[cursor].word)) return end;
        cursor += 1;
        steps += 1;
    }
    return end;
}

// majoritySpeaker (DiarizationAligner.swift:210-233): most frequent, ties to the first seen
Speaker majority_speaker(const std::vector<Word> & w, int start, int end) {
    std::vector<std::pair<Speaker, int>> counts;  // in first-seen order
    for (int i = start; i <= end; ++i) {
        auto it = std::find_if(counts.begin(), counts.end(), [&](const auto & p) { return p.first == w[i].speaker; });
        if (it == counts.end()) counts.emplace_back(w[i].speaker, 1);
        else it->second += 1;
    }
    size_t best = 0;
    for (size_t i = 1; i < counts.size(); ++i)
        if (counts[best].second < counts[i].second) best = i;  // equal counts: earlier first-seen wins
    return counts[best].first;
}

// smoothSentenceBoundaries (DiarizationAligner.swift:128-164)
void smooth(std::vector<Word> & w, int max_words) {
    if (w.size() <= 1) return;
    int index = 1;
    while (index < (int) w.size()) {
        if (w[index].speaker == w[index - 1].speaker) { index += 1; continue; }
        if (ends_sentence(w[index - 1].word)) { index += 1; continue; }
        const int start = sentence_start(w, index, max_words);
        const int end = sentence_end(w, index, max_words);
        const Speaker maj = majority_speaker(w, start, end);
        for (int i = start; i <= end; ++i) w[i].speaker = maj;
        index = end + 1;
    }
}

}  // namespace

struct owk_alignment {
    std::vector<Word> words;
    std::vector<Utterance> utt;
    std::string text;
};

struct owk_rttm {
    std::vector<Seg> segs;
};

extern "C" {

struct owk_align_options owk_align_default_options(void) {
    owk_align_options o;
    o.fill_nearest = 0;
    o.sentence_smoothing = 1;
    o.max_words_in_sentence = 50;
    return o;
}

// align (DiarizationAligner.swift:21-75)
struct owk_alignment * owk_align(const struct owk_word * words, int n_words, const struct owk_dseg * segs, int n_segs,
                                 struct owk_align_options options) {
    if (options.max_words_in_sentence <= 0) return nullptr;  // alignmentFailed
    if (n_words < 0 || n_segs < 0 || (n_words > 0 && !words) || (n_segs > 0 && !segs)) return nullptr;
    auto * a = new owk_alignment;
    if (n_words == 0) return a;
    // segments ordered by start, ties in input order (sorted with the offset tie-break)
    std::vector<Seg> ordered;
    ordered.reserve(n_segs);
    for (int i = 0; i < n_segs; ++i) ordered.push_back({segs[i].speaker ? segs[i].speaker : "", segs[i].start, segs[i].end});
    std::stable_sort(ordered.begin(), ordered.end(), [](const Seg & l, const Seg & r) { return l.start < r.start; });
    // buildSpeakerOrder (DiarizationAligner.swift:305-311)
    std::map<std::string, int> order;
    for (int i = 0; i < (int) ordered.size(); ++i) order.emplace(ordered[i].speaker, i);

    a->words.reserve(n_words);
    for (int i = 0; i < n_words; ++i) {
        Word w{words[i].word ? words[i].word : "", words[i].start, words[i].end, words[i].probability, std::nullopt};
        w.speaker = assign_speaker(w, ordered, order, options.fill_nearest != 0);
        a->words.push_back(std::move(w));
    }
    if (options.sentence_smoothing) smooth(a->words, options.max_words_in_sentence);

    // groupUtterances / makeUtterance (DiarizationAligner.swift:235-266)
    int first = 0;
    const int n = (int) a->words.size();
    for (int i = 1; i <= n; ++i) {
        if (i < n && a->words[i].speaker == a->words[first].speaker) continue;
        Utterance u;
        u.speaker = a->words[first].speaker;
        u.first = first;
        u.count = i - first;
        u.start = a->words[first].start;
        u.end = a->words[i - 1].end;
        for (int k = first; k < i; ++k) {
            if (k > first) u.text += ' ';
            u.text += a->words[k].word;
        }
        a->utt.push_back(std::move(u));
        first = i;
    }
    for (size_t k = 0; k < a->utt.size(); ++k) {
        if (k) a->text += '\n';
        a->text += "[" + (a->utt[k].speaker ? *a->utt[k].speaker : std::string("unknown")) + "]: " + a->utt[k].text;
    }
    return a;
}

void owk_alignment_free(struct owk_alignment * a) { delete a; }

int owk_alignment_n_words(const struct owk_alignment * a) { return a ? (int) a->words.size() : 0; }

const char * owk_alignment_word_speaker(const struct owk_alignment * a, int i) {
    if (!a || i < 0 || i >= (int) a->words.size() || !a->words[i].speaker) return nullptr;
    return a->words[i].speaker->c_str();
}

int owk_alignment_n_utterances(const struct owk_alignment * a) { return a ? (int) a->utt.size() : 0; }

int owk_alignment_utterance(const struct owk_alignment * a, int i, const char ** speaker, const char ** text,
                            float * start, float * end, int * first_word, int * n_words) {
    if (!a || i < 0 || i >= (int) a->utt.size()) return -1;
    const Utterance & u = a->utt[i];
    if (speaker) *speaker = u.speaker ? u.speaker->c_str() : nullptr;
    if (text) *text = u.text.c_str();
    if (start) *start = u.start;
    if (end) *end = u.end;
    if (first_word) *first_word = u.first;
    if (n_words) *n_words = u.count;
    return 0;
}

const char * owk_alignment_text(const struct owk_alignment * a) { return a ? a->text.c_str() : ""; }

// RTTMParser.parse (RTTMParser.swift:13-50)
struct owk_rttm * owk_rttm_parse(const char * text) {
    auto * r = new owk_rttm;
    if (!text) return r;
    auto split = [](const std::string & s, char sep) {
        std::vector<std::string> out;
        size_t i = 0;
        while (i <= s.size()) {
            size_t j = s.find(sep, i);
            if (j == std::string::npos) j = s.size();
            if (j > i) out.push_back(s.substr(i, j - i));  // omittingEmptySubsequences
            i = j + 1;
        }
        return out;
    };
    // Swift Float(String): the whole field must parse
    auto to_float = [](const std::string & f, float & v) {
        if (f.empty() || isspace((unsigned char) f[0])) return false;
        char * e = nullptr;
        v = strtof(f.c_str(), &e);
        return e && *e == '\0';
    };
    for (const std::string & line : split(text, '\n')) {
        const std::vector<std::string> fields = split(line, ' ');
        if (fields.size() < 8) continue;
        float start, dur;
        if (!to_float(fields[3], start) || !to_float(fields[4], dur)) continue;
        r->segs.push_back({fields[7], start, start + dur});
    }
    std::stable_sort(r->segs.begin(), r->segs.end(), [](const Seg & a, const Seg & b) { return a.start < b.start; });
    return r;
}

int owk_rttm_n_segments(const struct owk_rttm * r) { return r ? (int) r->segs.size() : 0; }

int owk_rttm_segment(const struct owk_rttm * r, int i, const char ** speaker, float * start, float * end) {
    if (!r || i < 0 || i >= (int) r->segs.size()) return -1;
    if (speaker) *speaker = r->segs[i].speaker.c_str();
    if (start) *start = r->segs[i].start;
    if (end) *end = r->segs[i].end;
    return 0;
}

void owk_rttm_free(struct owk_rttm * r) { delete r; }

// RTTMParser.generate (RTTMParser.swift:52-64); duration = end - start in f32
int owk_rttm_generate(const struct owk_dseg * segs, int n_segs, const char * filename, char * out, int cap) {
    std::string s;
    char buf[64];
    for (int i = 0; i < n_segs; ++i) {
        if (i) s += '\n';
        s += "SPEAKER ";
        s += filename ? filename : "";
        snprintf(buf, sizeof(buf), " 1 %.2f %.2f <NA> <NA> ", (double) segs[i].start,
                 (double) (segs[i].end - segs[i].start));
        s += buf;
        s += segs[i].speaker ? segs[i].speaker : "";
        s += " <NA> <NA>";
    }
    if (out && cap > 0) {
        const size_t n = std::min(s.size(), (size_t) cap - 1);
        memcpy(out, s.data(), n);
        out[n] = '\0';
    }
    return (int) s.size();
}

}  // extern "C"
