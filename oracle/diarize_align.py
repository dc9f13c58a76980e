"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product): a pure-Python
restatement of the reference SDK's Swift DiarizationAligner and RTTMParser, used as the
differential oracle for csrc/diarize_align.cpp on randomized inputs.

  ref Sources/OpenWhisperKit/DiarizationAligner.swift (align 21-75, assignSpeaker 77-126,
      smoothSentenceBoundaries 128-164, sentenceStartIndex 166-186, sentenceEndIndex 188-208,
      majoritySpeaker 210-233, groupUtterances 235-255, endsSentence 268-274,
      nearestSpeaker 280-293, distanceBetween 295-303, buildSpeakerOrder 305-311)
  ref Sources/OpenWhisperKit/RTTMParser.swift (parse 13-50, generate 52-64)

Swift `Float` arithmetic is emulated with numpy.float32. Parity pinned by the Swift unit
tests restated in tests/test_diarize_align.py (the reference's own known answers).
"""
import numpy as np

f32 = np.float32


def _ends_sentence(t):
    t = t.strip()
    return bool(t) and t[-1] in ".?!"


def _distance(ws, we, s):
    if we < s[1]:
        return f32(s[1] - we)
    if s[2] < ws:
        return f32(ws - s[2])
    return f32(0)


def _nearest(ws, we, segs):
    best = segs[0]
    for s in segs[1:]:
        di, db = _distance(ws, we, s), _distance(ws, we, best)
        if (s[1] < best[1]) if di == db else (di < db):
            best = s
    return best[0]


def _assign(w, segs, order, fill):
    if not segs:
        return None
    ws, we = min(w[1], w[2]), max(w[1], w[2])
    if ws == we:
        for s in segs:
            if s[1] <= ws <= s[2]:
                return s[0]
        return _nearest(ws, we, segs) if fill else None
    ov = {}
    for s in segs:
        inter = f32(min(s[2], we) - max(s[1], ws))
        if inter > 0:
            ov[s[0]] = f32(ov.get(s[0], f32(0)) + inter)
    if ov:
        items = list(ov.items())
        best = items[0]
        for e in items[1:]:
            if (order[best[0]] > order[e[0]]) if best[1] == e[1] else (best[1] < e[1]):
                best = e
        return best[0]
    return _nearest(ws, we, segs) if fill else None


def _majority(spk, start, end):
    counts, first = {}, {}
    for i in range(start, end + 1):
        counts[spk[i]] = counts.get(spk[i], 0) + 1
        first.setdefault(spk[i], len(first))
    return max(counts, key=lambda k: (counts[k], -first[k]))


def align(words, segments, fill_nearest=False, sentence_smoothing=True, max_words_in_sentence=50):
    if max_words_in_sentence <= 0:
        raise ValueError("maxWordsInSentence must be greater than 0")
    if not words:
        return {"words": [], "segments": [], "text": ""}
    words = [(w[0], f32(w[1]), f32(w[2])) for w in words]
    segs = sorted([(s[0], f32(s[1]), f32(s[2])) for s in segments], key=lambda s: s[1])  # stable
    order = {}
    for i, s in enumerate(segs):
        order.setdefault(s[0], i)
    spk = [_assign(w, segs, order, fill_nearest) for w in words]
    if sentence_smoothing and len(words) > 1:
        idx = 1
        while idx < len(words):
            if spk[idx] == spk[idx - 1] or _ends_sentence(words[idx - 1][0]):
                idx += 1
                continue
            start, cur, steps = max(0, idx - 1), idx - 1, 0
            while cur >= 0 and steps < max_words_in_sentence:
                if _ends_sentence(words[cur][0]):
                    start = min(idx - 1, cur + 1)
                    break
                start, cur, steps = cur, cur - 1, steps + 1
            end, cur, steps = min(len(words) - 1, idx), idx, 0
            while cur < len(words) and steps < max_words_in_sentence:
                end = cur
                if _ends_sentence(words[cur][0]):
                    break
                cur, steps = cur + 1, steps + 1
            maj = _majority(spk, start, end)
            for i in range(start, end + 1):
                spk[i] = maj
            idx = end + 1
    utts, first = [], 0
    for i in range(1, len(words) + 1):
        if i < len(words) and spk[i] == spk[first]:
            continue
        utts.append({"speaker": spk[first], "text": " ".join(w[0] for w in words[first:i]),
                     "start": float(words[first][1]), "end": float(words[i - 1][2]), "words": list(range(first, i))})
        first = i
    text = "\n".join(f"[{u['speaker'] if u['speaker'] is not None else 'unknown'}]: {u['text']}" for u in utts)
    return {"words": [(w[0], float(w[1]), float(w[2]), s) for w, s in zip(words, spk)], "segments": utts, "text": text}


def rttm_generate(segments, filename):
    return "\n".join(f"SPEAKER {filename} 1 {float(f32(s[1])):.2f} {float(f32(f32(s[2]) - f32(s[1]))):.2f} "
                     f"<NA> <NA> {s[0]} <NA> <NA>" for s in segments)


def rttm_parse(text):
    """RTTMParser.parse (ref RTTMParser.swift:13-50): lines of >= 8 space-separated fields, Float start and
    duration, end = start + duration (f32), sorted by start (stable) -> [(speaker, start, end)]."""
    out = []
    for line in text.split("\n"):
        f = [x for x in line.split(" ") if x]
        if len(f) < 8:
            continue
        try:
            start, dur = f32(float(f[3])), f32(float(f[4]))
        except ValueError:
            continue
        out.append((f[7], start, f32(start + dur)))
    return sorted(out, key=lambda s: s[1])
