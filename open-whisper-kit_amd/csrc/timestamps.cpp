// Heuristic token-level timestamps (params.token_timestamps; used by the Swift SDK's
// WhisperContext). Host-side, per emitted segment; restates the reference
// whisper_exp_compute_token_level_timestamps (ref src/whisper.cpp:8455-8680) with its
// helpers voice_length (8400-8422), get_signal_energy (8425-8441), the segment-relative
// sample mapping (8443-8453) and whisper_wrap_segment (6077-6128).
#include <algorithm>
#include <cmath>

#include "state.h"

namespace owk {

static float voice_length(const std::string & text) {
    float res = 0.0f;
    for (char c : text) {
        if (c == ' ') res += 0.01f;
        else if (c == ',') res += 2.00f;
        else if (c == '.' || c == '!' || c == '?') res += 3.00f;
        else if (c >= '0' && c <= '9') res += 3.00f;
        else res += 1.00f;
    }
    return res;
}

std::vector<float> signal_energy(const float * signal, int n_samples, int hw) {
    std::vector<float> out(n_samples);
    // every output's float sum runs over j = -hw .. hw in order, as the reference's; the interior
    // samples are summed in blocks with j outermost, so the loop over samples vectorises with the
    // per-sample order unchanged (a 10 min buffer: 9.6 M samples x 65 terms)
    auto edge = [&](int i) {
        float sum = 0;
        for (int j = -hw; j <= hw; j++)
            if (i + j >= 0 && i + j < n_samples) sum += fabsf(signal[i + j]);
        out[i] = sum / (2 * hw + 1);
    };
    const int lo = std::min(hw, n_samples), hi = std::max(lo, n_samples - hw);
    for (int i = 0; i < lo; ++i) edge(i);
    constexpr int B = 2048;
    float acc[B];
    for (int b = lo; b < hi; b += B) {
        const int nb = std::min(B, hi - b);
        for (int i = 0; i < nb; ++i) acc[i] = 0.0f;
        for (int j = -hw; j <= hw; ++j) {
            const float * s = signal + b + j;
            for (int i = 0; i < nb; ++i) acc[i] += fabsf(s[i]);
        }
        for (int i = 0; i < nb; ++i) out[b + i] = acc[i] / (2 * hw + 1);
    }
    for (int i = hi; i < n_samples; ++i) edge(i);
    return out;
}

static int ts_to_sample(int64_t t, int64_t seg_t0, int n_samples) {
    const int64_t rel = t - seg_t0;
    const int s = (int) ((rel * WHISPER_SAMPLE_RATE) / 100);
    return std::max(0, std::min(n_samples - 1, s));
}

static int64_t sample_to_ts(int i_sample, int64_t seg_t0) { return (100ll * i_sample) / WHISPER_SAMPLE_RATE + seg_t0; }

void compute_token_timestamps(whisper_context * ctx, whisper_state * st, int i_segment, float thold_pt, float thold_ptsum) {
    const Vocab & v = ctx->model->vocab;
    Segment & seg = st->result_all[i_segment];
    auto & tk = seg.tokens;
    const int n_samples = (int) st->energy.size();
    if (n_samples == 0) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_exp_compute_token_level_timestamps: no signal data available\n");
        return;
    }
    const int64_t t0 = seg.t0, t1 = seg.t1;
    const int n = (int) tk.size();
    if (n == 0) return;
    if (n == 1) {
        tk[0].t0 = t0;
        tk[0].t1 = t1;
        return;
    }
    int64_t & t_beg = st->t_beg;
    int64_t & t_last = st->t_last;
    whisper_token & tid_last = st->tid_last;

    for (int j = 0; j < n; ++j) {
        auto & token = tk[j];
        if (j == 0) {
            if (token.id == v.beg) {
                tk[j].t0 = t0;
                tk[j].t1 = t0;
                tk[j + 1].t0 = t0;
                t_beg = t0;
                t_last = t0;
                tid_last = v.beg;
            } else {
                tk[j].t0 = t_last;
            }
        }
        const int64_t tt = t_beg + 2 * (token.tid - v.beg);
        tk[j].vlen = voice_length(v.id_to_token[token.id].c_str());  // C string, as ref 8510
        if (token.pt > thold_pt && token.ptsum > thold_ptsum && token.tid > tid_last && tt <= t1) {
            if (j > 0) tk[j - 1].t1 = tt;
            tk[j].t0 = tt;
            tid_last = token.tid;
        }
    }
    tk[n - 2].t1 = t1;
    tk[n - 1].t0 = t1;
    tk[n - 1].t1 = t1;
    t_last = t1;

    // split runs of tokens without timestamps proportionally to voice length
    {
        int p0 = 0, p1 = 0;
        for (;;) {
            while (p1 < n && tk[p1].t1 < 0) p1++;
            if (p1 >= n) p1--;
            if (p1 > p0) {
                double psum = 0.0;
                for (int j = p0; j <= p1; j++) psum += tk[j].vlen;
                const double dt = tk[p1].t1 - tk[p0].t0;
                for (int j = p0 + 1; j <= p1; j++) {
                    const double ct = tk[j - 1].t0 + dt * tk[j - 1].vlen / psum;
                    tk[j - 1].t1 = ct;
                    tk[j].t0 = ct;
                }
            }
            p1++;
            p0 = p1;
            if (p1 >= n) break;
        }
    }
    for (int j = 0; j < n - 1; j++) {
        if (tk[j].t1 < 0) tk[j + 1].t0 = tk[j].t1;
        if (j > 0 && tk[j - 1].t1 > tk[j].t0) {
            tk[j].t0 = tk[j - 1].t1;
            tk[j].t1 = std::max(tk[j].t0, tk[j].t1);
        }
    }
    // snap to voice activity
    const int hw = WHISPER_SAMPLE_RATE / 8;
    const auto & e = st->energy;
    for (int j = 0; j < n; j++) {
        if (tk[j].id >= v.eot) continue;
        int s0 = ts_to_sample(tk[j].t0, seg.t0, n_samples);
        int s1 = ts_to_sample(tk[j].t1, seg.t0, n_samples);
        const int ss0 = std::max(s0 - hw, 0);
        const int ss1 = std::min(s1 + hw, n_samples);
        const int ns = ss1 - ss0;
        float sum = 0.0f;
        for (int k = ss0; k < ss1; k++) sum += e[k];
        const float thold = 0.5 * sum / ns;
        {
            int k = s0;
            if (e[k] > thold && j > 0) {
                while (k > 0 && e[k] > thold) k--;
                tk[j].t0 = sample_to_ts(k, seg.t0);
                if (tk[j].t0 < tk[j - 1].t1) tk[j].t0 = tk[j - 1].t1;
                else s0 = k;
            } else {
                while (e[k] < thold && k < s1) k++;
                s0 = k;
                tk[j].t0 = sample_to_ts(k, seg.t0);
            }
        }
        {
            int k = s1;
            if (e[k] > thold) {
                while (k < n_samples - 1 && e[k] > thold) k++;
                tk[j].t1 = sample_to_ts(k, seg.t0);
                if (j < n - 1 && tk[j].t1 > tk[j + 1].t0) tk[j].t1 = tk[j + 1].t0;
                else s1 = k;
            } else {
                while (e[k] < thold && k > s0) k--;
                s1 = k;
                tk[j].t1 = sample_to_ts(k, seg.t0);
            }
        }
    }
}

static int utf8_len(const char * s) {
    int c = 0;
    for (; *s; ++s)
        if ((*s & 0xC0) != 0x80) c++;
    return c;
}

int wrap_segment(whisper_context * ctx, whisper_state * st, int max_len, bool split_on_word) {
    const Vocab & v = ctx->model->vocab;
    Segment seg = st->result_all.back();
    int res = 1, acc = 0;
    std::string text;
    for (int i = 0; i < (int) seg.tokens.size(); i++) {
        const auto & token = seg.tokens[i];
        if (token.id >= v.eot) continue;
        const std::string & txt = v.id_to_token[token.id];
        const int cur = utf8_len(txt.c_str());
        const bool split_ok = !split_on_word || txt[0] == ' ';
        if (acc + cur > max_len && i > 0 && split_ok) {
            st->result_all.back().text = std::move(text);
            st->result_all.back().t1 = token.t0;
            st->result_all.back().tokens.resize(i);
            st->result_all.back().speaker_turn_next = false;
            Segment ns;
            ns.t0 = token.t0;
            ns.t1 = seg.t1;
            ns.tokens.insert(ns.tokens.end(), seg.tokens.begin() + i, seg.tokens.end());
            ns.speaker_turn_next = seg.speaker_turn_next;
            ns.no_speech_prob = 0.0f;
            st->result_all.push_back(ns);
            acc = 0;
            text = "";
            seg = st->result_all.back();
            i = -1;
            res++;
        } else {
            acc += cur;
            text += txt.c_str();  // C string (ref 6121)
        }
    }
    st->result_all.back().text = std::move(text);
    return res;
}

// ---------------------------------------------------------------------------------
// DTW token timestamps (ref whisper_exp_compute_token_level_timestamps_dtw, 8837-8998;
// median_filter 8802-8835; dtw_and_backtrace 8712-8796). `cap` holds the f32 cross-attention
// probabilities of the alignment heads from the re-decode of [sot (lang) not text.. eot]:
// cap[(k * n_audio_ctx + j) * n_tok + t] for head k, audio position j, token t -- the layout of
// the reference's aheads_cross_QKs.
// ---------------------------------------------------------------------------------
// DTW over the captured probabilities; returns, for each new text position of the path in
// order, the DTW time index (what the reference's placement loop assigns token by token)
std::vector<int32_t> dtw_time_indices(const float * cap, int n_ah, int n_audio_ctx, int n_tok, int sot_len, int n_frames,
                                      int medfilt) {
    std::vector<int32_t> out;
    const int n_audio = n_frames / 2;
    // the capture holds n_audio_ctx positions per head: the reference asserts n_frames <= 2 *
    // n_audio_ctx (ref whisper.cpp:8850; a reduced audio_ctx with a longer window); fail the call
    // instead of reading past the capture
    if (n_frames > 2 * n_audio_ctx)
        throw std::runtime_error("DTW timestamps: n_frames " + std::to_string(n_frames) + " > 2 * n_audio_ctx " +
                                 std::to_string(n_audio_ctx) + " (ref whisper.cpp:8850 asserts)");
    if (n_ah <= 0 || n_audio <= medfilt || n_tok <= sot_len + 1) return out;
    // copy the first n_audio positions and normalise over tokens (ggml_norm, eps 1e-9;
    // ops.cpp:3578-3623: float mean of a double sum, centred variance accumulated in double
    // over 16-lane partial sums (vec.cpp:472-546), scale = 1/sqrtf(var + eps))
    std::vector<float> w((size_t) n_ah * n_audio * n_tok);
    for (int k = 0; k < n_ah; ++k)
        for (int j = 0; j < n_audio; ++j) {
            const float * x = &cap[((size_t) k * n_audio_ctx + j) * n_tok];
            float * y = &w[((size_t) k * n_audio + j) * n_tok];
            double s = 0.0;
            for (int t = 0; t < n_tok; ++t) s += (double) x[t];
            const float mean = (float) s / (float) n_tok;
            double s2 = 0.0;
            int t = 0;
            for (; t + 15 < n_tok; t += 16) {
                float lane[16];
                for (int e = 0; e < 16; ++e) {
                    y[t + e] = x[t + e] - mean;
                    lane[e] = y[t + e] * y[t + e];
                }
                for (int h = 8; h > 0; h >>= 1)  // _mm512_reduce_add_ps: pairwise halves
                    for (int e = 0; e < h; ++e) lane[e] = lane[e] + lane[e + h];
                s2 += (double) lane[0];
            }
            for (; t < n_tok; ++t) {
                y[t] = x[t] - mean;
                s2 += (double) (y[t] * y[t]);
            }
            const float var = (float) (s2 / n_tok);
            const float sc = 1.0f / sqrtf(var + 1e-9f);
            for (int u = 0; u < n_tok; ++u) y[u] *= sc;
        }
    // median filter (width medfilt, reflect padding) along audio, mean over heads, * -1;
    // the sot sequence and eot columns are dropped. The median is a selection (exact whatever the
    // method): for each (head, audio position) the filter's rows are contiguous over the tokens, so
    // the width-7 filter is a 16-comparator sorting network over whole token rows (vectorised over
    // tokens); the head sum is accumulated in double in head order, as ggml_mean's ggml_vec_sum_f32
    const int N = n_tok - sot_len - 1, M = n_audio;
    std::vector<float> xm((size_t) N * M);  // [audio j][token i]
    std::vector<double> hsum((size_t) N * M, 0.0);
    const int fw = 2 * (medfilt / 2) + 1;  // the reference's window: offsets -medfilt/2 .. medfilt/2
    std::vector<float> med((size_t) N), filt((size_t) fw);
    auto reflect = [&](int idx) { return idx < 0 ? -idx : idx >= M ? 2 * (M - 1) - idx : idx; };
    for (int k = 0; k < n_ah; ++k)
        for (int j = 0; j < M; ++j) {
            if (fw == 7) {
                const float * r[7];
                for (int off = -3; off <= 3; ++off) r[off + 3] = &w[((size_t) k * n_audio + reflect(j + off)) * n_tok + sot_len];
                for (int i = 0; i < N; ++i) {
                    float a[7];
                    for (int e = 0; e < 7; ++e) a[e] = r[e][i];
                    auto ce = [&](int p, int q) {
                        const float lo = a[q] < a[p] ? a[q] : a[p], hi = a[q] < a[p] ? a[p] : a[q];
                        a[p] = lo;
                        a[q] = hi;
                    };
                    ce(0, 6); ce(2, 3); ce(4, 5); ce(0, 2); ce(1, 4); ce(3, 6); ce(0, 1); ce(2, 5);
                    ce(3, 4); ce(1, 2); ce(4, 6); ce(2, 3); ce(4, 5); ce(1, 2); ce(3, 4); ce(5, 6);
                    med[i] = a[3];
                }
            } else {
                for (int i = 0; i < N; ++i) {
                    for (int off = -medfilt / 2; off <= medfilt / 2; ++off)
                        filt[off + medfilt / 2] = w[((size_t) k * n_audio + reflect(j + off)) * n_tok + sot_len + i];
                    std::nth_element(filt.begin(), filt.begin() + medfilt / 2, filt.end());
                    med[i] = filt[medfilt / 2];
                }
            }
            double * hs = &hsum[(size_t) j * N];
            for (int i = 0; i < N; ++i) hs[i] += (double) med[i];
        }
    for (size_t q = 0; q < xm.size(); ++q) {
        float mval = (float) hsum[q];
        mval /= (float) n_ah;
        xm[q] = mval * -1.0f;
    }
    // DTW cost / trace over (token i, audio j), then backtrace
    std::vector<float> cost((size_t) (N + 1) * (M + 1), INFINITY);
    std::vector<int32_t> trace((size_t) (N + 1) * (M + 1), -1);
    auto C = [&](int i, int j) -> float & { return cost[(size_t) j * (N + 1) + i]; };
    auto Tr = [&](int i, int j) -> int32_t & { return trace[(size_t) j * (N + 1) + i]; };
    C(0, 0) = 0.0f;
    for (int j = 1; j <= M; ++j)
        for (int i = 1; i <= N; ++i) {
            const float c0 = C(i - 1, j - 1), c1 = C(i - 1, j), c2 = C(i, j - 1);
            float c;
            int32_t tt;
            if (c0 < c1 && c0 < c2) { c = c0; tt = 0; }
            else if (c1 < c0 && c1 < c2) { c = c1; tt = 1; }
            else { c = c2; tt = 2; }
            C(i, j) = xm[(size_t) (j - 1) * N + (i - 1)] + c;
            Tr(i, j) = tt;
        }
    for (int j = 0; j <= M; ++j) Tr(0, j) = 2;
    for (int i = 0; i <= N; ++i) Tr(i, 0) = 1;
    std::vector<std::pair<int32_t, int32_t>> path;  // (text index, time index), reversed
    for (int i = N, j = M; i > 0 || j > 0;) {
        path.emplace_back(i - 1, j - 1);
        const int32_t tt = Tr(i, j);
        if (tt == 0) { --i; --j; }
        else if (tt == 1) { --i; }
        else if (tt == 2) { --j; }
        else throw std::runtime_error("dtw: bad trace");
    }
    std::reverse(path.begin(), path.end());
    int32_t last_v = 0;
    for (const auto & pv : path) {
        if (pv.first == last_v) continue;
        last_v = pv.first;
        out.push_back(pv.second);
    }
    return out;
}

void dtw_timestamps(whisper_context * ctx, whisper_state * st, int i_segment, int n_segments, int seek, int n_frames,
                    int medfilt, const std::vector<float> & cap, int n_ah, int n_audio_ctx, int n_tok, int sot_len) {
    const std::vector<int32_t> tix = dtw_time_indices(cap.data(), n_ah, n_audio_ctx, n_tok, sot_len, n_frames, medfilt);
    // place timestamps on the text tokens of the segments (each DTW step = 20 ms)
    const whisper_token eot = ctx->model->vocab.eot;
    auto & res = st->result_all;
    size_t si = (size_t) i_segment, ti = 0;
    auto next = [&]() {
        if (++ti >= res[si].tokens.size()) { ++si; ti = 0; }
    };
    for (const int32_t time_index : tix) {
        while (si < res.size() && (res[si].tokens.empty() || !(res[si].tokens[ti].id < eot))) {
            if (res[si].tokens.empty()) { ++si; ti = 0; continue; }
            next();
        }
        if (si >= res.size()) break;  // (the reference would run past the last segment here)
        res[si].tokens[ti].t_dtw = (int64_t) time_index * 2 + seek;
        next();
        if (si >= res.size()) break;
    }
    (void) n_segments;
}

} // namespace owk
