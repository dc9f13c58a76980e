// whisper_full for the MI355X engine: per-clip decoding state machines driven by a
// batch-major scheduler.
//
// Each clip runs the control flow of the reference whisper_full_with_state
// (ref src/whisper.cpp:6827-7776) -- windows/seek, temperature fallback, greedy /
// best-of / beam decoders, completion and failure rules, segment assembly -- but
// instead of calling the encoder/decoder synchronously it yields a request; the
// scheduler gathers the requests of all clips and runs one batched encode or one
// batched decoder pass for all of them. Batching changes no numerics: every decoder
// row is computed independently and the per-clip KV cell map mirrors the reference.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <regex>
#include <set>

#include "state.h"

namespace owk {

int64_t time_us() {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static const float HISTORY_TEMP_CUTOFF = 0.5f;  // WHISPER_HISTORY_CONDITIONING_TEMP_CUTOFF (ref 145)

static const char * const k_non_speech[] = {
    "\"", "#", "(", ")", "*", "+", "/", ":", ";", "<", "=", ">", "@", "[", "\\", "]", "^", "_", "`", "{", "|", "}",
    "~", "\xe3\x80\x8c", "\xe3\x80\x8d", "\xe3\x80\x8e", "\xe3\x80\x8f", "<<", ">>", "<<<", ">>>", "--", "---", "-(",
    "-[", "('", "(\"", "((", "))", "(((", ")))", "[[", "]]", "{{", "}}", "\xe2\x99\xaa\xe2\x99\xaa",
    "\xe2\x99\xaa\xe2\x99\xaa\xe2\x99\xaa", "\xe2\x99\xa9", "\xe2\x99\xaa", "\xe2\x99\xab", "\xe2\x99\xac",
    "\xe2\x99\xad", "\xe2\x99\xae", "\xe2\x99\xaf"};  // non_speech_tokens (ref 6130-6135)

VocabInfo vocab_info(const whisper_context * ctx, const whisper_full_params & p, std::vector<int> & suppress) {
    const Vocab & v = ctx->model->vocab;
    VocabInfo vi{};
    vi.n_vocab = v.n_vocab;
    vi.eot = v.eot; vi.sot = v.sot; vi.solm = v.solm; vi.prev = v.prev; vi.nosp = v.nosp; vi.not_ = v.not_;
    vi.beg = v.beg; vi.translate = v.translate; vi.transcribe = v.transcribe;
    auto it = v.token_to_id.find(" ");
    vi.space = it != v.token_to_id.end() ? it->second : -1;
    vi.lang_begin = v.sot + 1;
    vi.n_lang = (int) languages().size();
    // the initial timestamp cannot exceed max_initial_ts (ref 6313-6320)
    const float precision = float(WHISPER_CHUNK_SIZE) / ctx->model->hp.n_audio_ctx;
    vi.tid0_max = (int) std::round(p.max_initial_ts / precision);
    suppress.clear();
    if (p.suppress_nst) {
        for (const char * t : k_non_speech) {
            for (const std::string & s : {std::string(t), std::string(" ") + t}) {
                auto f = v.token_to_id.find(s);
                if (f != v.token_to_id.end()) suppress.push_back(f->second);
            }
        }
        for (const char * s : {" -", " '"}) {
            auto f = v.token_to_id.find(s);
            if (f != v.token_to_id.end()) suppress.push_back(f->second);
        }
    }
    if (p.suppress_regex != nullptr) {
        std::regex re(p.suppress_regex);
        for (const auto & kv : v.token_to_id)
            if (std::regex_match(kv.first, re)) suppress.push_back(kv.second);
    }
    vi.suppress_list = suppress.data();
    vi.n_suppress = (int) suppress.size();
    return vi;
}

// ---------------------------------------------------------------------------------
// host-side logit processing: used when a logits_filter_callback is installed (it
// must see the logits mid-way through the filters, ref 6254-6256). Same steps and
// order as the device kernel / reference whisper_process_logits (6177-6445).
// ---------------------------------------------------------------------------------
static void host_logprobs(const std::vector<float> & logits, std::vector<float> & logprobs) {
    const int n = (int) logits.size();
    const float mx = *std::max_element(logits.begin(), logits.end());
    float lse = 0.0f;
    for (int i = 0; i < n; ++i)
        if (logits[i] > -INFINITY) lse += expf(logits[i] - mx);
    lse = logf(lse) + mx;
    logprobs.resize(n);
    for (int i = 0; i < n; ++i) logprobs[i] = logits[i] > -INFINITY ? logits[i] - lse : -INFINITY;
}

static void host_process_logits(whisper_context * ctx, whisper_state * st, Decoder & dec, const whisper_full_params & p,
                                float temperature, const float * raw, const VocabInfo & vi) {
    const Vocab & v = ctx->model->vocab;
    const int n = v.n_vocab;
    const auto & toks = dec.sequence.tokens;
    const bool is_initial = toks.empty();
    auto & L = dec.logits;
    L.assign(raw, raw + n);
    if (temperature > 0.0f)
        for (auto & x : L) x /= temperature;
    if (p.suppress_blank && is_initial) {
        L[v.eot] = -INFINITY;
        if (vi.space >= 0) L[vi.space] = -INFINITY;
    }
    L[v.not_] = -INFINITY;
    if (p.no_timestamps)
        for (int i = v.beg; i < n; ++i) L[i] = -INFINITY;
    L[v.sot] = -INFINITY;
    L[v.nosp] = -INFINITY;
    if (!p.tdrz_enable) L[v.solm] = -INFINITY;
    L[v.translate] = -INFINITY;
    L[v.transcribe] = -INFINITY;
    L[v.prev] = -INFINITY;
    for (int i = 0; i < vi.n_lang; ++i) L[vi.lang_begin + i] = -INFINITY;
    if (p.logits_filter_callback)
        p.logits_filter_callback(ctx, st, toks.data(), (int) toks.size(), L.data(), p.logits_filter_callback_user_data);
    for (int i = 0; i < vi.n_suppress; ++i) L[vi.suppress_list[i]] = -INFINITY;
    {
        const bool last_ts = !toks.empty() && toks.back().id >= v.beg;
        const bool penult_ts = toks.size() < 2 || toks[toks.size() - 2].id >= v.beg;
        if (last_ts) {
            if (penult_ts) for (int i = v.beg; i < n; ++i) L[i] = -INFINITY;
            else for (int i = 0; i < v.eot; ++i) L[i] = -INFINITY;
        }
    }
    if (is_initial && p.max_initial_ts > 0.0f)
        for (int i = v.beg + vi.tid0_max + 1; i < n; ++i) L[i] = -INFINITY;
    if (dec.has_ts) {
        const int tid0 = dec.seek_delta / 2;
        for (int i = v.beg; i < v.beg + tid0; ++i) L[i] = -INFINITY;
    }
    host_logprobs(L, dec.logprobs);
    auto & lp = dec.logprobs;
    {
        float ts_lp = -INFINITY;
        const float lpmax = *std::max_element(lp.begin() + v.beg, lp.end());
        float s = 0.0f;
        for (int i = v.beg; i < n; ++i)
            if (lp[i] > -INFINITY) s += expf(lp[i] - lpmax);
        if (s > 0.0f) ts_lp = logf(s) + lpmax;
        const float tx = *std::max_element(lp.begin(), lp.begin() + v.beg);
        if (ts_lp > tx) {
            for (int i = 0; i < v.beg; ++i) { L[i] = -INFINITY; lp[i] = -INFINITY; }
        } else if (p.n_grammar_rules > 0) {
            // grammar: penalise the text tokens no parse stack accepts, then log_softmax again
            // (ref 6362-6384)
            dec.grammar.suppress(v.id_to_token, v.eot, p.grammar_penalty, L.data());
            host_logprobs(L, lp);
        }
    }
    dec.probs.resize(n);
    for (int i = 0; i < n; ++i) dec.probs[i] = L[i] == -INFINITY ? 0.0f : expf(lp[i]);
}

// timestamp statistics shared by the samplers (ref 6475-6493)
static void ts_stats(const Vocab & v, const std::vector<float> & probs, whisper_token_data & r) {
    double sum_ts = 0.0, max_ts = 0.0;
    for (int i = v.beg; i < v.n_vocab; ++i) {
        sum_ts += probs[i];
        if (max_ts < probs[i]) { max_ts = probs[i]; r.tid = i; }
    }
    r.pt = (float) (max_ts / (sum_ts + 1e-10));
    r.ptsum = (float) sum_ts;
}

static whisper_token_data sample_host(const Vocab & v, Decoder & dec, bool best) {
    whisper_token_data r = {0, 0, 0.0f, 0.0f, 0.0f, 0.0f, -1, -1, -1, 0.0f};
    ts_stats(v, dec.probs, r);
    if (best) {
        for (int i = 0; i < v.n_vocab; ++i)
            if (r.p < dec.probs[i]) { r.id = i; r.p = dec.probs[i]; r.plog = dec.logprobs[i]; }
    } else {
        std::discrete_distribution<> dist(dec.probs.begin(), dec.probs.end());
        r.id = dist(dec.rng);
        r.p = dec.probs[r.id];
        r.plog = dec.logprobs[r.id];
    }
    if (r.id >= v.beg) { r.tid = r.id; r.pt = r.p; }
    return r;
}

static whisper_token_data from_device(const Vocab & v, const TokenOut & t) {
    whisper_token_data r = {t.id, t.tid, t.p, t.plog, t.pt, t.ptsum, -1, -1, -1, 0.0f};
    (void) v;
    return r;
}

// beam candidates: k draws from the distribution (whisper_sample_token_topk, ref 6519-6592)
static std::vector<whisper_token_data> sample_topk(const Vocab & v, Decoder & dec, int k) {
    std::vector<whisper_token_data> out;
    whisper_token_data base = {0, v.beg, 0.0f, 0.0f, 0.0f, 0.0f, -1, -1, -1, 0.0f};
    ts_stats(v, dec.probs, base);
    std::discrete_distribution<> dist(dec.probs.begin(), dec.probs.end());
    for (int i = 0; i < k; ++i) {
        const int id = dist(dec.rng);
        whisper_token_data t = {id, base.tid, dec.probs[id], dec.logprobs[id], base.pt, base.ptsum, -1, -1, -1, 0.0f};
        if (t.id >= v.beg) { t.tid = t.id; t.pt = t.p; }
        out.push_back(t);
    }
    return out;
}

// whisper_sequence_score (ref 6595-6641)
static void sequence_score(const whisper_full_params & p, Sequence & s) {
    if (s.result_len == 0) return;
    double res = 0.0;
    for (int i = 0; i < s.result_len; ++i) res += s.tokens[i].plog;
    s.sum_logprobs = res;
    s.avg_logprobs = res / s.result_len;
    double penalty = s.result_len;
    if (p.length_penalty > 0.0f) penalty = pow((5.0 + penalty) / 6.0, p.length_penalty);
    s.score = res / penalty;
    const int n = 32;
    int cnt = 0;
    double entropy = 0.0;
    std::map<whisper_token, int> counts;
    for (int i = std::max(0, s.result_len - n); i < s.result_len; ++i) { counts[s.tokens[i].id]++; cnt++; }
    for (const auto & kv : counts) {
        const double q = kv.second / (double) cnt;
        entropy -= q * log(q);
    }
    s.entropy = entropy;
}

static bool seq_equal(const Sequence & a, const Sequence & b) {
    if (a.tokens.size() != b.tokens.size()) return false;
    for (int i = (int) a.tokens.size() - 1; i >= 0; i--)
        if (a.tokens[i].id != b.tokens[i].id) return false;
    return true;
}

void compute_token_timestamps(whisper_context * ctx, whisper_state * st, int i_segment, float thold_pt, float thold_ptsum);
std::vector<float> signal_energy(const float * signal, int n_samples, int n_samples_per_half_window);
int wrap_segment(whisper_context * ctx, whisper_state * st, int max_len, bool split_on_word);

// ---------------------------------------------------------------------------------
// per-clip decoding state machine
// ---------------------------------------------------------------------------------
enum class Phase { START, WINDOW, WAIT_ENCODE, ATTEMPT, WAIT_PREFILL, STEP, WAIT_STEP, FINISH, EMIT, LANG_WAIT_ENC,
                   LANG_WAIT_DEC, WAIT_DTW, DONE };

struct Clip {
    whisper_context * ctx;
    whisper_state * st;
    whisper_full_params p;
    const float * pcm;
    int n;
    int slot;
    Phase phase = Phase::START;
    int ret = 0;
    bool device_logits = true;  // greedy path on the device
    bool suppress_eot = false;
    bool pcm_on_device = false;  // owk_full_ext::samples_on_device

    int seek = 0, seek_start = 0, seek_end = 0;
    const int delta_min = 10;
    std::vector<float> temps;
    int it = 0;
    float t_cur = 0.0f;
    int n_decoders = 1, n_decoders_cur = 1;
    int max_prompt_ctx = 0;
    std::vector<whisper_token> prompt, prompt_init, prompt_tokens_buf;
    int best_decoder_id = 0;
    int i = 0, n_max = 0;

    struct BeamCand {
        int decoder_idx, seek_delta;
        bool has_ts;
        Sequence sequence;
        Grammar grammar;
    };
    std::vector<std::vector<BeamCand>> bc_per_dec;
    std::vector<BeamCand> beam_candidates;

    // pending decode call
    std::vector<CallToken> rows;
    int64_t t_req = 0;
    // pending DTW re-decode of the window's segments (ref 7744-7756)
    int dtw_seg0 = 0, dtw_nseg = 0, dtw_seek_delta = 0, dtw_sot_len = 0;

    const Vocab & vocab() const { return ctx->model->vocab; }
    const HParams & hp() const { return ctx->model->hp; }
    bool done() const { return phase == Phase::DONE; }
    bool waiting_encode() const { return phase == Phase::WAIT_ENCODE || phase == Phase::LANG_WAIT_ENC; }
    bool waiting_decode() const {
        return phase == Phase::WAIT_PREFILL || phase == Phase::WAIT_STEP || phase == Phase::LANG_WAIT_DEC ||
               phase == Phase::WAIT_DTW;
    }
    int encode_offset() const { return phase == Phase::LANG_WAIT_ENC ? 0 : seek; }

    void fail(int code) {
        ret = code;
        phase = Phase::DONE;
    }

    bool needs_host_probs() const {
        return !device_logits || t_cur > 0.0f || p.strategy == WHISPER_SAMPLING_BEAM_SEARCH;
    }

    // ---- start: everything of whisper_full_with_state before the main loop ----
    void start() {
        st->result_all.clear();
        const bool auto_lang = p.language == nullptr || strlen(p.language) == 0 || strcmp(p.language, "auto") == 0 ||
                               p.detect_language;
        if (auto_lang) {
            if (st->mel_n_len_org <= 0) { fail(-3); return; }
            phase = Phase::LANG_WAIT_ENC;
            return;
        }
        start_after_lang();
    }

    void start_after_lang() {
        if (p.token_timestamps) {
            st->t_beg = 0;
            st->t_last = 0;
            st->tid_last = 0;
            if (n > 0 && pcm_on_device) {
                std::vector<float> host(n);
                OWK_HIP_CHECK(hipMemcpy(host.data(), pcm, (size_t) n * 4, hipMemcpyDeviceToHost));
                st->energy = signal_energy(host.data(), n, 32);
            } else if (n > 0) {
                st->energy = signal_energy(pcm, n, 32);
            }
        }
        seek_start = p.offset_ms / 10;
        seek_end = p.duration_ms == 0 ? st->mel_n_len_org : seek_start + p.duration_ms / 10;
        if (seek_end < seek_start + delta_min) {
            log_msg(GGML_LOG_LEVEL_WARN, "whisper_full_with_state: input is too short - %d ms < 100 ms\n",
                    (seek_end - seek_start) * 10);
            phase = Phase::DONE;
            return;
        }
        temps.clear();
        if (p.temperature_inc > 0.0f) {
            for (float t = p.temperature; t < 1.0f + 1e-6f; t += p.temperature_inc) temps.push_back(t);
        } else {
            temps.push_back(p.temperature);
        }
        n_decoders = 1;
        if (p.strategy == WHISPER_SAMPLING_GREEDY) n_decoders = p.greedy.best_of;
        else n_decoders = std::max(p.greedy.best_of, p.beam_search.beam_size);
        n_decoders = std::max(1, n_decoders);
        if (n_decoders > MAX_DECODERS) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full_with_state: too many decoders requested (%d), max = %d\n",
                    n_decoders, MAX_DECODERS);
            fail(-4);
            return;
        }
        for (int j = 1; j < n_decoders; ++j) st->decoders[j].rng = std::mt19937(j);
        if (p.no_context) {
            st->prompt_past0.clear();
            st->prompt_past1.clear();
        }
        max_prompt_ctx = std::min(p.n_max_text_ctx, hp().n_text_ctx / 2);
        // initial prompt (ref 6944-6979)
        if (!p.prompt_tokens && p.initial_prompt) {
            prompt_tokens_buf.resize(1024);
            int nn = whisper_tokenize(ctx, p.initial_prompt, prompt_tokens_buf.data(), (int) prompt_tokens_buf.size());
            if (nn < 0) {
                prompt_tokens_buf.resize(-nn);
                nn = whisper_tokenize(ctx, p.initial_prompt, prompt_tokens_buf.data(), (int) prompt_tokens_buf.size());
            }
            prompt_tokens_buf.resize(nn);
            p.prompt_tokens = prompt_tokens_buf.data();
            p.prompt_n_tokens = (int) prompt_tokens_buf.size();
        }
        if (p.prompt_tokens && p.prompt_n_tokens > 0) {
            if (p.carry_initial_prompt) {
                if (st->prompt_past0.empty()) {
                    const int max_tokens = std::max(1, max_prompt_ctx - 1);
                    const int nt = std::min(p.prompt_n_tokens, max_tokens);
                    st->prompt_past0.assign(p.prompt_tokens + (p.prompt_n_tokens - nt), p.prompt_tokens + p.prompt_n_tokens);
                }
            } else {
                for (int k = 0; k < p.prompt_n_tokens; ++k) st->prompt_past1.push_back(p.prompt_tokens[k]);
                std::rotate(st->prompt_past1.begin(), st->prompt_past1.end() - p.prompt_n_tokens, st->prompt_past1.end());
            }
        }
        if (p.audio_ctx > hp().n_audio_ctx) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full_with_state: audio_ctx is larger than the maximum allowed (%d > %d)\n",
                    p.audio_ctx, hp().n_audio_ctx);
            fail(-5);
            return;
        }
        st->exp_n_audio_ctx = p.audio_ctx;  // ref 6986 (the engine runs the batch at this n_ctx)
        prompt_init = {vocab().sot};
        if (vocab().is_multilingual()) {
            const int lid = whisper_lang_id(p.language);
            st->lang_id = lid;
            prompt_init.push_back(vocab().sot + 1 + lid);
            prompt_init.push_back(p.translate ? vocab().translate : vocab().transcribe);
        }
        {
            const bool is_distil = hp().n_text_layer == 2 && hp().n_vocab != 51866;
            if (is_distil && !p.no_timestamps) p.no_timestamps = true;
        }
        if (p.no_timestamps) prompt_init.push_back(vocab().not_);
        seek = seek_start;
        bc_per_dec.assign(n_decoders, {});
        n_max = hp().n_text_ctx / 2 - 4;
        phase = Phase::WINDOW;
    }

    // ---- drive until the clip waits on the device or is done ----
    void advance() {
        for (;;) {
            switch (phase) {
                case Phase::START: start(); break;
                case Phase::WINDOW: window(); break;
                case Phase::ATTEMPT: attempt(); break;
                case Phase::STEP: step(); break;
                case Phase::FINISH: finish(); break;
                case Phase::EMIT: emit(); break;
                default: return;  // waiting or done
            }
        }
    }

    void window() {
        if (p.progress_callback) {
            const int progress = (100 * (seek - seek_start)) / (seek_end - seek_start);
            p.progress_callback(ctx, st, progress, p.progress_callback_user_data);
        }
        if (seek + delta_min >= seek_end) { phase = Phase::DONE; return; }
        if (p.encoder_begin_callback && !p.encoder_begin_callback(ctx, st, p.encoder_begin_callback_user_data)) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full_with_state: encoder_begin_callback returned false - aborting\n");
            phase = Phase::DONE;
            return;
        }
        phase = Phase::WAIT_ENCODE;
    }

    void on_encoded() {
        st->n_encode++;
        if (phase == Phase::LANG_WAIT_ENC) {
            // the language probe encodes through whisper_encode_with_state: no abort check
            // (ref whisper.cpp:3918, 4047)
            rows.assign(1, CallToken{vocab().sot, 0, 0, true});
            st->kv.seq_rm(0, 0, -1);
            phase = Phase::LANG_WAIT_DEC;
            return;
        }
        // whisper_encode_internal's last act: the abort check (ref whisper.cpp:2455 -> 7055-7058)
        if (p.abort_callback && p.abort_callback(p.abort_callback_user_data)) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full_with_state: failed to encode\n");
            fail(-6);
            return;
        }
        if (seek > seek_start && seek + 500 >= seek_end) {
            st->prompt_past0.clear();
            st->prompt_past1.clear();
        }
        best_decoder_id = 0;
        it = 0;
        phase = Phase::ATTEMPT;
    }

    void attempt() {
        t_cur = temps[it];
        n_decoders_cur = 1;
        if (p.strategy == WHISPER_SAMPLING_GREEDY) {
            if (t_cur > 0.0f) n_decoders_cur = p.greedy.best_of;
        } else {
            n_decoders_cur = t_cur > 0.0f ? p.greedy.best_of : p.beam_search.beam_size;
        }
        n_decoders_cur = std::max(1, n_decoders_cur);
        for (int j = 0; j < n_decoders_cur; ++j) {
            Decoder & d = st->decoders[j];
            d.sequence.tokens.clear();
            d.sequence.result_len = 0;
            d.sequence.sum_logprobs_all = 0.0;
            d.sequence.sum_logprobs = -INFINITY;
            d.sequence.avg_logprobs = -INFINITY;
            d.sequence.entropy = 0.0;
            d.sequence.score = -INFINITY;
            d.seek_delta = 100 * WHISPER_CHUNK_SIZE;
            d.failed = false;
            d.completed = false;
            d.has_ts = false;
            // ref 7113-7117 (a rule count of 0 leaves the grammar inactive)
            if (p.grammar_rules != nullptr) d.grammar.init(p.grammar_rules, p.n_grammar_rules, p.i_start_rule);
            else d.grammar = Grammar{};
        }
        prompt.clear();
        if (p.n_max_text_ctx > 0 && t_cur < HISTORY_TEMP_CUTOFF) {
            const bool can0 = p.carry_initial_prompt && !st->prompt_past0.empty();
            const bool can1 = !st->prompt_past1.empty();
            if (max_prompt_ctx > 0 && (can0 || can1)) {
                prompt.push_back(vocab().prev);
                int n_take0 = 0;
                if (can0) {
                    n_take0 = (int) st->prompt_past0.size();
                    prompt.insert(prompt.end(), st->prompt_past0.end() - n_take0, st->prompt_past0.end());
                }
                const int n_take1 = std::min<int>(max_prompt_ctx - n_take0 - 1, (int) st->prompt_past1.size());
                prompt.insert(prompt.end(), st->prompt_past1.end() - n_take1, st->prompt_past1.end());
            }
        }
        prompt.insert(prompt.end(), prompt_init.begin(), prompt_init.end());
        // recreate (re-size) the KV cell map when more decoders are needed (ref 7157-7175)
        if (st->kv_self_n_dec < n_decoders_cur) {
            const int factor = n_decoders_cur > 1 ? n_decoders_cur + 2 : 1;
            st->kv.init((uint32_t) (((hp().n_text_ctx + 255) / 256 * 256) * factor));
            st->kv_self_n_dec = n_decoders_cur;
        }
        st->kv.clear();
        rows.clear();
        for (int k = 0; k < (int) prompt.size(); ++k) rows.push_back(CallToken{prompt[k], k, 0, k == (int) prompt.size() - 1});
        phase = Phase::WAIT_PREFILL;
    }

    // device results of the pending call (decoder rows are in call order)
    void on_prefill() {
        Decoder & d0 = st->decoders[0];
        d0.i_batch = (int) prompt.size() - 1;
        for (int j = 1; j < n_decoders_cur; ++j) {
            Decoder & d = st->decoders[j];
            st->kv.seq_cp(0, j, -1, -1);
            d.probs = d0.probs;
            d.logits = d0.logits;
            d.logprobs = d0.logprobs;
            d.gtok = d0.gtok;
        }
        i = 0;
        phase = Phase::STEP;
    }

    void step() {
        if (i >= n_max) { phase = Phase::FINISH; return; }
        const int64_t t0 = time_us();
        if (p.strategy == WHISPER_SAMPLING_BEAM_SEARCH)
            for (auto & bc : bc_per_dec) bc.clear();
        for (int j = 0; j < n_decoders_cur; ++j) {
            Decoder & d = st->decoders[j];
            if (d.completed || d.failed) continue;
            if (p.strategy == WHISPER_SAMPLING_GREEDY) {
                whisper_token_data tok;
                if (t_cur < 1e-6f) tok = device_logits ? from_device(vocab(), d.gtok) : sample_host(vocab(), d, true);
                else tok = sample_host(vocab(), d, false);
                d.sequence.tokens.push_back(tok);
                d.sequence.sum_logprobs_all += tok.plog;
            } else {
                const auto toks = sample_topk(vocab(), d, p.beam_search.beam_size);
                for (const auto & tok : toks) {
                    bc_per_dec[j].push_back({j, d.seek_delta, d.has_ts, d.sequence, d.grammar});
                    bc_per_dec[j].back().sequence.tokens.push_back(tok);
                    bc_per_dec[j].back().sequence.sum_logprobs_all += tok.plog;
                }
            }
        }
        beam_candidates.clear();
        for (const auto & bc : bc_per_dec) {
            beam_candidates.insert(beam_candidates.end(), bc.begin(), bc.end());
            if (!bc.empty()) st->n_sample += 1;
        }
        if (p.strategy == WHISPER_SAMPLING_BEAM_SEARCH) {
            std::sort(beam_candidates.begin(), beam_candidates.end(), [](const BeamCand & a, const BeamCand & b) {
                if (a.sequence.sum_logprobs_all != b.sequence.sum_logprobs_all)
                    return a.sequence.sum_logprobs_all > b.sequence.sum_logprobs_all;
                return a.decoder_idx < b.decoder_idx;
            });
            uint32_t cur_c = 0;
            for (int j = 0; j < n_decoders_cur; ++j) {
                Decoder & d = st->decoders[j];
                if (d.completed || d.failed) continue;
                if (cur_c >= beam_candidates.size()) cur_c = 0;
                auto & cur = beam_candidates[cur_c++];
                while (beam_candidates.size() > cur_c && seq_equal(beam_candidates[cur_c].sequence, cur.sequence) && i > 0)
                    ++cur_c;
                d.seek_delta = cur.seek_delta;
                d.has_ts = cur.has_ts;
                d.sequence = cur.sequence;
                d.grammar = cur.grammar;
                st->kv.seq_cp(cur.decoder_idx, MAX_DECODERS + j, -1, -1);
            }
            for (int j = 0; j < n_decoders_cur; ++j) {
                Decoder & d = st->decoders[j];
                if (d.completed || d.failed) continue;
                st->kv.seq_rm(j, -1, -1);
                st->kv.seq_cp(MAX_DECODERS + j, j, -1, -1);
                st->kv.seq_rm(MAX_DECODERS + j, -1, -1);
            }
        }
        // update decoder state (ref 7355-7441)
        const int beg = vocab().beg;
        for (int j = 0; j < n_decoders_cur; ++j) {
            Decoder & d = st->decoders[j];
            if (d.completed || d.failed) continue;
            int & result_len = d.sequence.result_len;
            const auto & token = d.sequence.tokens.back();
            if (token.id > beg) {
                const int seek_delta_new = 2 * (token.id - beg);
                if (d.has_ts && d.seek_delta > seek_delta_new && result_len < i) {
                    d.failed = true;
                    continue;
                }
                d.seek_delta = seek_delta_new;
                result_len = i + 1;
                d.has_ts = true;
            }
            d.grammar.accept(vocab().id_to_token[token.id]);  // ref 7391
            if (token.id == vocab().eot || (p.max_tokens > 0 && i >= p.max_tokens) ||
                (d.has_ts && seek + d.seek_delta + delta_min >= seek_end)) {
                if (result_len == 0 && !p.no_timestamps) {
                    if (seek + d.seek_delta + delta_min >= seek_end) {
                        result_len = i + 1;
                    } else {
                        d.failed = true;
                        continue;
                    }
                }
                if (p.single_segment || p.no_timestamps) {
                    result_len = i + 1;
                    d.seek_delta = 100 * WHISPER_CHUNK_SIZE;
                }
                d.completed = true;
                continue;
            }
            if (ctx->model->n_loaded == 0) {
                d.seek_delta = 100 * WHISPER_CHUNK_SIZE;
                d.completed = true;
                continue;
            }
            if (i == n_max - 1 && (result_len == 0 || d.seek_delta < 100 * WHISPER_CHUNK_SIZE / 2)) {
                d.failed = true;
                continue;
            }
        }
        bool completed_all = true;
        for (int j = 0; j < n_decoders_cur; ++j)
            if (!st->decoders[j].completed && !st->decoders[j].failed) completed_all = false;
        st->t_sample_us += time_us() - t0;
        if (completed_all) { phase = Phase::FINISH; return; }
        rows.clear();
        const int n_past = (int) prompt.size() + i;
        for (int j = 0; j < n_decoders_cur; ++j) {
            Decoder & d = st->decoders[j];
            if (d.failed || d.completed) continue;
            d.i_batch = (int) rows.size();
            rows.push_back(CallToken{d.sequence.tokens.back().id, n_past, j, true});
        }
        phase = Phase::WAIT_STEP;
    }

    void on_step() {
        ++i;
        phase = Phase::STEP;
    }

    void finish() {
        double best_score = -INFINITY;
        for (int j = 0; j < n_decoders_cur; ++j) {
            Decoder & d = st->decoders[j];
            if (d.failed) continue;
            d.sequence.tokens.resize(d.sequence.result_len);
            sequence_score(p, d.sequence);
            if (d.sequence.result_len > 32 && d.sequence.entropy < p.entropy_thold) {
                d.failed = true;
                st->n_fail_h++;
                continue;
            }
            if (best_score < d.sequence.score) {
                best_score = d.sequence.score;
                best_decoder_id = j;
            }
        }
        bool success = true;
        if (it != (int) temps.size() - 1) {
            const Decoder & d = st->decoders[best_decoder_id];
            if (d.failed || (d.sequence.avg_logprobs < p.logprob_thold && st->no_speech_prob < p.no_speech_thold)) {
                success = false;
                st->n_fail_p++;
            }
        }
        if (success || it + 1 >= (int) temps.size()) {
            phase = Phase::EMIT;
        } else {
            ++it;
            phase = Phase::ATTEMPT;
        }
    }

    void emit() {
        const Decoder & best = st->decoders[best_decoder_id];
        int seek_delta = best.seek_delta;
        const int n_segments_before = (int) st->result_all.size();
        const int result_len = best.sequence.result_len;
        const auto & toks = best.sequence.tokens;
        auto & result_all = st->result_all;
        const int beg = vocab().beg, eot = vocab().eot;
        const bool is_no_speech = st->no_speech_prob > p.no_speech_thold && best.sequence.avg_logprobs < p.logprob_thold;

        st->prompt_past1.clear();
        if (!p.carry_initial_prompt && !prompt.empty() && prompt.front() == vocab().prev)
            st->prompt_past1.insert(st->prompt_past1.end(), prompt.begin() + 1, prompt.end() - prompt_init.size());
        if (!is_no_speech)
            for (int k = 0; k < result_len; ++k) st->prompt_past1.push_back(toks[k].id);

        if (!toks.empty() && ctx->model->n_loaded > 0 && !is_no_speech) {
            int i0 = 0;
            int64_t t0 = seek + 2 * (toks.front().tid - beg);
            std::string text;
            bool speaker_turn_next = false;
            for (int k = 0; k < (int) toks.size(); k++) {
                // C string, as the reference's whisper_token_to_str (ref 7651): a NUL-byte token adds nothing
                if (p.print_special || toks[k].id < eot) text += vocab().id_to_token[toks[k].id].c_str();
                if (p.tdrz_enable && toks[k].id == vocab().solm) speaker_turn_next = true;
                if (toks[k].id > beg && !p.single_segment) {
                    const int64_t t1 = seek + 2 * (toks[k].tid - beg);
                    if (!text.empty()) {
                        if (p.print_realtime) printf("%s\n", text.c_str());
                        Segment s;
                        s.t0 = t0; s.t1 = t1; s.text = text; s.no_speech_prob = st->no_speech_prob;
                        s.speaker_turn_next = speaker_turn_next;
                        for (int jj = i0; jj <= k; jj++) s.tokens.push_back(toks[jj]);
                        result_all.push_back(std::move(s));
                        int n_new = 1;
                        if (p.token_timestamps) {
                            compute_token_timestamps(ctx, st, (int) result_all.size() - 1, p.thold_pt, p.thold_ptsum);
                            if (p.max_len > 0) n_new = wrap_segment(ctx, st, p.max_len, p.split_on_word);
                        }
                        if (p.new_segment_callback && !ctx->params.dtw_token_timestamps)
                            p.new_segment_callback(ctx, st, n_new, p.new_segment_callback_user_data);
                    }
                    text = "";
                    while (k < (int) toks.size() && toks[k].id > beg) k++;
                    k--;
                    t0 = t1;
                    i0 = k + 1;
                    speaker_turn_next = false;
                }
            }
            if (!text.empty()) {
                const int64_t t1 = seek + seek_delta;
                if (p.print_realtime) printf("%s\n", text.c_str());
                Segment s;
                s.t0 = t0; s.t1 = t1; s.text = text; s.no_speech_prob = st->no_speech_prob;
                s.speaker_turn_next = speaker_turn_next;
                for (int jj = i0; jj < (int) toks.size(); jj++) s.tokens.push_back(toks[jj]);
                result_all.push_back(std::move(s));
                int n_new = 1;
                if (p.token_timestamps) {
                    compute_token_timestamps(ctx, st, (int) result_all.size() - 1, p.thold_pt, p.thold_ptsum);
                    if (p.max_len > 0) n_new = wrap_segment(ctx, st, p.max_len, p.split_on_word);
                }
                if (p.new_segment_callback && !ctx->params.dtw_token_timestamps)
                    p.new_segment_callback(ctx, st, n_new, p.new_segment_callback_user_data);
            }
        }
        // [EXPERIMENTAL] DTW token timestamps (ref 7744-7756): re-decode the window's text with
        // soft_max attention, capturing the alignment heads' cross-attention
        const int n_segments = (int) result_all.size() - n_segments_before;
        if (ctx->params.dtw_token_timestamps && n_segments) {
            dtw_seg0 = (int) result_all.size() - n_segments;
            dtw_nseg = n_segments;
            dtw_seek_delta = seek_delta;
            std::vector<whisper_token> tk = {vocab().sot};
            if (vocab().is_multilingual()) {
                const int lang_id = whisper_lang_id(p.language);
                st->lang_id = lang_id;
                tk.push_back(vocab().sot + 1 + lang_id);
            }
            dtw_sot_len = (int) tk.size();
            tk.push_back(vocab().not_);
            for (int s = dtw_seg0; s < dtw_seg0 + n_segments; ++s)
                for (const auto & t : result_all[s].tokens)
                    if (t.id < eot) tk.push_back(t.id);
            tk.push_back(eot);
            st->kv.clear();
            rows.clear();
            for (int k = 0; k < (int) tk.size(); ++k) rows.push_back(CallToken{tk[k], k, 0, k == (int) tk.size() - 1});
            phase = Phase::WAIT_DTW;
            return;
        }
        emit_tail(seek_delta);
    }

    void emit_tail(int seek_delta) {
        const auto & toks = st->decoders[best_decoder_id].sequence.tokens;
        const int beg = vocab().beg;
        const bool single_ts_ending = toks.size() > 1 && toks[toks.size() - 2].id < beg && toks[toks.size() - 1].id > beg;
        if (single_ts_ending) seek_delta = std::min(seek_end - seek, WHISPER_CHUNK_SIZE * 100);
        seek += seek_delta;
        phase = Phase::WINDOW;
    }

    // captured alignment-head attention of the DTW call: [head][n_audio_ctx][rows]
    void on_dtw(const std::vector<float> & cap, int n_ah) {
        const int n_frames = std::min(std::min(WHISPER_CHUNK_SIZE * 100, dtw_seek_delta), seek_end - seek);
        dtw_timestamps(ctx, st, dtw_seg0, dtw_nseg, seek, n_frames, 7, cap, n_ah, st->exp_n_audio_ctx > 0 ? st->exp_n_audio_ctx : hp().n_audio_ctx, (int) rows.size(),
                       dtw_sot_len);
        if (p.new_segment_callback) {  // the reference's loop bounds, verbatim (ref 7750-7754)
            for (int seg = (int) st->result_all.size() - dtw_nseg; seg < dtw_nseg; seg++)
                p.new_segment_callback(ctx, st, seg, p.new_segment_callback_user_data);
        }
        emit_tail(dtw_seek_delta);
    }
};

// ---------------------------------------------------------------------------------
// scheduler
// ---------------------------------------------------------------------------------
int prepare_decode_call(whisper_state * st, int slot, const std::vector<CallToken> & toks, std::vector<DecodeRow> & rows,
                        std::vector<int> & keys, int & n_logit) {
    const int nt = (int) toks.size();
    std::vector<int32_t> tp(nt), ts(nt);
    for (int r = 0; r < nt; ++r) { tp[r] = toks[r].pos; ts[r] = toks[r].seq; }
    const int cell0 = st->kv.find_slot(nt, tp.data(), ts.data());
    if (cell0 < 0) return -1;
    st->kv.n = std::min<uint32_t>(st->kv.size, std::max<int32_t>(1, st->kv.cell_max()));
    // reference flash-attention path choice per ggml_flash_attn_ext call (ops.cpp:8624-8628)
    // (flash_attn = false contexts: the soft_max path for both, whisper.cpp:2614-2628, 2697-2738)
    const int mode_self = !st->flash_attn ? 2 : (nt >= 32 && st->kv.n % 16 == 0) ? 1 : 0;
    const int mode_cross = !st->flash_attn ? 2 : nt >= 32 ? 1 : 0;
    for (int r = 0; r < nt; ++r) {
        DecodeRow x;
        x.slot = slot;
        x.token = toks[r].token;
        x.pos = toks[r].pos;
        x.cell = cell0 + r;
        x.key_off = (int) keys.size();
        st->kv.visible(toks[r].seq, toks[r].pos, keys);
        x.n_keys = (int) keys.size() - x.key_off;
        x.mode_self = mode_self;
        x.mode_cross = mode_cross;
        x.logit_row = toks[r].logits ? n_logit++ : -1;
        rows.push_back(x);
    }
    return cell0;
}

int full_batch(whisper_context * ctx, whisper_state ** states, const whisper_full_params * params_v,
               const owk_full_ext * ext, const float * const * samples, const int * n_samples, int n_clips) {
    if (n_clips <= 0) return 0;
    const whisper_full_params & params = params_v[0];
    // params.vad is whisper_full's pre-pass (whisper_api.cpp); like the reference's
    // whisper_full_with_state, the per-state path ignores it
    const Model & M = *ctx->model;
    OWK_HIP_CHECK(hipSetDevice(M.device));
    whisper_state * st0 = states[0];
    if (!st0->eng) st0->eng.reset(new Engine(&M, &ctx->prof));
    configure_engine(ctx, st0);
    Engine & eng = *st0->eng;

    // capacity: one slot per clip; self-KV cells for the largest decoder count
    int n_dec_max = params.strategy == WHISPER_SAMPLING_GREEDY ? params.greedy.best_of
                                                               : std::max(params.greedy.best_of, params.beam_search.beam_size);
    n_dec_max = std::max(1, std::min(n_dec_max, MAX_DECODERS));
    const int base_cells = (M.hp.n_text_ctx + 255) / 256 * 256;
    const int cells = base_cells * (n_dec_max > 1 ? n_dec_max + 2 : 1);
    eng.reserve(n_clips, std::max(cells, eng.kv_cells));
    // audio_ctx (ref whisper.cpp:6981-6986): one encoder width per batched call
    for (int c = 1; c < n_clips; ++c)
        if (params_v[c].audio_ctx != params.audio_ctx) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full: clips of one batch must share audio_ctx\n");
            return -5;
        }
    eng.audio_ctx = params.audio_ctx > 0 && params.audio_ctx <= M.hp.n_audio_ctx ? params.audio_ctx : 0;

    std::vector<Clip> clips(n_clips);
    for (int c = 0; c < n_clips; ++c) {
        Clip & k = clips[c];
        k.ctx = ctx;
        k.st = states[c];
        k.p = params_v[c];
        k.pcm = samples[c];
        k.n = n_samples[c];
        k.slot = c;
        // a logits_filter_callback or a grammar needs the logits on the host mid-filter (ref 6254, 6363)
        k.device_logits = params.logits_filter_callback == nullptr && params.n_grammar_rules == 0;
        k.suppress_eot = ext && ext->suppress_eot;
        k.pcm_on_device = ext && ext->samples_on_device;
        whisper_state * st = states[c];
        st->result_all.clear();
        if (st->kv.size == 0 || st->kv.size < (uint32_t) base_cells) st->kv.init(base_cells * (st->kv_self_n_dec > 1 ? st->kv_self_n_dec + 2 : 1));
        st->logits_rows = (int) st->logits_rowmax.size();
        eng.load_logits_state(c, st->logits_rowmax, st->logits_row0);
    }
    eng.sync();

    // mel for every clip with samples (whisper_pcm_to_mel_with_state)
    {
        std::vector<int> slots, ns;
        std::vector<const float *> pcm;
        for (int c = 0; c < n_clips; ++c)
            if (n_samples[c] > 0) { slots.push_back(c); pcm.push_back(samples[c]); ns.push_back(n_samples[c]); }
        const int64_t t0 = time_us();
        eng.compute_mel(slots, pcm, ns, ext && ext->samples_on_device);
        const int64_t dt = time_us() - t0;
        for (size_t i = 0; i < slots.size(); ++i) {
            whisper_state * st = states[slots[i]];
            st->mel_n_len = eng.mel_len(slots[i]);
            st->mel_n_len_org = 1 + (ns[i] + 200 - 400) / 160;
            st->mel_n_mel = M.n_filters_mel;
            st->t_mel_us += dt;
        }
        for (int c = 0; c < n_clips; ++c)
            if (n_samples[c] <= 0 && states[c]->mel_n_len <= 0) clips[c].fail(-2);
    }

    std::vector<int> suppress;
    VocabInfo vi = vocab_info(ctx, params, suppress);
    const int nv = M.hp.n_vocab;
    std::vector<float> hostbuf;

    for (;;) {
        for (auto & c : clips) c.advance();
        // 1) batched encoder for every clip waiting on it
        std::vector<int> enc_slots, enc_off;
        for (auto & c : clips)
            if (c.waiting_encode()) { enc_slots.push_back(c.slot); enc_off.push_back(c.encode_offset()); }
        if (!enc_slots.empty()) {
            const int64_t t0 = time_us();
            eng.encode(enc_slots, enc_off);
            eng.sync();
            const int64_t dt = time_us() - t0;
            for (auto & c : clips)
                if (c.waiting_encode()) { c.st->t_encode_us += dt; c.on_encoded(); }
            continue;
        }
        // 2) one batched decoder pass over every pending call
        std::vector<Clip *> dec;
        for (auto & c : clips)
            if (c.waiting_decode()) dec.push_back(&c);
        if (dec.empty()) break;

        std::vector<DecodeRow> rows;
        std::vector<int> keys;
        struct Span { int row0, n, lrow0; };
        std::vector<Span> spans;
        int n_logit = 0;
        for (Clip * c : dec) {
            const int row0 = (int) rows.size(), lrow0 = n_logit;
            if (prepare_decode_call(c->st, c->slot, c->rows, rows, keys, n_logit) < 0) {
                log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full: failed to find a KV slot\n");
                c->fail(c->phase == Phase::WAIT_PREFILL ? -8 : -9);
                spans.push_back({row0, 0, lrow0});
                continue;
            }
            spans.push_back({row0, (int) c->rows.size(), lrow0});
            c->t_req = time_us();
        }
        const int64_t t0 = time_us();
        bool capture = false;
        for (Clip * c : dec) capture = capture || c->phase == Phase::WAIT_DTW;
        eng.decode(rows, keys, n_logit, capture);

        // state->logits emulation (no-speech probability after each prefill, ref 7185-7195):
        // the reference resizes state->logits to the call's rows and overwrites only rows
        // that request logits; the rest keep stale values (zeros where the buffer grew)
        StepPost post;
        std::vector<Clip *> nclip;
        for (size_t ci = 0; ci < dec.size(); ++ci) {
            Clip * c = dec[ci];
            if (c->done() || spans[ci].n == 0) continue;
            const int old = c->st->logits_rows;
            const int nt = spans[ci].n;
            for (int r = 0; r < nt; ++r) {
                const DecodeRow & x = rows[spans[ci].row0 + r];
                const bool zero = r >= old;
                if (x.logit_row >= 0 || zero) post.rowmax.push_back(make_int4(c->slot, r, x.logit_row, zero ? 1 : 0));
            }
            c->st->logits_rows = nt;
            const DecodeRow & x0 = rows[spans[ci].row0];
            if (x0.logit_row >= 0) post.row0.push_back(make_int2(x0.logit_row, c->slot));
            else if (old == 0) post.row0.push_back(make_int2(-1, c->slot));
            if (c->phase == Phase::WAIT_PREFILL) {
                post.nosp.push_back(make_int2(c->slot, nt));
                nclip.push_back(c);
            }
        }

        // logits -> tokens: device path for every decoder row that needs no host callback
        std::vector<LogitJob> jobs;
        std::vector<std::pair<Clip *, int>> job_owner;  // (clip, decoder index)
        bool want_probs = false;
        for (size_t ci = 0; ci < dec.size(); ++ci) {
            Clip * c = dec[ci];
            if (c->done()) continue;
            const Span & sp = spans[ci];
            if (c->phase == Phase::LANG_WAIT_DEC || c->phase == Phase::WAIT_DTW) continue;  // handled below
            whisper_state * st = c->st;
            auto add_job = [&](int j, int lrow, bool nosp) {
                const Decoder & d = st->decoders[j];
                LogitJob jb;
                jb.row = lrow;
                const auto & toks = d.sequence.tokens;
                int f = 0;
                if (toks.empty()) f |= 1;
                if (!toks.empty() && toks.back().id >= vi.beg) f |= 2;
                if (toks.size() < 2 || toks[toks.size() - 2].id >= vi.beg) f |= 4;
                if (d.has_ts) f |= 8;
                if (c->p.suppress_blank) f |= 16;
                if (c->p.no_timestamps) f |= 32;
                if (c->p.tdrz_enable) f |= 64;
                if (c->suppress_eot) f |= 128;
                if (nosp) f |= 256;
                if (c->p.max_initial_ts > 0.0f) f |= 512;
                jb.flags = f;
                jb.ts_min = d.seek_delta / 2;
                jb.temperature = c->t_cur;
                jobs.push_back(jb);
                job_owner.push_back({c, j});
                if (c->needs_host_probs()) want_probs = true;
            };
            if (c->phase == Phase::WAIT_PREFILL) {
                add_job(0, sp.lrow0, false);
            } else {
                for (int j = 0; j < c->n_decoders_cur; ++j) {
                    const Decoder & d = st->decoders[j];
                    if (d.failed || d.completed) continue;
                    add_job(j, sp.lrow0 + d.i_batch, false);
                }
            }
        }
        // host path (logits_filter_callback): raw logits for every row, processed on the host
        const bool host_path = !clips.empty() && !clips[0].device_logits;
        std::vector<TokenOut> outs;
        std::vector<float> ns_out, probs_h, lp_h;
        if (host_path || jobs.empty()) {
            eng.step_post(post, {}, vi, outs, ns_out, nullptr, nullptr);
            if (host_path) {
                hostbuf.resize(nv);
                for (size_t q = 0; q < jobs.size(); ++q) {
                    Clip * c = job_owner[q].first;
                    Decoder & d = c->st->decoders[job_owner[q].second];
                    eng.download_logits(jobs[q].row, hostbuf.data());
                    host_process_logits(ctx, c->st, d, c->p, c->t_cur, hostbuf.data(), vi);
                }
            }
        } else {
            if (want_probs) {
                probs_h.resize(jobs.size() * (size_t) nv);
                lp_h.resize(jobs.size() * (size_t) nv);
            }
            eng.step_post(post, jobs, vi, outs, ns_out, want_probs ? probs_h.data() : nullptr,
                          want_probs ? lp_h.data() : nullptr);
            for (size_t q = 0; q < jobs.size(); ++q) {
                Clip * c = job_owner[q].first;
                Decoder & d = c->st->decoders[job_owner[q].second];
                d.gtok = outs[q];
                if (want_probs) {
                    d.probs.assign(probs_h.begin() + q * nv, probs_h.begin() + (q + 1) * nv);
                    d.logprobs.assign(lp_h.begin() + q * nv, lp_h.begin() + (q + 1) * nv);
                }
            }
        }
        for (size_t q = 0; q < nclip.size(); ++q) nclip[q]->st->no_speech_prob = ns_out[q];
        const int64_t dt = time_us() - t0;
        // completions
        for (size_t ci = 0; ci < dec.size(); ++ci) {
            Clip * c = dec[ci];
            if (c->done()) continue;
            whisper_state * st = c->st;
            const int nt = spans[ci].n;
            if (nt == 1) { st->t_decode_us += dt; st->n_decode++; }
            else if (nt < 16) { st->t_batchd_us += dt; st->n_batchd += nt; }
            else { st->t_prompt_us += dt; st->n_prompt += nt; }
            // whisper_decode_internal's abort check (ref whisper.cpp:2977) for the prompt and step
            // decodes of whisper_full (7181, 7493); the language probe and the DTW re-decode pass
            // no callback (4047, 8891)
            if (c->phase != Phase::LANG_WAIT_DEC && c->phase != Phase::WAIT_DTW && c->p.abort_callback &&
                c->p.abort_callback(c->p.abort_callback_user_data)) {
                c->fail(c->phase == Phase::WAIT_PREFILL ? -8 : -9);
                continue;
            }
            if (c->phase == Phase::LANG_WAIT_DEC) {
                // language probabilities over the language tokens (ref 4052-4093)
                hostbuf.resize(nv);
                eng.download_logits(spans[ci].lrow0, hostbuf.data());
                std::vector<std::pair<float, int>> lid;
                for (const auto & kv : languages()) lid.emplace_back(hostbuf[vi.sot + 1 + kv.second.first], kv.second.first);
                std::sort(lid.begin(), lid.end(), [](const std::pair<float, int> & a, const std::pair<float, int> & b) {
                    return a.first > b.first;
                });
                const float mx = lid[0].first;
                double sum = 0.0;
                for (auto & kv : lid) { kv.first = exp(kv.first - mx); sum += kv.first; }
                for (auto & kv : lid) kv.first /= sum;
                st->lang_id = lid[0].second;
                c->p.language = whisper_lang_str(st->lang_id);
                log_msg(GGML_LOG_LEVEL_INFO, "whisper_full_with_state: auto-detected language: %s (p = %f)\n",
                        c->p.language, lid[0].first);
                if (c->p.detect_language) { c->phase = Phase::DONE; continue; }
                c->start_after_lang();
                continue;
            }
            if (c->phase == Phase::WAIT_DTW) {
                std::vector<float> cap;
                eng.download_capture(spans[ci].row0, nt, cap);
                c->on_dtw(cap, eng.n_aheads());
                continue;
            }
            if (c->phase == Phase::WAIT_PREFILL) c->on_prefill();
            else c->on_step();
        }
    }
    for (int c = 0; c < n_clips; ++c)
        eng.save_logits_state(c, states[c]->logits_rows, states[c]->logits_rowmax, states[c]->logits_row0);
    int ret = 0;
    for (auto & c : clips)
        if (c.ret != 0 && ret == 0) ret = c.ret;
    return ret;
}

} // namespace owk
