// TEST INFRASTRUCTURE — parity oracle probe, never part of the product.
//
// Compiles the reference implementation in place (#include of
// /root/reference/src/whisper.cpp; nothing is copied into this repo) and adds a
// handful of extern "C" accessors so tests/golden generators and bench.py's
// cpu_baseline leg can read reference intermediates through ctypes:
//   - the log-mel spectrogram        (whisper_state::mel, whisper.cpp:3170-3260)
//   - the encoder output embd_enc    (whisper_build_graph_encoder, whisper.cpp:2038-2269)
//   - the cross-attention K/V cache  (whisper_build_graph_cross, whisper.cpp:2272-2346)
//   - decoder logits                 (whisper_decode_internal, whisper.cpp:2848-2978)
//   - whisper_full with a flat config struct (whisper_full_with_state, whisper.cpp:6827-7776)
#include "whisper.cpp"
#include "grammar-parser.h"

#include <mutex>

extern "C" {

struct ref_full_cfg {
    int   strategy;         // 0 greedy, 1 beam search
    int   n_threads;
    int   best_of;
    int   beam_size;
    float temperature;
    float temperature_inc;
    int   no_timestamps;
    int   max_tokens;
    int   suppress_eot;     // fixed-work mode: logits_filter_callback sets logits[eot] = -inf
    int   token_timestamps;
    int   no_context;
    int   single_segment;
    const char * language;
    int   suppress_nst;
    float length_penalty;
    int   record_topk;      // record + truncate logits to a top-K set (see ref_record_cb)
    int   audio_ctx;        // whisper_full_params.audio_ctx (0 = n_audio_ctx; whisper.cpp:6986)
    int   n_processors;     // > 1: whisper_full_parallel (whisper.cpp:7801-7929)
};

// ---------------------------------------------------------------------------------
// Logit recording for the stochastic strategies (sampling, beam search, temperature
// fallback). Their outcome depends on where an mt19937 draw lands in the CDF of the
// probabilities, so any f32 reordering can change a pick. For an exact comparison of
// the decoding *logic*, the golden run truncates every decoder's logits (at the
// logits_filter_callback point, whisper.cpp:6254) to a recorded set of entries:
//   top REC_TEXT finite text tokens (< token_beg), token_eot if finite, and the top
//   REC_TS finite timestamp tokens; everything else becomes -inf.
// The GPU test installs a callback that substitutes exactly these recorded values,
// keyed by the decoder's token prefix (nearest match on values when a prefix repeats).
static constexpr int REC_TEXT = 24, REC_TS = 16, REC_W = REC_TEXT + 1 + REC_TS;
static std::vector<int>   g_rec_prefix, g_rec_off, g_rec_idx;
static std::vector<float> g_rec_val;
static bool               g_rec_suppress_eot = false;
static std::mutex         g_rec_mtx;  // whisper_full runs process_logits of the decoders on worker threads

static bool g_rec_trace_only = false;  // record_topk == 2: record the prefixes, leave the logits alone

static void ref_record_cb(struct whisper_context * ctx, struct whisper_state * /*state*/,
                          const whisper_token_data * tokens, int n_tokens, float * logits, void * /*user_data*/) {
    const int n_vocab = whisper_n_vocab(ctx), eot = whisper_token_eot(ctx), beg = whisper_token_beg(ctx);
    if (g_rec_suppress_eot) logits[eot] = -INFINITY;
    auto top = [&](int lo, int hi, int k, std::vector<int> & out) {
        std::vector<int> ids;
        for (int i = lo; i < hi; ++i)
            if (logits[i] > -INFINITY && i != eot) ids.push_back(i);
        k = std::min<int>(k, (int) ids.size());
        std::partial_sort(ids.begin(), ids.begin() + k, ids.end(), [&](int a, int b) {
            return logits[a] > logits[b] || (logits[a] == logits[b] && a < b);
        });
        out.insert(out.end(), ids.begin(), ids.begin() + k);
    };
    std::vector<int> keep;
    top(0, beg, REC_TEXT, keep);
    if (logits[eot] > -INFINITY) keep.push_back(eot);
    top(beg, n_vocab, REC_TS, keep);
    {
        std::lock_guard<std::mutex> lock(g_rec_mtx);
        g_rec_off.push_back((int) g_rec_prefix.size());
        for (int i = 0; i < n_tokens; ++i) g_rec_prefix.push_back(tokens[i].id);
        for (int j = 0; j < REC_W; ++j) {
            const int id = j < (int) keep.size() ? keep[j] : -1;
            g_rec_idx.push_back(id);
            g_rec_val.push_back(id >= 0 ? logits[id] : -INFINITY);
        }
    }
    if (g_rec_trace_only) return;
    std::vector<float> kept(keep.size());
    for (size_t j = 0; j < keep.size(); ++j) kept[j] = logits[keep[j]];
    for (int i = 0; i < n_vocab; ++i) logits[i] = -INFINITY;
    for (size_t j = 0; j < keep.size(); ++j) logits[keep[j]] = kept[j];
}

// recorded entries: returns their count; with non-null outputs copies
//   off[n+1] (prefix offsets), prefix[off[n]], idx[n*REC_W], val[n*REC_W]
int ref_record_get(int * off, int * prefix, int * idx, float * val, int * width) {
    const int n = (int) g_rec_off.size();
    *width = REC_W;
    if (off) {
        for (int i = 0; i < n; ++i) off[i] = g_rec_off[i];
        off[n] = (int) g_rec_prefix.size();
        std::copy(g_rec_prefix.begin(), g_rec_prefix.end(), prefix);
        std::copy(g_rec_idx.begin(), g_rec_idx.end(), idx);
        std::copy(g_rec_val.begin(), g_rec_val.end(), val);
    }
    return n;
}

int ref_record_prefix_len() { return (int) g_rec_prefix.size(); }

static void ref_suppress_eot_cb(struct whisper_context * ctx, struct whisper_state * /*state*/,
                                const whisper_token_data * /*tokens*/, int /*n_tokens*/,
                                float * logits, void * /*user_data*/) {
    logits[whisper_token_eot(ctx)] = -INFINITY;
}

void * ref_init(const char * path, int flash_attn, int dtw_preset) {
    whisper_log_set([](ggml_log_level, const char *, void *) {}, nullptr);
    auto cp = whisper_context_default_params();
    cp.use_gpu    = false;
    cp.flash_attn = flash_attn != 0;
    if (dtw_preset > 0) {
        cp.dtw_token_timestamps = true;
        cp.dtw_aheads_preset    = (whisper_alignment_heads_preset) dtw_preset;
    }
    return whisper_init_from_file_with_params(path, cp);
}

// as ref_init with the N_TOP_MOST preset's layer count (whisper_context_params.dtw_n_top)
void * ref_init_ex(const char * path, int flash_attn, int dtw_preset, int dtw_n_top) {
    whisper_log_set([](ggml_log_level, const char *, void *) {}, nullptr);
    auto cp = whisper_context_default_params();
    cp.use_gpu    = false;
    cp.flash_attn = flash_attn != 0;
    if (dtw_preset > 0) {
        cp.dtw_token_timestamps = true;
        cp.dtw_aheads_preset    = (whisper_alignment_heads_preset) dtw_preset;
        cp.dtw_n_top            = dtw_n_top;
    }
    return whisper_init_from_file_with_params(path, cp);
}

void ref_free(void * ctx) { whisper_free((whisper_context *) ctx); }

// returns n_mel*n_len floats written (row-major [n_mel][n_len]); -1 on error
int ref_mel(void * vctx, const float * pcm, int n, int n_threads, float * out, int cap,
            int * n_len, int * n_len_org, int * n_mel) {
    auto * ctx = (whisper_context *) vctx;
    if (whisper_pcm_to_mel(ctx, pcm, n, n_threads) != 0) return -1;
    const auto & mel = ctx->state->mel;
    *n_len = mel.n_len; *n_len_org = mel.n_len_org; *n_mel = mel.n_mel;
    const int total = mel.n_len * mel.n_mel;
    if (out) {
        if (cap < total) return -1;
        memcpy(out, mel.data.data(), total * sizeof(float));
    }
    return total;
}

int ref_encode(void * vctx, int offset, int n_threads) {
    return whisper_encode((whisper_context *) vctx, offset, n_threads);
}

static int tensor_f32_out(ggml_tensor * t, float * out, int cap) {
    if (!t) return -1;
    const int64_t n = ggml_nelements(t);
    if (out) {
        if (cap < n) return -1;
        if (t->type == GGML_TYPE_F32) {
            ggml_backend_tensor_get(t, out, 0, n * sizeof(float));
        } else {
            return -2;
        }
    }
    return (int) n;
}

// encoder output [n_ctx][n_state] (token-major)
int ref_get_enc(void * vctx, float * out, int cap) {
    return tensor_f32_out(((whisper_context *) vctx)->state->embd_enc, out, cap);
}

// conv-stack output (layout ggml [n_state (ne0=time? see ref) ...])
int ref_get_conv(void * vctx, float * out, int cap, int * ne0, int * ne1) {
    ggml_tensor * t = ((whisper_context *) vctx)->state->embd_conv;
    if (!t) return -1;
    *ne0 = (int) t->ne[0]; *ne1 = (int) t->ne[1];
    return tensor_f32_out(t, out, cap);
}

// raw F16 cross K/V cache bytes; layout per whisper.cpp:2320-2325 (FA) or 2327-2334 (no FA)
long ref_get_cross(void * vctx, uint16_t * k, uint16_t * v, long cap) {
    auto * st = ((whisper_context *) vctx)->state;
    const long n = ggml_nelements(st->kv_cross.k);
    if (k && v) {
        if (cap < n) return -1;
        ggml_backend_tensor_get(st->kv_cross.k, k, 0, n * 2);
        ggml_backend_tensor_get(st->kv_cross.v, v, 0, n * 2);
    }
    return n;
}

int ref_decode(void * vctx, const int * tokens, int n_tokens, int n_past, int n_threads) {
    return whisper_decode((whisper_context *) vctx, tokens, n_tokens, n_past, n_threads);
}

float * ref_logits(void * vctx) { return whisper_get_logits((whisper_context *) vctx); }

// whisper_full's VAD pre-pass (whisper.cpp:7785-7796, 6643-6826): a non-null path turns it
// on for the following ref_full calls with whisper_vad_default_params()
static std::string g_vad_path;
void ref_set_vad(const char * path) { g_vad_path = path ? path : ""; }

// whisper_full_params fields beyond ref_full_cfg (the SDK / CLI branches: whisper.cpp:6944-6979
// initial prompt, 6990-6996 translate, 7035-7052 progress / encoder_begin, 7626-7760 segments,
// 6077-6128 wrap, 6213-6250 suppress_regex / nst / tdrz) and a recorder of every callback the
// reference invokes, in order.
struct ref_full_ext {
    const char * initial_prompt;
    int   carry_initial_prompt;
    int   translate;
    int   max_len;
    int   split_on_word;
    int   tdrz_enable;
    int   offset_ms;
    int   duration_ms;
    const char * suppress_regex;
    int   n_max_text_ctx;       // 0 = default
    int   print_special;
    int   callbacks;            // 1: install the recording callbacks (log: ref_cb_log)
    int   cancel_at_progress;   // > 0: CallbackBridge semantics -- the progress callback whose value is
                                // >= this sets shouldCancel, the abort callback returns it (-1 = never)
    int   enc_begin_false_at;   // > 0: encoder_begin_callback returns false on this call
    int   tdrz_boost;           // logits_filter: solm := 1000 when finite and n_tokens % 5 == 2
    float max_initial_ts;       // < 0: default
    int   suppress_blank;       // < 0: default
    int   detect_language;
};

// callback log: (kind, a, b) triples. kind 1 progress (value, n_segments), 2 encoder_begin (call #,
// returned), 3 abort checks (consecutive calls folded: count, last returned), 4 new_segment (n_new,
// n_segments), 5 new_segment segment text follows in g_cb_text
static std::vector<int> g_cb_log;
static std::vector<std::string> g_cb_text;
static int g_cb_enc_calls = 0, g_cb_enc_false_at = 0, g_cb_cancel_at = -1;
static bool g_cb_cancel = false;

static void cb_push(int k, int a, int b) {
    g_cb_log.push_back(k); g_cb_log.push_back(a); g_cb_log.push_back(b);
}
static void ref_cb_progress(whisper_context *, whisper_state * st, int progress, void *) {
    cb_push(1, progress, (int) st->result_all.size());
    if (g_cb_cancel_at >= 0 && progress >= g_cb_cancel_at) g_cb_cancel = true;
}
static bool ref_cb_enc_begin(whisper_context *, whisper_state *, void *) {
    ++g_cb_enc_calls;
    const bool ret = g_cb_enc_calls != g_cb_enc_false_at;
    cb_push(2, g_cb_enc_calls, ret ? 1 : 0);
    return ret;
}
static bool ref_cb_abort(void *) {
    const int n = (int) g_cb_log.size();
    if (n >= 3 && g_cb_log[n - 3] == 3 && g_cb_log[n - 1] == (g_cb_cancel ? 1 : 0)) {
        g_cb_log[n - 2]++;
    } else {
        cb_push(3, 1, g_cb_cancel ? 1 : 0);
    }
    return g_cb_cancel;
}
// as the Swift CallbackBridge reads it: the last n_new segments of the context's default state
static void ref_cb_new_segment(whisper_context * ctx, whisper_state * st, int n_new, void *) {
    const int total = (int) st->result_all.size();
    cb_push(4, n_new, total);
    for (int i = std::max(0, total - n_new); i < total; ++i) {
        g_cb_text.push_back(std::to_string(st->result_all[i].t0) + "|" + std::to_string(st->result_all[i].t1) + "|" +
                            st->result_all[i].text);
    }
    (void) ctx;
}
static void ref_tdrz_boost_cb(struct whisper_context * ctx, struct whisper_state *, const whisper_token_data *,
                              int n_tokens, float * logits, void *) {
    const int solm = whisper_token_solm(ctx);
    if (n_tokens % 5 == 2 && logits[solm] > -INFINITY) logits[solm] = 1000.0f;
}

int ref_cb_log(int * out, int cap) {
    if (out) std::copy(g_cb_log.begin(), g_cb_log.begin() + std::min<size_t>(cap, g_cb_log.size()), out);
    return (int) g_cb_log.size();
}
int ref_cb_n_text() { return (int) g_cb_text.size(); }
const char * ref_cb_text(int i) { return i >= 0 && i < (int) g_cb_text.size() ? g_cb_text[i].c_str() : nullptr; }

// whisper_tokenize as the reference runs it (whisper.cpp:3272-3320, 3957-3973)
int ref_tokenize(void * vctx, const char * text, int * out, int cap) {
    return whisper_tokenize((whisper_context *) vctx, text, out, cap);
}

static int ref_full_impl(void * vctx, const float * pcm, int n, const ref_full_cfg * cfg, const ref_full_ext * ext);

// ---------------------------------------------------------------------------------
// Teacher forcing with the reference's OWN greedy pick recorded at every step (round 5).
// ref_tf_set(tokens, off, n_windows, force): the per-window decoded token lists the next
// ref_full / ref_full_ex follows (force = 0: record only, nothing forced). At each
// logits_filter_callback (whisper.cpp:6254, inside whisper_process_logits) the callback
//   1. applies the run's own filter callback (fixed-work EOT suppression, tdrz boost);
//   2. runs the REST of the reference's whisper_process_logits and its greedy
//      whisper_sample_token (whisper.cpp:6177-6445, 6460-6592) on a copy of the decoder --
//      no restatement: the reference's own code decides what it would pick here;
//   3. records (window, step, pick, logprob of the pick, logprob of the teacher token);
//   4. forces the teacher token (its logit 40 above the finite maximum; <|endoftext|> after
//      a window's last listed token), as tests/parity_util.Forcer does on the GPU.
// Greedy at temperature 0 only (one decoder, no fallback; the callback has no temperature).
static std::vector<int> g_tf_tok, g_tf_off, g_tf_rec;
static std::vector<float> g_tf_lp;
static int g_tf_window = -1;
static bool g_tf_active = false, g_tf_force = true;
static whisper_full_params g_tf_params;
static whisper_logits_filter_callback g_tf_base = nullptr;

static std::vector<int> g_tf_open;  // per window: 1 = its end is open (no <|endoftext|> forced after it)

void ref_tf_set(const int * tokens, const int * off, int n_windows, int force) {
    g_tf_active = n_windows >= 0;
    g_tf_force = force != 0;
    g_tf_off.assign(off, off + std::max(n_windows, 0) + 1);
    g_tf_tok.assign(tokens, tokens + (n_windows > 0 ? off[n_windows] : 0));
    g_tf_open.assign(std::max(n_windows, 0), 0);
}

// windows whose end is open (the step limit, or a timestamp reaching the end of the audio): the step after
// the last listed token is left to the reference, as on the GPU (tests/parity_util.Forcer). Call after ref_tf_set.
void ref_tf_set_open(const int * open, int n_windows) {
    g_tf_open.assign(open, open + std::min<int>(n_windows, (int) g_tf_open.size()));
    g_tf_open.resize(g_tf_off.size() - 1, 0);
}

// recorded steps: returns their count; with non-null outputs rec[TF_NI n] = (window, step, pick,
// teacher token or -1, decoder index, TF_NC candidate ids) and lp[TF_NF n] = (logprob of pick, logprob
// of teacher, TF_NC candidate logits, timestamp log-mass, best text logit). The candidates are the
// TF_NC largest text / <|endoftext|> logits at the callback point (before forcing); the timestamp
// log-mass is the logsumexp of the timestamp logits the rest of whisper_process_logits leaves finite
// and the best text logit the largest text logit the timestamp pairing rule leaves (whisper.cpp:
// 6289-6357): the two sides of the timestamp rule, in logit units (same normaliser).
static constexpr int TF_NC = 16, TF_NI = 5 + TF_NC, TF_NF = 4 + TF_NC;
int ref_tf_get(int * rec, float * lp) {
    const int n = (int) g_tf_rec.size() / TF_NI;
    if (rec) std::copy(g_tf_rec.begin(), g_tf_rec.end(), rec);
    if (lp) std::copy(g_tf_lp.begin(), g_tf_lp.end(), lp);
    return n;
}

static void ref_tf_cb(struct whisper_context * ctx, struct whisper_state * state, const whisper_token_data * tokens,
                      int n_tokens, float * logits, void * ud) {
    if (g_tf_base) g_tf_base(ctx, state, tokens, n_tokens, logits, ud);
    if (n_tokens == 0) ++g_tf_window;
    const int w = g_tf_window;
    const int n_win = (int) g_tf_off.size() - 1;
    int teacher = -1;
    if (w >= 0 && w < n_win) {
        const int len = g_tf_off[w + 1] - g_tf_off[w];
        teacher = n_tokens < len ? g_tf_tok[g_tf_off[w] + n_tokens]
                                 : (n_tokens == len && !g_tf_open[w] ? whisper_token_eot(ctx) : -1);
    }
    int j = -1;
    for (int i = 0; i < WHISPER_MAX_DECODERS; ++i)
        if (state->decoders[i].logits.data() == logits) j = i;
    const int n_vocab = whisper_n_vocab(ctx), eot = whisper_token_eot(ctx), beg = whisper_token_beg(ctx);
    int pick = -1;
    float lp_pick = -INFINITY, lp_teacher = -INFINITY, ts_lse = -INFINITY, text_max = -INFINITY;
    if (j >= 0) {
        whisper_decoder dec = state->decoders[j];
        whisper_full_params p2 = g_tf_params;
        p2.logits_filter_callback = g_tf_base;
        whisper_process_logits(*ctx, *state, dec, p2, 0.0f);
        const whisper_token_data td = whisper_sample_token(*ctx, dec, true);
        pick = td.id;
        lp_pick = dec.logprobs[pick];
        if (teacher >= 0) lp_teacher = dec.logprobs[teacher];
        // the timestamp rule's two sides in logits: timestamps the filters left finite
        double mx = -INFINITY, acc = 0.0;
        for (int i = beg; i < n_vocab; ++i) if (dec.logits[i] > -INFINITY) mx = std::max(mx, (double) logits[i]);
        if (mx > -INFINITY) {
            for (int i = beg; i < n_vocab; ++i) if (dec.logits[i] > -INFINITY) acc += exp((double) logits[i] - mx);
            ts_lse = (float) (log(acc) + mx);
        }
        const bool last_ts = n_tokens > 0 && tokens[n_tokens - 1].id >= beg;
        const bool pen_ts = n_tokens < 2 || tokens[n_tokens - 2].id >= beg;
        if (!(last_ts && !pen_ts))
            for (int i = 0; i < beg; ++i) text_max = std::max(text_max, logits[i]);
    }
    std::vector<int> cand;
    for (int i = 0; i < beg; ++i) if (logits[i] > -INFINITY) cand.push_back(i);
    const int nc = std::min<int>(TF_NC, (int) cand.size());
    std::partial_sort(cand.begin(), cand.begin() + nc, cand.end(),
                      [&](int a, int b) { return logits[a] > logits[b] || (logits[a] == logits[b] && a < b); });
    g_tf_rec.insert(g_tf_rec.end(), {w, n_tokens, pick, teacher, j});
    g_tf_lp.insert(g_tf_lp.end(), {lp_pick, lp_teacher});
    for (int c = 0; c < TF_NC; ++c) {
        g_tf_rec.push_back(c < nc ? cand[c] : -1);
        g_tf_lp.push_back(c < nc ? logits[cand[c]] : -INFINITY);
    }
    g_tf_lp.insert(g_tf_lp.end(), {ts_lse, text_max});
    (void) eot;
    if (!g_tf_force || teacher < 0) return;
    float mx = -INFINITY;
    for (int i = 0; i < n_vocab; ++i) mx = std::max(mx, logits[i] > -INFINITY && logits[i] < INFINITY ? logits[i] : mx);
    logits[teacher] = (mx > -INFINITY ? mx : 0.0f) + 40.0f;
}

int ref_full(void * vctx, const float * pcm, int n, const ref_full_cfg * cfg) {
    return ref_full_impl(vctx, pcm, n, cfg, nullptr);
}

int ref_full_ex(void * vctx, const float * pcm, int n, const ref_full_cfg * cfg, const ref_full_ext * ext) {
    return ref_full_impl(vctx, pcm, n, cfg, ext);
}

static int ref_full_impl(void * vctx, const float * pcm, int n, const ref_full_cfg * cfg, const ref_full_ext * ext) {
    auto * ctx = (whisper_context *) vctx;
    auto p = whisper_full_default_params(cfg->strategy == 1 ? WHISPER_SAMPLING_BEAM_SEARCH
                                                            : WHISPER_SAMPLING_GREEDY);
    p.n_threads        = cfg->n_threads;
    p.print_progress   = false;
    p.print_realtime   = false;
    p.print_timestamps = false;
    if (cfg->best_of   > 0) p.greedy.best_of        = cfg->best_of;
    if (cfg->beam_size > 0) p.beam_search.beam_size = cfg->beam_size;
    p.temperature      = cfg->temperature;
    p.temperature_inc  = cfg->temperature_inc;
    p.no_timestamps    = cfg->no_timestamps != 0;
    p.max_tokens       = cfg->max_tokens;
    p.token_timestamps = cfg->token_timestamps != 0;
    p.no_context       = cfg->no_context != 0;
    p.single_segment   = cfg->single_segment != 0;
    p.suppress_nst     = cfg->suppress_nst != 0;
    p.length_penalty   = cfg->length_penalty;
    if (cfg->language) p.language = cfg->language;
    p.audio_ctx        = cfg->audio_ctx;
    if (cfg->suppress_eot) p.logits_filter_callback = ref_suppress_eot_cb;
    // every golden run starts from a freshly initialised state's sampler (whisper.cpp:3470):
    // decoders[0].rng otherwise carries the draws of earlier runs on this context
    ctx->state->decoders[0].rng = std::mt19937(0);
    g_rec_prefix.clear(); g_rec_off.clear(); g_rec_idx.clear(); g_rec_val.clear();
    if (cfg->record_topk) {
        g_rec_suppress_eot = cfg->suppress_eot != 0;
        g_rec_trace_only = cfg->record_topk == 2;
        p.logits_filter_callback = ref_record_cb;
    }
    if (!g_vad_path.empty()) {
        p.vad = true;
        p.vad_model_path = g_vad_path.c_str();
    }
    g_cb_log.clear(); g_cb_text.clear();
    g_cb_enc_calls = 0; g_cb_enc_false_at = 0; g_cb_cancel_at = -1; g_cb_cancel = false;
    if (ext) {
        p.initial_prompt       = ext->initial_prompt;
        p.carry_initial_prompt = ext->carry_initial_prompt != 0;
        p.translate            = ext->translate != 0;
        p.max_len              = ext->max_len;
        p.split_on_word        = ext->split_on_word != 0;
        p.tdrz_enable          = ext->tdrz_enable != 0;
        p.offset_ms            = ext->offset_ms;
        p.duration_ms          = ext->duration_ms;
        p.suppress_regex       = ext->suppress_regex;
        p.print_special        = ext->print_special != 0;
        p.detect_language      = ext->detect_language != 0;
        if (ext->n_max_text_ctx > 0) p.n_max_text_ctx = ext->n_max_text_ctx;
        if (ext->max_initial_ts >= 0.0f) p.max_initial_ts = ext->max_initial_ts;
        if (ext->suppress_blank >= 0) p.suppress_blank = ext->suppress_blank != 0;
        if (ext->tdrz_boost) p.logits_filter_callback = ref_tdrz_boost_cb;
        if (ext->callbacks) {
            g_cb_enc_false_at = ext->enc_begin_false_at;
            g_cb_cancel_at = ext->cancel_at_progress;
            p.progress_callback = ref_cb_progress;
            p.encoder_begin_callback = ref_cb_enc_begin;
            p.abort_callback = ref_cb_abort;
            p.new_segment_callback = ref_cb_new_segment;
        }
    }
    g_tf_rec.clear(); g_tf_lp.clear();
    g_tf_window = -1;
    if (g_tf_active) {  // teacher forcing (ref_tf_set): chain the run's own filter callback
        g_tf_base = p.logits_filter_callback;
        p.logits_filter_callback = ref_tf_cb;
        g_tf_params = p;
    }
    if (cfg->n_processors > 1) return whisper_full_parallel(ctx, p, pcm, n, cfg->n_processors);
    return whisper_full(ctx, p, pcm, n);
}

// the alignment-head attention of the last DTW re-decode (state->aheads_cross_QKs_data,
// whisper.cpp:8910-8912): [head][n_audio_ctx][n_tokens] floats; returns the count
long ref_dtw_data(void * vctx, float * out, long cap) {
    const auto & d = ((whisper_context *) vctx)->state->aheads_cross_QKs_data;
    if (out) {
        if (cap < (long) d.size()) return -1;
        std::copy(d.begin(), d.end(), out);
    }
    return (long) d.size();
}

// decoders[j].seek_delta after whisper_full (greedy t = 0: the last window's best decoder)
int ref_decoder_seek_delta(void * vctx, int j) { return ((whisper_context *) vctx)->state->decoders[j].seek_delta; }

// state counters for the CPU-baseline breakdown (whisper.cpp:835-848)
void ref_timings(void * vctx, double * t_mel_ms, double * t_enc_ms, double * t_dec_ms,
                 double * t_batchd_ms, double * t_prompt_ms, double * t_sample_ms, int * n_decode) {
    auto * st = ((whisper_context *) vctx)->state;
    *t_mel_ms = st->t_mel_us / 1e3; *t_enc_ms = st->t_encode_us / 1e3;
    *t_dec_ms = st->t_decode_us / 1e3; *t_batchd_ms = st->t_batchd_us / 1e3;
    *t_prompt_ms = st->t_prompt_us / 1e3; *t_sample_ms = st->t_sample_us / 1e3;
    *n_decode = st->n_decode;
}

// Node-by-node capture of the encoder graph (debug: localises a numerical divergence).
// ref_capture_encoder(ctx, n) records the first n f32 nodes the scheduler evaluates on
// the next whisper_encode; ref_capture_get(i, ...) returns node i's op, shape and data.
struct ref_node { int op; int64_t ne[4]; std::vector<float> data; };
static std::vector<ref_node> g_nodes;
static int g_nodes_max = 0;

static bool ref_eval_cb(struct ggml_tensor * t, bool ask, void *) {
    if (ask) return (int) g_nodes.size() < g_nodes_max;
    if ((int) g_nodes.size() >= g_nodes_max) return true;
    ref_node n;
    n.op = (int) t->op;
    for (int i = 0; i < 4; ++i) n.ne[i] = t->ne[i];
    if (t->type == GGML_TYPE_F32 && ggml_is_contiguous(t)) {
        n.data.resize(ggml_nelements(t));
        memcpy(n.data.data(), t->data, n.data.size() * 4);
    }
    g_nodes.push_back(std::move(n));
    return true;
}

void ref_capture_encoder(void * vctx, int max_nodes) {
    auto * st = ((whisper_context *) vctx)->state;
    g_nodes.clear();
    g_nodes_max = max_nodes;
    ggml_backend_sched_set_eval_callback(st->sched_encode.sched, max_nodes > 0 ? ref_eval_cb : nullptr, nullptr);
}

int ref_capture_count() { return (int) g_nodes.size(); }

long ref_capture_get(int i, int * op, int64_t * ne, float * out, long cap) {
    if (i < 0 || i >= (int) g_nodes.size()) return -1;
    const ref_node & n = g_nodes[i];
    *op = n.op;
    for (int k = 0; k < 4; ++k) ne[k] = n.ne[k];
    if (out && cap >= (long) n.data.size()) memcpy(out, n.data.data(), n.data.size() * 4);
    return (long) n.data.size();
}

// ggml's CPU mul_mat on one weight tensor: w (N rows of K, ggml type wtype, raw blocks)
// times a (M rows of K, f32) -> out [M][N] f32. Pins the quantized-weight GEMM numerics.
int ref_mul_mat(int wtype, const void * w, int N, int K, const float * a, int M, float * out, int n_threads) {
    if (M <= 0 || N <= 0 || K <= 0 || n_threads <= 0) return -1;
    const size_t wbytes = ggml_row_size((ggml_type) wtype, K) * N;
    // the context holds the operands, the result, the graph AND the compute plan's work buffer
    // (ggml_graph_compute_with_ctx allocates it there: src1 converted to the weight's vec_dot
    // type, M rows of K, plus per-thread padding), sized from the operands -- planned on a
    // metadata-only context first
    size_t work = 0;
    {
        ggml_init_params mp = {64 * ggml_tensor_overhead() + ggml_graph_overhead(), nullptr, true};
        ggml_context * mc = ggml_init(mp);
        if (!mc) return -1;
        ggml_tensor * y0 = ggml_mul_mat(mc, ggml_new_tensor_2d(mc, (ggml_type) wtype, K, N),
                                        ggml_new_tensor_2d(mc, GGML_TYPE_F32, K, M));
        ggml_cgraph * g0 = ggml_new_graph(mc);
        ggml_build_forward_expand(g0, y0);
        work = ggml_graph_plan(g0, n_threads, nullptr).work_size;
        ggml_free(mc);
    }
    ggml_init_params ip = {wbytes + (size_t) M * K * 4 + (size_t) M * N * 4 + work + 64 * ggml_tensor_overhead() +
                               ggml_graph_overhead() + (1 << 20), nullptr, false};
    ggml_context * c = ggml_init(ip);
    if (!c) return -1;
    ggml_tensor * tw = ggml_new_tensor_2d(c, (ggml_type) wtype, K, N);
    ggml_tensor * ta = ggml_new_tensor_2d(c, GGML_TYPE_F32, K, M);
    memcpy(tw->data, w, wbytes);
    memcpy(ta->data, a, (size_t) M * K * 4);
    ggml_tensor * y = ggml_mul_mat(c, tw, ta);
    ggml_cgraph * gf = ggml_new_graph(c);
    ggml_build_forward_expand(gf, y);
    const int rc = ggml_graph_compute_with_ctx(c, gf, n_threads) == GGML_STATUS_SUCCESS ? 0 : -2;
    if (rc == 0) memcpy(out, y->data, (size_t) M * N * 4);
    ggml_free(c);
    return rc;
}

// GBNF grammar (ref examples/grammar-parser.cpp, compiled into this probe) -> the reference's own
// grammar engine (whisper_grammar_init / _accept_token / whisper_suppress_invalid_grammar,
// whisper.cpp:5498-5905): parse `gbnf`, start at rule `root`, accept `accept` tokens, then return
// the ids the constraint penalises (penalty 1 on zero logits). Also the parsed rules, flattened:
// rule r's elements at [rule_off[r], rule_off[r + 1]) of (types, values), END included.
int ref_grammar_parse(const char * gbnf, const char * root, int * types, uint32_t * values, int cap, int * rule_off,
                      int cap_rules, int * n_rules, int * i_start) {
    const auto st = grammar_parser::parse(gbnf);
    if (st.rules.empty() || !st.symbol_ids.count(root)) return -1;
    int n = 0;
    *n_rules = (int) st.rules.size();
    *i_start = (int) st.symbol_ids.at(root);
    for (size_t r = 0; r < st.rules.size(); ++r) {
        if ((int) r < cap_rules) rule_off[r] = n;
        for (const auto & e : st.rules[r]) {
            if (n < cap) { types[n] = (int) e.type; values[n] = e.value; }
            ++n;
        }
    }
    if ((int) st.rules.size() < cap_rules) rule_off[st.rules.size()] = n;
    return n;
}

int ref_grammar_rejects(void * vctx, const char * gbnf, const char * root, const int * accept, int n_accept, int * out,
                        int cap) {
    whisper_context * ctx = (whisper_context *) vctx;
    const auto st = grammar_parser::parse(gbnf);
    if (st.rules.empty() || !st.symbol_ids.count(root)) return -1;
    auto rules = st.c_rules();
    whisper_grammar g = whisper_grammar_init(rules.data(), rules.size(), st.symbol_ids.at(root));
    for (int i = 0; i < n_accept; ++i) whisper_grammar_accept_token(*ctx, g, accept[i]);
    whisper_full_params p = whisper_full_default_params(WHISPER_SAMPLING_GREEDY);
    p.grammar_penalty = 1.0f;
    std::vector<float> logits(whisper_n_vocab(ctx), 0.0f);
    whisper_suppress_invalid_grammar(*ctx, p, logits, g);
    int n = 0;
    for (int id = 0; id < (int) logits.size(); ++id)
        if (logits[id] != 0.0f) {
            if (n < cap) out[n] = id;
            ++n;
        }
    return n;
}

} // extern "C"

extern "C" {

// ---------------------------------------------------------------------------------
// The reference's self-attention KV-cell allocator driven by a script (round 5; pins
// csrc/kv_cells.h, tests/test_sanitize_host.py): whisper_kv_cache_find_slot / _seq_rm /
// _seq_cp / _cell_max (whisper.cpp:1019-1137) on a cache of n_ctx cells (no tensors).
// ops: n_ops records of 5 ints (op, a, b, c, d):
//   0 find_slot: a tokens at positions c .. c + a - 1, all of sequence b  -> result head or -1
//   1 seq_rm(a, b, c)   2 seq_cp(a, b, c, d)   3 cell_max -> result   4 clear
// out: n_ops results, then head, then per cell (pos, sequence bitmask of ids 0..31).
int ref_kv_script(int n_ctx, const int * ops, int n_ops, int * out, int cap) {
    if (cap < n_ops + 1 + 2 * n_ctx) return -1;
    whisper_kv_cache cache;
    cache.head = 0;
    cache.size = n_ctx;
    cache.cells.assign(n_ctx, whisper_kv_cell{});
    for (int i = 0; i < n_ops; ++i) {
        const int * o = ops + 5 * i;
        int r = 0;
        if (o[0] == 0) {
            whisper_batch b = whisper_batch_init(o[1], 1);
            b.n_tokens = o[1];
            for (int t = 0; t < o[1]; ++t) {
                b.pos[t] = o[3] + t;
                b.n_seq_id[t] = 1;
                b.seq_id[t][0] = o[2];
            }
            r = whisper_kv_cache_find_slot(cache, b) ? (int) cache.head : -1;
            whisper_batch_free(b);
        } else if (o[0] == 1) {
            whisper_kv_cache_seq_rm(cache, o[1], o[2], o[3]);
        } else if (o[0] == 2) {
            whisper_kv_cache_seq_cp(cache, o[1], o[2], o[3], o[4]);
        } else if (o[0] == 3) {
            r = whisper_kv_cache_cell_max(cache);
        } else if (o[0] == 4) {  // whisper_kv_cache_clear's cell reset (its ggml buffer clear: no tensors here)
            for (int32_t c = 0; c < (int32_t) cache.size; ++c) {
                cache.cells[c].pos = -1;
                cache.cells[c].seq_id.clear();
            }
            cache.head = 0;
        } else {
            return -2;
        }
        out[i] = r;
    }
    out[n_ops] = (int) cache.head;
    for (int c = 0; c < n_ctx; ++c) {
        unsigned m = 0;
        for (int s : cache.cells[c].seq_id) m |= 1u << s;
        out[n_ops + 1 + 2 * c] = cache.cells[c].pos;
        out[n_ops + 2 + 2 * c] = (int) m;
    }
    return n_ops + 1 + 2 * n_ctx;
}

}  // extern "C"
