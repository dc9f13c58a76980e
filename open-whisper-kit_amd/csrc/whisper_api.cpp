// The drop-in C ABI (include/whisper.h) of the MI355X engine.
//
// Lifecycle, getters, staged encode/decode and error conventions follow the reference
// implementation cited per function; the compute behind them is the batch engine.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <regex>
#include <thread>

#include "state.h"
#include "kv_cells.h"
#include "kquant.h"

using namespace owk;

namespace owk {
void set_log_callback(ggml_log_callback cb, void * ud);
const std::vector<uint16_t> & gelu_table_host();
}

// OWK_BACKTRACE=1: print a native backtrace on SIGSEGV/SIGABRT/SIGBUS (host-side debugging on
// the GPU box, where no debugger may attach to a GPU process). Each frame is printed as the file of
// its mapping + the file offset (resolvable offline with llvm-addr2line / llvm-objdump against the
// same image's libraries), then the /proc/self/maps lines around the faulting address. The handler
// only uses async-signal-safe calls (open / read / write / close, hand-written formatting): an abort
// raised inside malloc holds the heap lock, where stdio or dladdr could deadlock. backtrace() is
// called once at install time so its unwinder library is loaded before any signal.
#include <csignal>
#include <execinfo.h>
#include <fcntl.h>
#include <ucontext.h>
#include <unistd.h>
static char g_crash_maps[1 << 18];  // /proc/self/maps, read by the handler
static size_t g_crash_maps_n = 0;
static void crash_put(const char * s) {
    size_t n = 0;
    while (s[n]) ++n;
    (void) !write(2, s, n);
}
static void crash_put_n(const char * s, size_t n) { (void) !write(2, s, n); }
static void crash_put_hex(uintptr_t v) {
    char b[19];
    int i = 18;
    b[i] = 0;
    do {
        b[--i] = "0123456789abcdef"[v & 15];
        v >>= 4;
    } while (v && i > 2);
    b[--i] = 'x';
    b[--i] = '0';
    crash_put(b + i);
}
static uintptr_t crash_parse_hex(const char *& p, const char * end) {
    uintptr_t v = 0;
    for (; p < end; ++p) {
        const char c = *p;
        const int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1;
        if (d < 0) break;
        v = v * 16 + (uintptr_t) d;
    }
    return v;
}
static void crash_read_maps() {
    g_crash_maps_n = 0;
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd < 0) return;
    for (;;) {
        const ssize_t r = read(fd, g_crash_maps + g_crash_maps_n, sizeof(g_crash_maps) - 1 - g_crash_maps_n);
        if (r <= 0) break;
        g_crash_maps_n += (size_t) r;
        if (g_crash_maps_n >= sizeof(g_crash_maps) - 1) break;
    }
    close(fd);
    g_crash_maps[g_crash_maps_n] = '\n';  // a last line printed with its terminator
}
// visits the maps lines: f(line start, line end, lo, hi, file offset, path start)
template <typename F> static void crash_maps_each(F && f) {
    const char * p = g_crash_maps, * end = g_crash_maps + g_crash_maps_n;
    while (p < end) {
        const char * e = p;
        while (e < end && *e != '\n') ++e;
        const char * q = p;
        const uintptr_t lo = crash_parse_hex(q, e);
        ++q;
        const uintptr_t hi = crash_parse_hex(q, e);
        while (q < e && *q != ' ') ++q;  // " perms offset"
        ++q;
        while (q < e && *q != ' ') ++q;
        ++q;
        const uintptr_t off = crash_parse_hex(q, e);
        const char * path = e;
        for (const char * c = q; c < e; ++c)
            if (*c == '/' || *c == '[') {
                path = c;
                break;
            }
        if (!f(p, e, lo, hi, off, path)) return;
        p = e + 1;
    }
}
static void owk_crash_print_pc(const void * pc) {
    const uintptr_t a = (uintptr_t) pc;
    bool found = false;
    crash_put("  ");
    crash_put_hex(a);
    crash_maps_each([&](const char *, const char * e, uintptr_t lo, uintptr_t hi, uintptr_t off, const char * path) {
        if (a < lo || a >= hi) return true;
        crash_put("  ");
        crash_put_n(path, (size_t) (e - path));
        crash_put("+");
        crash_put_hex(a - lo + off);
        found = true;
        return false;
    });
    crash_put(found ? "\n" : "  (no mapping)\n");
}
static void owk_crash_handler(int sig, siginfo_t * si, void * uc_) {
    const ucontext_t * uc = (const ucontext_t *) uc_;
    const void * pc = uc ? (const void *) uc->uc_mcontext.gregs[REG_RIP] : nullptr;
    crash_read_maps();
    crash_put("\n[owk] fatal signal ");
    crash_put_hex((uintptr_t) sig);
    crash_put(", fault address ");
    crash_put_hex(si ? (uintptr_t) si->si_addr : 0);
    crash_put(", pc:\n");
    owk_crash_print_pc(pc);
    void * frames[64];
    const int nf = backtrace(frames, 64);
    crash_put("[owk] native backtrace (mapped file + file offset):\n");
    for (int i = 0; i < nf; ++i) owk_crash_print_pc(frames[i]);
    if (si && sig != SIGABRT) {  // the mappings around the fault address: which allocation the access ran off
        const uintptr_t a = (uintptr_t) si->si_addr;
        crash_put("[owk] /proc/self/maps around the fault address:\n");
        const char * prev = nullptr, * prev_e = nullptr;
        crash_maps_each([&](const char * p, const char * e, uintptr_t lo, uintptr_t hi, uintptr_t, const char *) {
            if (hi + (64ul << 20) >= a && lo <= a + (64ul << 20)) {
                if (prev) crash_put_n(prev, (size_t) (prev_e - prev) + 1);
                prev = nullptr;
                crash_put_n(p, (size_t) (e - p) + 1);
                return true;
            }
            if (lo > a) return false;
            prev = p, prev_e = e;
            return true;
        });
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
static int owk_install_crash_handler = [] {
    const char * e = getenv("OWK_BACKTRACE");
    if (e && e[0] == '1') {
        void * warm[2];
        (void) backtrace(warm, 2);  // loads the unwinder now, not inside the handler
        struct sigaction sa{};
        sa.sa_sigaction = owk_crash_handler;
        sa.sa_flags = SA_SIGINFO;
        sigaction(SIGSEGV, &sa, nullptr);
        sigaction(SIGABRT, &sa, nullptr);
        sigaction(SIGBUS, &sa, nullptr);
    }
    return 0;
}();

namespace owk {

// alignment-head presets of the reference (whisper.cpp:384-410): {text layer, head}
static const std::map<int, std::vector<std::pair<int, int>>> & aheads_presets() {
    static const std::map<int, std::vector<std::pair<int, int>>> m = {
        {WHISPER_AHEADS_TINY_EN, {{1, 0}, {2, 0}, {2, 5}, {3, 0}, {3, 1}, {3, 2}, {3, 3}, {3, 4}}},
        {WHISPER_AHEADS_TINY, {{2, 2}, {3, 0}, {3, 2}, {3, 3}, {3, 4}, {3, 5}}},
        {WHISPER_AHEADS_BASE_EN, {{3, 3}, {4, 7}, {5, 1}, {5, 5}, {5, 7}}},
        {WHISPER_AHEADS_BASE, {{3, 1}, {4, 2}, {4, 3}, {4, 7}, {5, 1}, {5, 2}, {5, 4}, {5, 6}}},
        {WHISPER_AHEADS_SMALL_EN, {{6, 6}, {7, 0}, {7, 3}, {7, 8}, {8, 2}, {8, 5}, {8, 7}, {9, 0}, {9, 4}, {9, 8},
                                   {9, 10}, {10, 0}, {10, 1}, {10, 2}, {10, 3}, {10, 6}, {10, 11}, {11, 2}, {11, 4}}},
        {WHISPER_AHEADS_SMALL, {{5, 3}, {5, 9}, {8, 0}, {8, 4}, {8, 7}, {8, 8}, {9, 0}, {9, 7}, {9, 9}, {10, 5}}},
        {WHISPER_AHEADS_MEDIUM_EN, {{11, 4}, {14, 1}, {14, 12}, {14, 14}, {15, 4}, {16, 0}, {16, 4}, {16, 9}, {17, 12},
                                    {17, 14}, {18, 7}, {18, 10}, {18, 15}, {20, 0}, {20, 3}, {20, 9}, {20, 14}, {21, 12}}},
        {WHISPER_AHEADS_MEDIUM, {{13, 15}, {15, 4}, {15, 15}, {16, 1}, {20, 0}, {23, 4}}},
        {WHISPER_AHEADS_LARGE_V1, {{9, 19}, {11, 2}, {11, 4}, {11, 17}, {22, 7}, {22, 11}, {22, 17}, {23, 2}, {23, 15}}},
        {WHISPER_AHEADS_LARGE_V2, {{10, 12}, {13, 17}, {16, 11}, {16, 12}, {16, 13}, {17, 15}, {17, 16}, {18, 4}, {18, 11},
                                   {18, 19}, {19, 11}, {21, 2}, {21, 3}, {22, 3}, {22, 9}, {22, 12}, {23, 5}, {23, 7},
                                   {23, 13}, {25, 5}, {26, 1}, {26, 12}, {27, 15}}},
        {WHISPER_AHEADS_LARGE_V3, {{7, 0}, {10, 17}, {12, 18}, {13, 12}, {16, 1}, {17, 14}, {19, 11}, {21, 4}, {24, 1}, {25, 6}}},
        {WHISPER_AHEADS_LARGE_V3_TURBO, {{2, 4}, {2, 11}, {3, 3}, {3, 6}, {3, 11}, {3, 14}}},
    };
    return m;
}

bool alignment_heads(const whisper_context * ctx, std::vector<int> & amap, int & n_ah) {
    const whisper_context_params & cp = ctx->params;
    const int L = ctx->model->hp.n_text_layer, H = ctx->model->hp.n_text_head;
    std::vector<std::pair<int, int>> heads;
    if (cp.dtw_aheads_preset == WHISPER_AHEADS_NONE) {
        log_msg(GGML_LOG_LEVEL_ERROR, "aheads_masks_init: dtw_aheads_preset should be != DTW_AHEADS_NONE\n");
        return false;
    } else if (cp.dtw_aheads_preset == WHISPER_AHEADS_N_TOP_MOST) {
        if (cp.dtw_n_top > L || cp.dtw_n_top <= 0) {
            log_msg(GGML_LOG_LEVEL_ERROR, "aheads_masks_init: dtw_n_top must be between %d and %d for this model.", 1, L);
            return false;
        }
        for (int l = L - cp.dtw_n_top; l < L; ++l)
            for (int h = 0; h < H; ++h) heads.emplace_back(l, h);
    } else {
        if (cp.dtw_aheads_preset == WHISPER_AHEADS_CUSTOM) {
            if (cp.dtw_aheads.n_heads == 0 || cp.dtw_aheads.heads == nullptr) {
                log_msg(GGML_LOG_LEVEL_ERROR, "aheads_masks_init: dtw_aheads unset\n");
                return false;
            }
            for (size_t i = 0; i < cp.dtw_aheads.n_heads; ++i)
                heads.emplace_back(cp.dtw_aheads.heads[i].n_text_layer, cp.dtw_aheads.heads[i].n_head);
        } else {
            auto it = aheads_presets().find(cp.dtw_aheads_preset);
            if (it == aheads_presets().end()) return false;
            heads = it->second;
        }
        for (const auto & hh : heads)
            if (hh.first < 0 || hh.first >= L || hh.second < 0 || hh.second >= H) {
                log_msg(GGML_LOG_LEVEL_ERROR, "aheads_masks_init: alignment head (%d, %d) outside the model\n",
                        hh.first + 1, hh.second + 1);
                return false;
            }
    }
    // global index: layer-major, and within a layer the preset order (the mask rows)
    amap.assign((size_t) L * H, -1);
    n_ah = 0;
    for (int l = 0; l < L; ++l)
        for (const auto & hh : heads)
            if (hh.first == l) amap[(size_t) l * H + hh.second] = n_ah++;
    return n_ah > 0;
}

void configure_engine(const whisper_context * ctx, whisper_state * st) {
    if (!st->eng) return;
    st->eng->flash_attn = ctx->params.flash_attn;
    if (ctx->params.dtw_token_timestamps && st->dtw_n_ah > 0 && st->eng->n_aheads() == 0)
        st->eng->set_alignment_heads(st->dtw_amap, st->dtw_n_ah);
}

}  // namespace owk

static whisper_state * new_state(whisper_context * ctx) {
    auto * st = new whisper_state();
    st->flash_attn = ctx->params.flash_attn;
    if (ctx->params.dtw_token_timestamps && !alignment_heads(ctx, st->dtw_amap, st->dtw_n_ah)) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_init_state: aheads_masks_init() failed for alignment heads masks\n");
        delete st;
        return nullptr;
    }
    try {
        st->eng.reset(new Engine(ctx->model.get(), &ctx->prof));
        configure_engine(ctx, st);
    } catch (const std::exception & e) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_init_state: %s\n", e.what());
        delete st;
        return nullptr;
    }
    const int cells = (ctx->model->hp.n_text_ctx + 255) / 256 * 256;  // GGML_PAD(n_text_ctx, 256), ref 3387-3390
    st->kv.init(cells);
    st->kv_self_n_dec = 1;
    st->decoders[0].rng = std::mt19937(0);  // ref 3470
    return st;
}

extern "C" {

void ggml_backend_load_all(void) {}

const char * whisper_version(void) { return "1.8.3-mi355x"; }

// ---------------------------------------------------------------------------------
// defaults (ref whisper.cpp:3606-3622, 5928-6034)
// ---------------------------------------------------------------------------------
struct whisper_context_params whisper_context_default_params(void) {
    whisper_context_params r{};
    r.use_gpu = true;
    r.flash_attn = true;
    r.gpu_device = 0;
    r.dtw_token_timestamps = false;
    r.dtw_aheads_preset = WHISPER_AHEADS_NONE;
    r.dtw_n_top = -1;
    r.dtw_aheads = {0, nullptr};
    r.dtw_mem_size = 1024 * 1024 * 128;
    return r;
}

struct whisper_context_params * whisper_context_default_params_by_ref(void) {
    return new whisper_context_params(whisper_context_default_params());
}


struct whisper_full_params whisper_full_default_params(enum whisper_sampling_strategy strategy) {
    whisper_full_params r{};
    r.strategy = strategy;
    r.n_threads = std::min(4, (int32_t) std::thread::hardware_concurrency());
    r.n_max_text_ctx = 16384;
    r.offset_ms = 0;
    r.duration_ms = 0;
    r.translate = false;
    r.no_context = true;
    r.no_timestamps = false;
    r.single_segment = false;
    r.print_special = false;
    r.print_progress = true;
    r.print_realtime = false;
    r.print_timestamps = true;
    r.token_timestamps = false;
    r.thold_pt = 0.01f;
    r.thold_ptsum = 0.01f;
    r.max_len = 0;
    r.split_on_word = false;
    r.max_tokens = 0;
    r.debug_mode = false;
    r.audio_ctx = 0;
    r.tdrz_enable = false;
    r.suppress_regex = nullptr;
    r.initial_prompt = nullptr;
    r.carry_initial_prompt = false;
    r.prompt_tokens = nullptr;
    r.prompt_n_tokens = 0;
    r.language = "en";
    r.detect_language = false;
    r.suppress_blank = true;
    r.suppress_nst = false;
    r.temperature = 0.0f;
    r.max_initial_ts = 1.0f;
    r.length_penalty = -1.0f;
    r.temperature_inc = 0.2f;
    r.entropy_thold = 2.4f;
    r.logprob_thold = -1.0f;
    r.no_speech_thold = 0.6f;
    r.greedy.best_of = -1;
    r.beam_search.beam_size = -1;
    r.beam_search.patience = -1.0f;
    r.grammar_rules = nullptr;
    r.n_grammar_rules = 0;
    r.i_start_rule = 0;
    r.grammar_penalty = 100.0f;
    r.vad = false;
    r.vad_model_path = nullptr;
    r.vad_params = whisper_vad_default_params();
    if (strategy == WHISPER_SAMPLING_GREEDY) r.greedy.best_of = 5;
    else r.beam_search.beam_size = 5;
    return r;
}

struct whisper_full_params * whisper_full_default_params_by_ref(enum whisper_sampling_strategy strategy) {
    return new whisper_full_params(whisper_full_default_params(strategy));
}

void whisper_free_params(struct whisper_full_params * params) { delete params; }
void whisper_free_context_params(struct whisper_context_params * params) { delete params; }

// ---------------------------------------------------------------------------------
// init / free (ref 3624-3861)
// ---------------------------------------------------------------------------------
struct whisper_context * whisper_init_with_params_no_state(struct whisper_model_loader * loader,
                                                           struct whisper_context_params params) {
    const int64_t t0 = time_us();
    if (params.flash_attn && params.dtw_token_timestamps) {
        log_msg(GGML_LOG_LEVEL_WARN, "%s: dtw_token_timestamps is not supported with flash_attn - disabling\n", __func__);
        params.dtw_token_timestamps = false;
    }
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev <= 0) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: no MI355X (gfx950) device available\n", __func__);
        loader->close(loader->context);
        return nullptr;
    }
    const int dev = std::max(0, std::min(params.gpu_device, n_dev - 1));
    std::string err;
    Model * m = nullptr;
    try {
        m = load_model(loader, dev, err);
    } catch (const std::exception & e) {
        err = e.what();
    }
    loader->close(loader->context);
    if (!m) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_model_load: %s\n", err.c_str());
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: failed to load model\n", __func__);
        return nullptr;
    }
    auto * ctx = new whisper_context();
    ctx->params = params;
    ctx->model.reset(m);
    ctx->t_start_us = t0;
    ctx->t_load_us = time_us() - t0;
    return ctx;
}

struct whisper_context * whisper_init_from_file_with_params_no_state(const char * path_model,
                                                                     struct whisper_context_params params) {
    auto * fin = new std::ifstream(path_model, std::ios::binary);
    if (!*fin) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: failed to open '%s'\n", __func__, path_model);
        delete fin;
        return nullptr;
    }
    whisper_model_loader loader = {};
    loader.context = fin;
    loader.read = [](void * c, void * out, size_t n) {
        auto * f = (std::ifstream *) c;
        f->read((char *) out, n);
        return (size_t) f->gcount();
    };
    loader.eof = [](void * c) { return ((std::ifstream *) c)->eof(); };
    loader.close = [](void * c) {
        auto * f = (std::ifstream *) c;
        f->close();
        delete f;
    };
    auto * ctx = whisper_init_with_params_no_state(&loader, params);
    if (ctx) ctx->path_model = path_model;
    return ctx;
}

struct whisper_context * whisper_init_from_buffer_with_params_no_state(void * buffer, size_t buffer_size,
                                                                       struct whisper_context_params params) {
    struct Buf {
        uint8_t * p;
        size_t size, off;
    } buf = {(uint8_t *) buffer, buffer_size, 0};
    whisper_model_loader loader = {};
    loader.context = &buf;
    loader.read = [](void * c, void * out, size_t n) {
        Buf * b = (Buf *) c;
        const size_t k = b->off + n < b->size ? n : b->size - b->off;
        memcpy(out, b->p + b->off, k);
        b->off += k;
        return k;
    };
    loader.eof = [](void * c) { Buf * b = (Buf *) c; return b->off >= b->size; };
    loader.close = [](void *) {};
    return whisper_init_with_params_no_state(&loader, params);
}

static whisper_context * with_state(whisper_context * ctx) {
    if (!ctx) return nullptr;
    ctx->state = whisper_init_state(ctx);
    if (!ctx->state) {
        whisper_free(ctx);
        return nullptr;
    }
    return ctx;
}

struct whisper_context * whisper_init_from_file_with_params(const char * path_model, struct whisper_context_params params) {
    return with_state(whisper_init_from_file_with_params_no_state(path_model, params));
}
struct whisper_context * whisper_init_from_buffer_with_params(void * buffer, size_t buffer_size,
                                                              struct whisper_context_params params) {
    return with_state(whisper_init_from_buffer_with_params_no_state(buffer, buffer_size, params));
}
struct whisper_context * whisper_init_with_params(struct whisper_model_loader * loader, struct whisper_context_params params) {
    return with_state(whisper_init_with_params_no_state(loader, params));
}
struct whisper_context * whisper_init_from_file(const char * path_model) {
    return whisper_init_from_file_with_params(path_model, whisper_context_default_params());
}
struct whisper_context * whisper_init_from_buffer(void * buffer, size_t buffer_size) {
    return whisper_init_from_buffer_with_params(buffer, buffer_size, whisper_context_default_params());
}
struct whisper_context * whisper_init(struct whisper_model_loader * loader) {
    return whisper_init_with_params(loader, whisper_context_default_params());
}
struct whisper_context * whisper_init_from_file_no_state(const char * path_model) {
    return whisper_init_from_file_with_params_no_state(path_model, whisper_context_default_params());
}
struct whisper_context * whisper_init_from_buffer_no_state(void * buffer, size_t buffer_size) {
    return whisper_init_from_buffer_with_params_no_state(buffer, buffer_size, whisper_context_default_params());
}
struct whisper_context * whisper_init_no_state(struct whisper_model_loader * loader) {
    return whisper_init_with_params_no_state(loader, whisper_context_default_params());
}

struct whisper_state * whisper_init_state(struct whisper_context * ctx) {
    if (!ctx) return nullptr;
    return new_state(ctx);
}

int whisper_ctx_init_openvino_encoder_with_state(struct whisper_context *, struct whisper_state *, const char *,
                                                 const char *, const char *) {
    return 1;
}
int whisper_ctx_init_openvino_encoder(struct whisper_context *, const char *, const char *, const char *) { return 1; }

void whisper_free_state(struct whisper_state * state) {
    if (state && state->vad_context) whisper_vad_free(state->vad_context);  // ref 3838-3841
    delete state;
}

void whisper_free(struct whisper_context * ctx) {
    if (!ctx) return;
    whisper_free_state(ctx->state);
    ctx->state = nullptr;
    delete ctx;
}

// ---------------------------------------------------------------------------------
// staged API (ref 3875-3955)
// ---------------------------------------------------------------------------------
static Engine & eng_of(whisper_context * ctx, whisper_state * st) {
    if (!st->eng) st->eng.reset(new Engine(ctx->model.get(), &ctx->prof));
    configure_engine(ctx, st);
    const int cells = std::max<int>((int) st->kv.size, (ctx->model->hp.n_text_ctx + 255) / 256 * 256);
    st->eng->reserve(1, std::max(cells, st->eng->kv_cells));
    return *st->eng;
}

int whisper_pcm_to_mel_with_state(struct whisper_context * ctx, struct whisper_state * st, const float * samples,
                                  int n_samples, int) {
    try {
        OWK_HIP_CHECK(hipSetDevice(ctx->model->device));
        Engine & e = eng_of(ctx, st);
        const int64_t t0 = time_us();
        e.compute_mel({0}, {samples}, {n_samples});
        st->t_mel_us += time_us() - t0;
        st->mel_n_len = e.mel_len(0);
        st->mel_n_len_org = 1 + (n_samples + 200 - 400) / 160;
        st->mel_n_mel = ctx->model->n_filters_mel;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: failed to compute mel spectrogram: %s\n", __func__, ex.what());
        return -1;
    }
    return 0;
}

int whisper_pcm_to_mel(struct whisper_context * ctx, const float * samples, int n_samples, int n_threads) {
    return whisper_pcm_to_mel_with_state(ctx, ctx->state, samples, n_samples, n_threads);
}

int whisper_set_mel_with_state(struct whisper_context * ctx, struct whisper_state * st, const float * data, int n_len,
                               int n_mel) {
    if (n_mel != ctx->model->n_filters_mel) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: invalid number of mel bands: %d (expected %d)\n", __func__, n_mel,
                ctx->model->n_filters_mel);
        return -1;
    }
    try {
        OWK_HIP_CHECK(hipSetDevice(ctx->model->device));
        eng_of(ctx, st).set_mel(0, data, n_len, n_mel);
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: %s\n", __func__, ex.what());
        return -1;
    }
    st->mel_n_len = n_len;
    st->mel_n_len_org = n_len;
    st->mel_n_mel = n_mel;
    return 0;
}

int whisper_set_mel(struct whisper_context * ctx, const float * data, int n_len, int n_mel) {
    return whisper_set_mel_with_state(ctx, ctx->state, data, n_len, n_mel);
}

int whisper_encode_with_state(struct whisper_context * ctx, struct whisper_state * st, int offset, int) {
    try {
        OWK_HIP_CHECK(hipSetDevice(ctx->model->device));
        Engine & e = eng_of(ctx, st);
        e.audio_ctx = st->exp_n_audio_ctx;
        const int64_t t0 = time_us();
        e.encode({0}, {offset});
        e.sync();
        st->t_encode_us += time_us() - t0;
        st->n_encode++;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: failed to eval: %s\n", __func__, ex.what());
        return -1;
    }
    return 0;
}

int whisper_encode(struct whisper_context * ctx, int offset, int n_threads) {
    return whisper_encode_with_state(ctx, ctx->state, offset, n_threads);
}

int whisper_decode_with_state(struct whisper_context * ctx, struct whisper_state * st, const whisper_token * tokens,
                              int n_tokens, int n_past, int) {
    if (n_tokens <= 0) return 1;
    try {
        OWK_HIP_CHECK(hipSetDevice(ctx->model->device));
        Engine & e = eng_of(ctx, st);
        e.audio_ctx = st->exp_n_audio_ctx;
        // whisper_batch_prep_legacy + seq_rm (ref 511-523, 3935-3946)
        std::vector<CallToken> toks(n_tokens);
        for (int i = 0; i < n_tokens; ++i) toks[i] = CallToken{tokens[i], n_past + i, 0, i == n_tokens - 1};
        st->kv.seq_rm(0, n_past, -1);
        std::vector<DecodeRow> rows;
        std::vector<int> keys;
        int n_logit = 0;
        if (prepare_decode_call(st, 0, toks, rows, keys, n_logit) < 0) {
            log_msg(GGML_LOG_LEVEL_ERROR, "%s: failed to eval\n", __func__);
            return 1;
        }
        const int64_t t0 = time_us();
        e.decode(rows, keys, n_logit);
        const int nv = ctx->model->hp.n_vocab;
        st->logits.resize((size_t) n_tokens * nv);
        e.download_logits(0, st->logits.data() + (size_t) (n_tokens - 1) * nv);
        // keep the no-speech emulation consistent for a following whisper_full on this state
        StepPost post;
        const int old = st->logits_rows;
        for (int r = 0; r < n_tokens && r < Engine::RMX; ++r) {
            const bool zero = r >= old;
            const int lrow = r == n_tokens - 1 ? 0 : -1;
            if (lrow >= 0 || zero) post.rowmax.push_back(make_int4(0, r, lrow, zero ? 1 : 0));
        }
        if (n_tokens == 1) post.row0.push_back(make_int2(0, 0));
        else if (old == 0) post.row0.push_back(make_int2(-1, 0));
        std::vector<TokenOut> outs;
        std::vector<float> ns;
        VocabInfo vi{};
        e.step_post(post, {}, vi, outs, ns, nullptr, nullptr);
        st->logits_rows = n_tokens;
        e.save_logits_state(0, n_tokens, st->logits_rowmax, st->logits_row0);
        const int64_t dt = time_us() - t0;
        if (n_tokens == 1) { st->t_decode_us += dt; st->n_decode++; }
        else if (n_tokens < 16) { st->t_batchd_us += dt; st->n_batchd += n_tokens; }
        else { st->t_prompt_us += dt; st->n_prompt += n_tokens; }
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: failed to eval: %s\n", __func__, ex.what());
        return 1;
    }
    return 0;
}

int whisper_decode(struct whisper_context * ctx, const whisper_token * tokens, int n_tokens, int n_past, int n_threads) {
    if (ctx->state == nullptr) {
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: ERROR state was not loaded.\n", __func__);
        return -1;
    }
    return whisper_decode_with_state(ctx, ctx->state, tokens, n_tokens, n_past, n_threads);
}

// ---------------------------------------------------------------------------------
// tokenizer (tokenize_text: greedy longest match over regex-split words, ref 3272-3320)
// ---------------------------------------------------------------------------------
int whisper_tokenize(struct whisper_context * ctx, const char * text, whisper_token * tokens, int n_max_tokens) {
    const std::vector<int> res = tokenize_text(ctx->model->vocab, text);
    if (n_max_tokens < (int) res.size()) {
        if (n_max_tokens > 0)
            log_msg(GGML_LOG_LEVEL_ERROR, "%s: too many resulting tokens: %d (max %d)\n", __func__, (int) res.size(),
                    n_max_tokens);
        return -(int) res.size();
    }
    for (size_t i = 0; i < res.size(); ++i) tokens[i] = res[i];
    return (int) res.size();
}

int whisper_token_count(struct whisper_context * ctx, const char * text) { return -whisper_tokenize(ctx, text, NULL, 0); }

// ---------------------------------------------------------------------------------
// languages (ref 3976-4102)
// ---------------------------------------------------------------------------------
int whisper_lang_max_id(void) {
    int mx = 0;
    for (const auto & kv : languages()) mx = std::max(mx, kv.second.first);
    return mx;
}

int whisper_lang_id(const char * lang) {
    const auto & L = languages();
    if (!L.count(lang)) {
        for (const auto & kv : L)
            if (kv.second.second == lang) return kv.second.first;
        log_msg(GGML_LOG_LEVEL_ERROR, "%s: unknown language '%s'\n", __func__, lang);
        return -1;
    }
    return L.at(lang).first;
}

const char * whisper_lang_str(int id) {
    for (const auto & kv : languages())
        if (kv.second.first == id) return kv.first.c_str();
    log_msg(GGML_LOG_LEVEL_ERROR, "%s: unknown language id %d\n", __func__, id);
    return nullptr;
}

const char * whisper_lang_str_full(int id) {
    for (const auto & kv : languages())
        if (kv.second.first == id) return kv.second.second.c_str();
    log_msg(GGML_LOG_LEVEL_ERROR, "%s: unknown language id %d\n", __func__, id);
    return nullptr;
}

int whisper_lang_auto_detect_with_state(struct whisper_context * ctx, struct whisper_state * st, int offset_ms,
                                        int n_threads, float * lang_probs) {
    const int seek = offset_ms / 10;
    if (seek < 0) return -1;
    if (seek >= st->mel_n_len_org) return -2;
    if (whisper_encode_with_state(ctx, st, seek, n_threads) != 0) return -6;
    const whisper_token sot = ctx->model->vocab.sot;
    if (whisper_decode_with_state(ctx, st, &sot, 1, 0, n_threads) != 0) return -7;
    std::vector<std::pair<float, int>> lid;
    for (const auto & kv : languages()) lid.emplace_back(st->logits[sot + 1 + kv.second.first], kv.second.first);
    std::sort(lid.begin(), lid.end(), [](const std::pair<float, int> & a, const std::pair<float, int> & b) {
        return a.first > b.first;
    });
    const float mx = lid[0].first;
    double sum = 0.0;
    for (auto & kv : lid) { kv.first = exp(kv.first - mx); sum += kv.first; }
    for (auto & kv : lid) kv.first /= sum;
    if (lang_probs)
        for (const auto & kv : lid) lang_probs[kv.second] = kv.first;
    return lid[0].second;
}

int whisper_lang_auto_detect(struct whisper_context * ctx, int offset_ms, int n_threads, float * lang_probs) {
    return whisper_lang_auto_detect_with_state(ctx, ctx->state, offset_ms, n_threads, lang_probs);
}

// ---------------------------------------------------------------------------------
// model / vocab queries (ref 4104-4243)
// ---------------------------------------------------------------------------------
int whisper_model_n_vocab(struct whisper_context * ctx) { return ctx->model->hp.n_vocab; }
int whisper_model_n_audio_ctx(struct whisper_context * ctx) { return ctx->model->hp.n_audio_ctx; }
int whisper_model_n_audio_state(struct whisper_context * ctx) { return ctx->model->hp.n_audio_state; }
int whisper_model_n_audio_head(struct whisper_context * ctx) { return ctx->model->hp.n_audio_head; }
int whisper_model_n_audio_layer(struct whisper_context * ctx) { return ctx->model->hp.n_audio_layer; }
int whisper_model_n_text_ctx(struct whisper_context * ctx) { return ctx->model->hp.n_text_ctx; }
int whisper_model_n_text_state(struct whisper_context * ctx) { return ctx->model->hp.n_text_state; }
int whisper_model_n_text_head(struct whisper_context * ctx) { return ctx->model->hp.n_text_head; }
int whisper_model_n_text_layer(struct whisper_context * ctx) { return ctx->model->hp.n_text_layer; }
int whisper_model_n_mels(struct whisper_context * ctx) { return ctx->model->hp.n_mels; }
int whisper_model_ftype(struct whisper_context * ctx) { return ctx->model->hp.ftype; }
int whisper_model_type(struct whisper_context * ctx) { return (int) ctx->model->type; }

const char * whisper_model_type_readable(struct whisper_context * ctx) {
    switch (ctx->model->type) {
        case MODEL_TINY: return "tiny";
        case MODEL_BASE: return "base";
        case MODEL_SMALL: return "small";
        case MODEL_MEDIUM: return "medium";
        case MODEL_LARGE: return "large";
        default: return "unknown";
    }
}

int whisper_n_len_from_state(struct whisper_state * state) { return state->mel_n_len_org; }
int whisper_n_len(struct whisper_context * ctx) { return ctx->state->mel_n_len_org; }
int whisper_n_vocab(struct whisper_context * ctx) { return ctx->model->vocab.n_vocab; }
int whisper_n_text_ctx(struct whisper_context * ctx) { return ctx->model->hp.n_text_ctx; }
int whisper_n_audio_ctx(struct whisper_context * ctx) { return ctx->model->hp.n_audio_ctx; }
int whisper_is_multilingual(struct whisper_context * ctx) { return ctx->model->vocab.is_multilingual() ? 1 : 0; }
float * whisper_get_logits(struct whisper_context * ctx) { return ctx->state->logits.data(); }
float * whisper_get_logits_from_state(struct whisper_state * state) { return state->logits.data(); }
const char * whisper_token_to_str(struct whisper_context * ctx, whisper_token token) {
    return ctx->model->vocab.id_to_token.at(token).c_str();
}
whisper_token whisper_token_eot(struct whisper_context * ctx) { return ctx->model->vocab.eot; }
whisper_token whisper_token_sot(struct whisper_context * ctx) { return ctx->model->vocab.sot; }
whisper_token whisper_token_solm(struct whisper_context * ctx) { return ctx->model->vocab.solm; }
whisper_token whisper_token_prev(struct whisper_context * ctx) { return ctx->model->vocab.prev; }
whisper_token whisper_token_nosp(struct whisper_context * ctx) { return ctx->model->vocab.nosp; }
whisper_token whisper_token_not(struct whisper_context * ctx) { return ctx->model->vocab.not_; }
whisper_token whisper_token_beg(struct whisper_context * ctx) { return ctx->model->vocab.beg; }
whisper_token whisper_token_lang(struct whisper_context * ctx, int lang_id) { return ctx->model->vocab.sot + 1 + lang_id; }
whisper_token whisper_token_translate(struct whisper_context * ctx) { return ctx->model->vocab.translate; }
whisper_token whisper_token_transcribe(struct whisper_context * ctx) { return ctx->model->vocab.transcribe; }

// ---------------------------------------------------------------------------------
// timings (ref 4245-4297)
// ---------------------------------------------------------------------------------
struct whisper_timings * whisper_get_timings(struct whisper_context * ctx) {
    if (!ctx->state) return nullptr;
    const whisper_state * s = ctx->state;
    // the reference returns a heap object the caller never frees; a context-owned one here
    whisper_timings & t = ctx->timings;
    t.sample_ms = 1e-3f * s->t_sample_us / std::max(1, s->n_sample);
    t.encode_ms = 1e-3f * s->t_encode_us / std::max(1, s->n_encode);
    t.decode_ms = 1e-3f * s->t_decode_us / std::max(1, s->n_decode);
    t.batchd_ms = 1e-3f * s->t_batchd_us / std::max(1, s->n_batchd);
    t.prompt_ms = 1e-3f * s->t_prompt_us / std::max(1, s->n_prompt);
    return &t;
}

void whisper_print_timings(struct whisper_context * ctx) {
    const int64_t t_end = time_us();
    log_msg(GGML_LOG_LEVEL_INFO, "\nwhisper_print_timings:     load time = %8.2f ms\n", ctx->t_load_us / 1000.0f);
    if (ctx->state) {
        const whisper_state * s = ctx->state;
        const int ns = std::max(1, s->n_sample), ne = std::max(1, s->n_encode), nd = std::max(1, s->n_decode),
                  nb = std::max(1, s->n_batchd), np = std::max(1, s->n_prompt);
        log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:     fallbacks = %3d p / %3d h\n", s->n_fail_p, s->n_fail_h);
        log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:      mel time = %8.2f ms\n", s->t_mel_us / 1000.0f);
        log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:   sample time = %8.2f ms / %5d runs ( %8.2f ms per run)\n",
                1e-3f * s->t_sample_us, ns, 1e-3f * s->t_sample_us / ns);
        log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:   encode time = %8.2f ms / %5d runs ( %8.2f ms per run)\n",
                1e-3f * s->t_encode_us, ne, 1e-3f * s->t_encode_us / ne);
        log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:   decode time = %8.2f ms / %5d runs ( %8.2f ms per run)\n",
                1e-3f * s->t_decode_us, nd, 1e-3f * s->t_decode_us / nd);
        log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:   batchd time = %8.2f ms / %5d runs ( %8.2f ms per run)\n",
                1e-3f * s->t_batchd_us, nb, 1e-3f * s->t_batchd_us / nb);
        log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:   prompt time = %8.2f ms / %5d runs ( %8.2f ms per run)\n",
                1e-3f * s->t_prompt_us, np, 1e-3f * s->t_prompt_us / np);
    }
    log_msg(GGML_LOG_LEVEL_INFO, "whisper_print_timings:    total time = %8.2f ms\n", (t_end - ctx->t_start_us) / 1000.0f);
}

void whisper_reset_timings(struct whisper_context * ctx) {
    ctx->t_start_us = time_us();
    if (whisper_state * s = ctx->state) {
        s->t_mel_us = s->t_sample_us = s->t_encode_us = s->t_decode_us = s->t_batchd_us = s->t_prompt_us = 0;
        s->n_sample = s->n_encode = s->n_decode = s->n_batchd = s->n_prompt = 0;
    }
}

const char * whisper_print_system_info(void) {
    static std::string s;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    s = "MI355X/HIP : devices = " + std::to_string(n) + " | gfx950 MFMA f16 | ";
    return s.c_str();
}

// ---------------------------------------------------------------------------------
// whisper_full (ref 6827-7929)
// ---------------------------------------------------------------------------------
int whisper_full_with_state(struct whisper_context * ctx, struct whisper_state * state, struct whisper_full_params params,
                            const float * samples, int n_samples) {
    try {
        if (!state) throw std::runtime_error("null state");
        // this state only (other states of the context may run concurrently); the context lock
        // while the shared per-kernel recorder is on
        std::unique_lock<std::mutex> ctx_lock(ctx->mu, std::defer_lock);
        if (ctx->prof.on) ctx_lock.lock();
        std::lock_guard<std::mutex> lk(state->mu);
        return full_batch(ctx, &state, &params, nullptr, &samples, &n_samples, 1);
    } catch (const std::exception & e) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full_with_state: %s\n", e.what());
        return -6;
    }
}

// ref 7778-7799: the VAD pre-pass belongs to whisper_full (not whisper_full_with_state)
int whisper_full(struct whisper_context * ctx, struct whisper_full_params params, const float * samples, int n_samples) {
    std::vector<float> vad_samples;
    if (params.vad) {
        std::lock_guard<std::mutex> lk(ctx->state->mu);  // the pre-pass writes the default state's VAD fields
        if (!vad_filter(ctx, ctx->state, params, samples, n_samples, vad_samples)) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full: failed to compute VAD\n");
            return -1;
        }
        if (vad_samples.empty()) {
            ctx->state->result_all.clear();
            return 0;
        }
        samples = vad_samples.data();
        n_samples = (int) vad_samples.size();
    }
    return whisper_full_with_state(ctx, ctx->state, params, samples, n_samples);
}

// Splits the audio into n_processors chunks (ref 7801-7929). The chunks run as one
// batch on the device instead of n_processors CPU threads; merging is unchanged.
int whisper_full_parallel(struct whisper_context * ctx, struct whisper_full_params params, const float * samples,
                          int n_samples, int n_processors) {
    if (n_processors == 1) return whisper_full(ctx, params, samples, n_samples);
    std::vector<float> vad_samples;  // ref 7812-7824
    if (params.vad) {
        std::lock_guard<std::mutex> lk(ctx->state->mu);
        if (!vad_filter(ctx, ctx->state, params, samples, n_samples, vad_samples)) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full_parallel: failed to compute VAD\n");
            return -1;
        }
        if (vad_samples.empty()) return 0;
        samples = vad_samples.data();
        n_samples = (int) vad_samples.size();
    }
    const int offset_samples = (WHISPER_SAMPLE_RATE * params.offset_ms) / 1000;
    const int per = (n_samples - offset_samples) / n_processors;
    std::vector<whisper_state *> states(n_processors);
    std::vector<whisper_full_params> ps(n_processors, params);
    std::vector<const float *> ptr(n_processors);
    std::vector<int> ns(n_processors);
    states[0] = ctx->state;
    ps[0].print_realtime = false;
    ptr[0] = samples;
    ns[0] = offset_samples + per;
    for (int i = 1; i < n_processors; ++i) {
        states[i] = whisper_init_state(ctx);
        if (!states[i]) {
            for (int j = 1; j < i; ++j) whisper_free_state(states[j]);
            return -1;
        }
        const int start = offset_samples + i * per;
        ns[i] = (i == n_processors - 1) ? n_samples - start : per;
        ptr[i] = samples + start;
        ps[i].offset_ms = 0;
        ps[i].print_progress = false;
        ps[i].print_realtime = false;
        ps[i].new_segment_callback = nullptr;
        ps[i].new_segment_callback_user_data = nullptr;
        ps[i].progress_callback = nullptr;
        ps[i].progress_callback_user_data = nullptr;
    }
    int ret = 0;
    // the states of this call (the context's default state and the fresh ones), locked in address
    // order like owk_full_batch, and held through the merge below (it writes ctx->state's results
    // and timings); the context lock while the shared recorder is on
    std::vector<whisper_state *> held(states);
    std::sort(held.begin(), held.end());
    std::vector<std::unique_lock<std::mutex>> locks;
    std::unique_lock<std::mutex> ctx_lock(ctx->mu, std::defer_lock);
    if (ctx->prof.on) ctx_lock.lock();
    for (whisper_state * st : held) locks.emplace_back(st->mu);
    try {
        ret = full_batch(ctx, states.data(), ps.data(), nullptr, ptr.data(), ns.data(), n_processors);
    } catch (const std::exception & e) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_full_parallel: %s\n", e.what());
        ret = -6;
    }
    const int64_t offset_t = (int64_t) (params.offset_ms / 10.0);
    for (int i = 1; i < n_processors; ++i) {
        for (auto & r : states[i]->result_all) {
            r.t0 += 100 * ((i) * per) / WHISPER_SAMPLE_RATE + offset_t;
            r.t1 += 100 * ((i) * per) / WHISPER_SAMPLE_RATE + offset_t;
            if (!ctx->state->result_all.empty()) r.t0 = std::max(r.t0, ctx->state->result_all.back().t1);
            ctx->state->result_all.push_back(std::move(r));
            if (params.new_segment_callback)
                params.new_segment_callback(ctx, ctx->state, 1, params.new_segment_callback_user_data);
        }
        whisper_state * s = states[i];
        ctx->state->t_mel_us += s->t_mel_us;
        ctx->state->t_sample_us += s->t_sample_us;
        ctx->state->t_encode_us += s->t_encode_us;
        ctx->state->t_decode_us += s->t_decode_us;
        ctx->state->t_batchd_us += s->t_batchd_us;
        ctx->state->t_prompt_us += s->t_prompt_us;
        ctx->state->n_sample += s->n_sample;
        ctx->state->n_encode += s->n_encode;
        ctx->state->n_decode += s->n_decode;
        ctx->state->n_batchd += s->n_batchd;
        ctx->state->n_prompt += s->n_prompt;
    }
    ctx->state->t_mel_us /= n_processors;
    ctx->state->t_sample_us /= n_processors;
    ctx->state->t_encode_us /= n_processors;
    ctx->state->t_decode_us /= n_processors;
    locks.clear();  // release before freeing the helper states (their mutexes die with them)
    for (int i = 1; i < n_processors; ++i) whisper_free_state(states[i]);
    return ret;
}

int whisper_full_n_segments_from_state(struct whisper_state * state) { return (int) state->result_all.size(); }
int whisper_full_n_segments(struct whisper_context * ctx) { return (int) ctx->state->result_all.size(); }
int whisper_full_lang_id_from_state(struct whisper_state * state) { return state->lang_id; }
int whisper_full_lang_id(struct whisper_context * ctx) { return ctx->state->lang_id; }
// segment times in the original audio when whisper_full ran the VAD pre-pass (ref 7986-8025)
int64_t whisper_full_get_segment_t0_from_state(struct whisper_state * state, int i) {
    if (!state->has_vad_segments || state->vad_map.empty()) return state->result_all[i].t0;
    return vad_map_time(state->result_all[i].t0, state->vad_map);
}
int64_t whisper_full_get_segment_t1_from_state(struct whisper_state * state, int i) {
    if (!state->has_vad_segments || state->vad_map.empty()) return state->result_all[i].t1;
    int64_t t1 = vad_map_time(state->result_all[i].t1, state->vad_map);
    const int64_t t0 = whisper_full_get_segment_t0_from_state(state, i);
    if (t1 - t0 < 10) t1 = t0 + 10;
    return t1;
}
int64_t whisper_full_get_segment_t0(struct whisper_context * ctx, int i) { return whisper_full_get_segment_t0_from_state(ctx->state, i); }
int64_t whisper_full_get_segment_t1(struct whisper_context * ctx, int i) { return whisper_full_get_segment_t1_from_state(ctx->state, i); }
bool whisper_full_get_segment_speaker_turn_next_from_state(struct whisper_state * state, int i) {
    return state->result_all[i].speaker_turn_next;
}
bool whisper_full_get_segment_speaker_turn_next(struct whisper_context * ctx, int i) {
    return ctx->state->result_all[i].speaker_turn_next;
}
const char * whisper_full_get_segment_text_from_state(struct whisper_state * state, int i) {
    return state->result_all[i].text.c_str();
}
const char * whisper_full_get_segment_text(struct whisper_context * ctx, int i) { return ctx->state->result_all[i].text.c_str(); }
int whisper_full_n_tokens_from_state(struct whisper_state * state, int i) { return (int) state->result_all[i].tokens.size(); }
int whisper_full_n_tokens(struct whisper_context * ctx, int i) { return (int) ctx->state->result_all[i].tokens.size(); }
const char * whisper_full_get_token_text_from_state(struct whisper_context * ctx, struct whisper_state * state, int i, int j) {
    return ctx->model->vocab.id_to_token[state->result_all[i].tokens[j].id].c_str();
}
const char * whisper_full_get_token_text(struct whisper_context * ctx, int i, int j) {
    return ctx->model->vocab.id_to_token[ctx->state->result_all[i].tokens[j].id].c_str();
}
whisper_token whisper_full_get_token_id_from_state(struct whisper_state * state, int i, int j) {
    return state->result_all[i].tokens[j].id;
}
whisper_token whisper_full_get_token_id(struct whisper_context * ctx, int i, int j) { return ctx->state->result_all[i].tokens[j].id; }
struct whisper_token_data whisper_full_get_token_data_from_state(struct whisper_state * state, int i, int j) {
    return state->result_all[i].tokens[j];
}
struct whisper_token_data whisper_full_get_token_data(struct whisper_context * ctx, int i, int j) {
    return ctx->state->result_all[i].tokens[j];
}
float whisper_full_get_token_p_from_state(struct whisper_state * state, int i, int j) { return state->result_all[i].tokens[j].p; }
float whisper_full_get_token_p(struct whisper_context * ctx, int i, int j) { return ctx->state->result_all[i].tokens[j].p; }
float whisper_full_get_segment_no_speech_prob(struct whisper_context * ctx, int i) {
    return ctx->state->result_all[i].no_speech_prob;
}
float whisper_full_get_segment_no_speech_prob_from_state(struct whisper_state * state, int i) {
    return state->result_all[i].no_speech_prob;
}

// ---------------------------------------------------------------------------------
// microbenchmarks (ref 8107-8375: memcpy and ggml_mul_mat GFLOPS) on the device
// ---------------------------------------------------------------------------------
static std::string g_bench_str;

int whisper_bench_memcpy(int n_threads) {
    fputs(whisper_bench_memcpy_str(n_threads), stderr);
    return 0;
}

const char * whisper_bench_memcpy_str(int) {
    g_bench_str.clear();
    try {
        const size_t n = (size_t) 1 << 30;
        DevBuf a, b;
        a.alloc(n);
        b.alloc(n);
        OWK_HIP_CHECK(hipMemset(a.ptr, 1, n));
        hipEvent_t e0, e1;
        OWK_HIP_CHECK(hipEventCreate(&e0));
        OWK_HIP_CHECK(hipEventCreate(&e1));
        OWK_HIP_CHECK(hipMemcpy(b.ptr, a.ptr, n, hipMemcpyDeviceToDevice));
        OWK_HIP_CHECK(hipEventRecord(e0, nullptr));
        for (int i = 0; i < 10; ++i) OWK_HIP_CHECK(hipMemcpyAsync(b.ptr, a.ptr, n, hipMemcpyDeviceToDevice, nullptr));
        OWK_HIP_CHECK(hipEventRecord(e1, nullptr));
        OWK_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        OWK_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        char buf[256];
        snprintf(buf, sizeof(buf), "memcpy: %.2f GB/s (device to device, 1 GiB x 10, read+write)\n",
                 2.0 * 10.0 * n / (ms * 1e-3) / 1e9);
        g_bench_str = buf;
        (void) hipEventDestroy(e0);
        (void) hipEventDestroy(e1);
    } catch (const std::exception & e) {
        g_bench_str = std::string("memcpy: failed: ") + e.what() + "\n";
    }
    return g_bench_str.c_str();
}

int whisper_bench_ggml_mul_mat(int n_threads) {
    fputs(whisper_bench_ggml_mul_mat_str(n_threads), stderr);
    return 0;
}

const char * whisper_bench_ggml_mul_mat_str(int) {
    g_bench_str.clear();
    try {
        for (int N : {1024, 2048, 4096, 8192}) {
            DevBuf a, w, c;
            a.alloc((size_t) N * N * 2);
            w.alloc((size_t) N * N * 2);
            c.alloc((size_t) N * N * 2);
            OWK_HIP_CHECK(hipMemset(a.ptr, 0x11, a.bytes));
            OWK_HIP_CHECK(hipMemset(w.ptr, 0x11, w.bytes));
            EpiParams ep;
            ep.out16 = c.as<_Float16>();
            ep.ldo = N;
            gemm_f16(nullptr, EPI_F16, N, N, N, a.as<_Float16>(), N, w.as<_Float16>(), N, ep);
            OWK_HIP_CHECK(hipDeviceSynchronize());
            hipEvent_t e0, e1;
            OWK_HIP_CHECK(hipEventCreate(&e0));
            OWK_HIP_CHECK(hipEventCreate(&e1));
            const int iters = N >= 4096 ? 10 : 50;
            OWK_HIP_CHECK(hipEventRecord(e0, nullptr));
            for (int i = 0; i < iters; ++i)
                gemm_f16(nullptr, EPI_F16, N, N, N, a.as<_Float16>(), N, w.as<_Float16>(), N, ep);
            OWK_HIP_CHECK(hipEventRecord(e1, nullptr));
            OWK_HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0;
            OWK_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            char buf[256];
            snprintf(buf, sizeof(buf), "%5zu x %5zu: F16 %8.1f TFLOPS (MFMA gemm, %d runs)\n", (size_t) N, (size_t) N,
                     2.0 * N * (double) N * N * iters / (ms * 1e-3) / 1e12, iters);
            g_bench_str += buf;
            (void) hipEventDestroy(e0);
            (void) hipEventDestroy(e1);
        }
    } catch (const std::exception & e) {
        g_bench_str += std::string("mul_mat: failed: ") + e.what() + "\n";
    }
    return g_bench_str.c_str();
}

void whisper_log_set(ggml_log_callback log_callback, void * user_data) { set_log_callback(log_callback, user_data); }

// ---------------------------------------------------------------------------------
// owk.h extensions
// ---------------------------------------------------------------------------------
int owk_full_batch(struct whisper_context * ctx, struct whisper_state ** states, struct whisper_full_params params,
                   const struct owk_full_ext * ext, const float * const * samples, const int * n_samples, int n_clips) {
    // the states of this call, locked in address order (no lock-order inversion between concurrent
    // calls); the context lock only while the shared per-kernel recorder is on
    std::vector<whisper_state *> held(states, states + std::max(n_clips, 0));
    std::sort(held.begin(), held.end());
    held.erase(std::unique(held.begin(), held.end()), held.end());
    std::vector<std::unique_lock<std::mutex>> locks;
    std::unique_lock<std::mutex> ctx_lock(ctx->mu, std::defer_lock);
    if (ctx->prof.on) ctx_lock.lock();
    for (whisper_state * st : held)
        if (st) locks.emplace_back(st->mu);
    std::vector<whisper_full_params> ps(std::max(n_clips, 1), params);
    // (Round 2 measured clip groups on concurrent streams: 2 x 16 clips took exactly as long as one
    // batch of 32 and 4 x 8 took 2.3x as long, so the engine runs one stage-major batch per call.)
    try {
        return full_batch(ctx, states, ps.data(), ext, samples, n_samples, n_clips);
    } catch (const std::exception & e) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_full_batch: %s\n", e.what());
        return -6;
    }
}

void owk_prof_enable(struct whisper_context * ctx, int enable) {
    ctx->prof.flush();
    ctx->prof.on = enable != 0;
}

void owk_prof_reset(struct whisper_context * ctx) { ctx->prof.reset(); }

void owk_prof_select(struct whisper_context * ctx, const char * classes) {
    ctx->prof.flush();
    ctx->prof.only.clear();
    if (!classes) return;
    std::string cur;
    for (const char * c = classes;; ++c) {
        if (*c == ',' || *c == 0) {
            if (!cur.empty()) ctx->prof.only.push_back(cur);
            cur.clear();
            if (*c == 0) break;
        } else {
            cur += *c;
        }
    }
}

int owk_prof_read(struct whisper_context * ctx, const char * cls, double * total_ms, long * launches) {
    ctx->prof.flush();
    for (size_t i = 0; i < ctx->prof.names.size(); ++i)
        if (ctx->prof.names[i] == cls) {
            if (total_ms) *total_ms = ctx->prof.tot[i].ms;
            if (launches) *launches = ctx->prof.tot[i].n;
            return 0;
        }
    return -1;
}

int owk_prof_work(struct whisper_context * ctx, const char * cls, double * flops, double * bytes) {
    ctx->prof.flush();
    for (size_t i = 0; i < ctx->prof.names.size(); ++i)
        if (ctx->prof.names[i] == cls) {
            if (flops) *flops = ctx->prof.tot[i].flops;
            if (bytes) *bytes = ctx->prof.tot[i].bytes;
            return 0;
        }
    return -1;
}

const char * owk_prof_classes(struct whisper_context * ctx) {
    ctx->prof.flush();
    ctx->prof.classes_csv.clear();
    for (size_t i = 0; i < ctx->prof.names.size(); ++i) {
        if (i) ctx->prof.classes_csv += ",";
        ctx->prof.classes_csv += ctx->prof.names[i];
    }
    return ctx->prof.classes_csv.c_str();
}

int owk_device_ok(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device >= n) return 0;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return 0;
    return strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

const char * owk_build_info(void) { return "open-whisper-kit MI355X engine: gfx950 HIP kernels (MFMA f16), batch-major"; }

// debug / test hooks: reference intermediates of the last staged call on a state
int owk_debug_mel(struct whisper_state * st, float * out, int cap) {
    if (!st->eng) return -1;
    const int n = st->mel_n_mel * st->eng->mel_len(0);
    if (out) {
        if (cap < n) return -1;
        st->eng->download_mel(0, out);
    }
    return n;
}

int owk_debug_enc(struct whisper_context * ctx, struct whisper_state * st, int index, float * out, int cap) {
    const int n = (st->eng ? st->eng->n_ctx() : ctx->model->hp.n_audio_ctx) * ctx->model->hp.n_audio_state;
    if (!st->eng) return -1;
    if (out) {
        if (cap < n) return -1;
        st->eng->download_enc(index, out);
    }
    return n;
}

int owk_debug_cross(struct whisper_context * ctx, struct whisper_state * st, int slot, int layer, uint16_t * k, uint16_t * v) {
    if (!st->eng) return -1;
    const int n = st->eng->n_ctx() * ctx->model->hp.n_text_state;
    if (k && v) st->eng->download_cross(slot, layer, k, v);
    return n;
}

// host-only: the KV-cell allocator (kv_cells.h) driven by a script of find_slot / seq_rm / seq_cp /
// cell_max / clear records (include/owk.h)
int owk_debug_kv_cells(int n_ctx, const int * ops, int n_ops, int * out, int cap) {
    if (n_ctx <= 0 || n_ops < 0 || (n_ops > 0 && !ops) || !out) return -2;
    if (cap < n_ops + 1 + 2 * n_ctx) return -1;
    KvCells kv;
    kv.init((uint32_t) n_ctx);
    std::vector<int32_t> tpos, tseq;
    for (int i = 0; i < n_ops; ++i) {
        const int * o = ops + 5 * i;
        int r = 0;
        switch (o[0]) {
            case 0:
                if (o[1] < 0 || o[2] < 0 || o[2] > 31) return -2;
                tpos.resize(o[1]);
                tseq.assign(o[1], o[2]);
                for (int t = 0; t < o[1]; ++t) tpos[t] = o[3] + t;
                r = kv.find_slot(o[1], tpos.data(), tseq.data());
                break;
            case 1:
                if (o[1] > 31) return -2;
                kv.seq_rm(o[1], o[2], o[3]);
                break;
            case 2:
                if (o[1] < 0 || o[1] > 31 || o[2] < 0 || o[2] > 31) return -2;
                kv.seq_cp(o[1], o[2], o[3], o[4]);
                break;
            case 3: r = kv.cell_max(); break;
            case 4: kv.clear(); break;
            default: return -2;
        }
        out[i] = r;
    }
    out[n_ops] = (int) kv.head;
    for (int c = 0; c < n_ctx; ++c) {
        out[n_ops + 1 + 2 * c] = kv.pos[c];
        out[n_ops + 2 + 2 * c] = (int) kv.seq[c];
    }
    return n_ops + 1 + 2 * n_ctx;
}

// host-only: whisper_tokenize over the vocabulary of a model file (header, mel filters and vocab
// parsed by the product loader, no weights, no device)
int owk_debug_tokenize(const char * path_model, const char * text, int * out, int cap) {
    // the parsed vocabulary of the last file is kept (tests tokenize thousands of strings)
    static std::mutex mu;
    static std::string cached_path;
    static std::unique_ptr<Model> cached;
    try {
        std::lock_guard<std::mutex> lock(mu);
        if (!cached || cached_path != path_model) {
            cached.reset();
            std::ifstream fin(path_model, std::ios::binary);
            if (!fin) return INT32_MIN;
            whisper_model_loader loader = {};
            loader.context = &fin;
            loader.read = [](void * c, void * o, size_t n) {
                auto * f = (std::ifstream *) c;
                f->read((char *) o, n);
                return (size_t) f->gcount();
            };
            loader.eof = [](void * c) { return ((std::ifstream *) c)->eof(); };
            loader.close = [](void *) {};
            std::string err;
            cached.reset(load_model(&loader, 0, err, true));
            if (!cached) {
                log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_tokenize: %s\n", err.c_str());
                return INT32_MIN;
            }
            cached_path = path_model;
        }
        const std::vector<int> res = tokenize_text(cached->vocab, text);
        if (cap < (int) res.size()) return -(int) res.size();
        std::copy(res.begin(), res.end(), out);
        return (int) res.size();
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_tokenize: %s\n", ex.what());
        return INT32_MIN;
    }
}

const uint16_t * owk_debug_gelu_table(void) { return gelu_table_host().data(); }

// average device microseconds of `iters` back-to-back decode GEMM launches (event-timed)
long owk_debug_capture(struct whisper_state * st, float * out, long cap) {
    try {
        if (!st || !st->eng || st->eng->capture_rows() <= 0) return -1;
        std::vector<float> v;
        st->eng->download_capture(0, st->eng->capture_rows(), v);
        if (out) {
            if (cap < (long) v.size()) return -1;
            std::copy(v.begin(), v.end(), out);
        }
        return (long) v.size();
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_capture: %s\n", ex.what());
        return -1;
    }
}

int owk_debug_dtw(const float * cap, int n_ah, int n_audio_ctx, int n_tok, int sot_len, int n_frames, int medfilt,
                  int * out, int cap_out) {
    try {
        const auto v = owk::dtw_time_indices(cap, n_ah, n_audio_ctx, n_tok, sot_len, n_frames, medfilt);
        const int n = std::min<int>((int) v.size(), cap_out);
        for (int i = 0; i < n; ++i) out[i] = v[i];
        return n;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_dtw: %s\n", ex.what());
        return -1;
    }
}

int owk_debug_grammar_rejects(const whisper_grammar_element ** rules, size_t n_rules, size_t i_start_rule,
                              const char * const * vocab, int n_vocab, int eot, const int * accept, int n_accept, int * out,
                              int cap) {
    try {
        if (!vocab || eot < 0 || eot > n_vocab) throw std::runtime_error("bad vocabulary");
        std::vector<std::string> v(vocab, vocab + n_vocab);
        owk::Grammar g;
        g.init(rules, n_rules, i_start_rule);
        for (int i = 0; i < n_accept; ++i) {
            if (accept[i] < 0 || accept[i] >= n_vocab) throw std::runtime_error("accepted token out of range");
            g.accept(v[accept[i]]);
        }
        std::vector<float> logits(n_vocab, 0.0f);
        g.suppress(v, eot, 1.0f, logits.data());
        int n = 0;
        for (int id = 0; id < n_vocab; ++id)
            if (logits[id] != 0.0f) {
                if (n < cap) out[n] = id;
                ++n;
            }
        return n;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_grammar_rejects: %s\n", ex.what());
        return -1;
    }
}

// uniform random f16 in [-1, 1) from a per-element hash: GEMM timings on random data (zero-filled
// operands run 15-21 % faster through DVFS, CDNA guide 5.4 rule 25)
__global__ static void k_fill_rand_f16(_Float16 * p, size_t n, uint32_t seed) {
    for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t) i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        p[i] = (_Float16) ((float) (h & 0xFFFF) / 32768.0f - 1.0f);
    }
}

// mode bit 0x100: force the 128x128 large-GEMM kernel; 0x800 (the default): the 8-phase 256x256 kernel;
// 0x1000 / 0x2000: the 64x64 / 32x32 ring tile; bit 0x200: random operands
double owk_debug_gemm_bench(int device, int mode, int M, int N, int K, int iters) {
    const bool force128 = mode & 0x100, rnd = mode & 0x200, mid = mode & 0x1000, mid32 = mode & 0x2000;
    mode &= 0xFF;
    GemmOverride ov(force128 ? 0 : mid ? GEMM_MID_FORCED : mid32 ? GEMM_MID32_FORCED : 8);
    try {
        OWK_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        DevBuf da, dw, dwt, d32, d16, dres, part, bias, gtab;
        da.alloc((size_t) M * K * 2);
        gtab.alloc(65536 * 2);  // EPI_GELU_F16 timing: table contents do not matter
        OWK_HIP_CHECK(hipMemset(gtab.ptr, 0, gtab.bytes));
        dw.alloc((size_t) N * K * 2);
        dwt.alloc(tiled_weight_elems(N, K) * 2);
        d32.alloc((size_t) M * N * 4);
        d16.alloc((size_t) M * N * 2);
        dres.alloc((size_t) M * N * 4);
        bias.alloc((size_t) N * 4);
        OWK_HIP_CHECK(hipMemset(da.ptr, 0, da.bytes));
        OWK_HIP_CHECK(hipMemset(dw.ptr, 0, dw.bytes));
        if (rnd) {
            hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, da.as<_Float16>(), (size_t) M * K, 1u);
            hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, dw.as<_Float16>(), (size_t) N * K, 7u);
        }
        OWK_HIP_CHECK(hipMemset(dres.ptr, 0, dres.bytes));
        OWK_HIP_CHECK(hipMemset(bias.ptr, 0, bias.bytes));
        tile_weights(s, dw.as<_Float16>(), N, K, dwt.as<_Float16>());
        const size_t fl = std::max(gemm_ws_floats(N, K), gemm_partial_floats(N, K));
        part.alloc(std::max<size_t>(fl, 1) * 4);
        GemmWs ws;
        ws.partial = part.as<float>();
        ws.partial_floats = fl;
        EpiParams ep;
        ep.bias = bias.as<float>();
        ep.resid = dres.as<float>();
        ep.out32 = d32.as<float>();
        ep.out16 = d16.as<_Float16>();
        ep.ldo = N;
        ep.gelu_tab = gtab.as<uint16_t>();
        if (mode == EPI_QKV_ENC || mode == EPI_KV_CROSS) {  // the encoder's head-major outputs, 1500-row clips
            ep.d = mode == EPI_QKV_ENC ? N / 3 : N / 2;
            ep.T = 1500;
            ep.Tpad = 1536;
            ep.scale = 1.0f;
            ep.bias2 = bias.as<float>();
            ep.out16b = d16.as<_Float16>();
            ep.out16c = d16.as<_Float16>() + (size_t) M * ep.d;
            const size_t v_elems = mode == EPI_QKV_ENC ? (size_t) (M / 1500) * ep.d * 1536 : (size_t) M * ep.d;
            if (M % 1500 != 0 || v_elems > (size_t) M * N - (size_t) M * ep.d)
                throw std::runtime_error("gemm bench: head-major outputs need M = clips x 1500 and room for V");
        }
        hipEvent_t e0, e1;
        OWK_HIP_CHECK(hipEventCreate(&e0));
        OWK_HIP_CHECK(hipEventCreate(&e1));
        for (int i = 0; i < 3; ++i)
            gemm(s, mode, M, N, K, da.as<_Float16>(), K, dw.as<_Float16>(), K, ep, &ws, dwt.as<_Float16>());
        OWK_HIP_CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; ++i)
            gemm(s, mode, M, N, K, da.as<_Float16>(), K, dw.as<_Float16>(), K, ep, &ws, dwt.as<_Float16>());
        OWK_HIP_CHECK(hipEventRecord(e1, s));
        OWK_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        OWK_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void) hipEventDestroy(e0);
        (void) hipEventDestroy(e1);
        OWK_HIP_CHECK(hipStreamDestroy(s));
        return 1e3 * ms / iters;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_gemm_bench: %s\n", ex.what());
        return -1;
    }
}

// The decoder's per-layer matmul + residual/LayerNorm chain of a large-v3-shaped model (d = 1280,
// 32 layers, R rows) WITHOUT the attention kernels, as the engine's fused R <= 32 path launches it
// (engine.cpp launch_decode): QKV (EPI_QKV_DEC) -> O partial + resid_layernorm -> cross Q -> cross-O
// partial + resid_layernorm -> mlp.0 (GELU) -> mlp.2 partial + resid_layernorm. Distinct random
// weights per layer (1.47 GB: every replay streams them from HBM as a decode step does), the whole
// chain captured in one hipGraph; returns device microseconds per layer (events around replays).
double owk_debug_decode_chain(int device, int R, int n_layers, int iters) {
    return owk_debug_decode_chain2(device, R, n_layers, iters, 0);
}

// variant 0: split-K partial residual matmuls + resid_layernorm, consumers read the f16 LayerNorm rows
// (the round-3 chain); 1: LayerNorm in the consumer prologue (gemm_rows_ln) + whole-K residual epilogues;
// 2: as 1 with the prologue statistics skipped (timing only); 3: as 1 but mlp.2 split-K + resid_layernorm
// and the next QKV from its f16 rows; 4: as 0 but attn.out / cross_attn.out whole-K + LN prologue consumers;
// 5: the bit-exact whole-K chain the engine runs at <= whole_k_rows() rows (gemm_rows_res + gemm_rows_lnx)
double owk_debug_decode_chain2(int device, int R, int n_layers, int iters, int variant) {
    try {
        OWK_HIP_CHECK(hipSetDevice(device));
        if (R < 1 || R > 32 || n_layers < 1) throw std::runtime_error("bad shape");
        const int d = 1280;
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        struct LW { DevBuf qkv, o, cq, co, m0, m1; };
        std::vector<LW> lw(n_layers);
        auto fill = [&](DevBuf & b, int N, int K) {
            b.alloc(tiled_weight_elems(N, K) * 2);
            hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, b.as<_Float16>(), tiled_weight_elems(N, K),
                               (uint32_t) (size_t) b.ptr);
        };
        for (auto & l : lw) {
            fill(l.qkv, 3 * d, d); fill(l.o, d, d); fill(l.cq, d, d); fill(l.co, d, d); fill(l.m0, 4 * d, d);
            fill(l.m1, d, 4 * d);
        }
        DevBuf x, xn, q, ao, h, kc, vc, bias, bias4, lnw, lnb, part, rowoff, gt;
        x.alloc((size_t) R * d * 4); xn.alloc((size_t) R * d * 2); q.alloc((size_t) R * d * 2); ao.alloc((size_t) R * d * 2);
        h.alloc((size_t) R * 4 * d * 2);
        const int cells = 512;
        kc.alloc((size_t) 32 * cells * d * 2); vc.alloc((size_t) 32 * cells * d * 2);
        bias.alloc((size_t) 3 * d * 4); bias4.alloc((size_t) 4 * d * 4); lnw.alloc((size_t) d * 4); lnb.alloc((size_t) d * 4);
        gt.alloc(65536 * 2);
        for (DevBuf * b : {&x, &xn, &q, &ao, &h, &bias, &bias4, &lnb, &gt}) OWK_HIP_CHECK(hipMemsetAsync(b->ptr, 0, b->bytes, s));
        std::vector<float> ones(d, 1.0f);
        OWK_HIP_CHECK(hipMemcpy(lnw.ptr, ones.data(), d * 4, hipMemcpyHostToDevice));
        std::vector<int64_t> ro(R);
        for (int r = 0; r < R; ++r) ro[r] = (int64_t) r * cells * d + 7 * 64;
        rowoff.alloc(R * 8);
        OWK_HIP_CHECK(hipMemcpy(rowoff.ptr, ro.data(), R * 8, hipMemcpyHostToDevice));
        size_t fl = 0;
        for (int N : {3 * d, d, 4 * d})
            for (int K : {d, 4 * d}) fl = std::max(fl, std::max(gemm_ws_floats(N, K), gemm_partial_floats(N, K)));
        part.alloc(fl * 4);
        GemmWs ws;
        ws.partial = part.as<float>();
        ws.partial_floats = fl;
        // site 0 attn.out, 1 cross_attn.out, 2 mlp.2: split (partial + resid_layernorm) or whole-K
        auto split_site = [&](int site) {
            if (variant == 0) return true;
            if (variant == 3) return site == 2;
            if (variant == 4) return site == 2;
            return false;
        };
        // consumer c (0 QKV, 1 cross-Q, 2 mlp.0) takes the LayerNorm in its prologue unless its producer
        // (c = 0: the previous mlp.2, 1: attn.out, 2: cross_attn.out) finished the rows with resid_layernorm
        auto ln_prologue = [&](int c) { return !split_site(c == 0 ? 2 : c - 1); };
        if (variant == 5 && !gemm_rows_exact_applies(R, d)) throw std::runtime_error("variant 5: too many rows");
        auto resid = [&](int site, const _Float16 * A, const _Float16 * Wt, int K) {
            if (variant == 5) {
                gemm_rows_res(s, R, d, K, A, Wt, bias.as<float>(), x.as<float>());
            } else if (split_site(site)) {
                gemm(s, EPI_PARTIAL, R, d, K, A, K, nullptr, K, EpiParams(), &ws, Wt);
                resid_layernorm(s, R, d, gemm_partial_splits(K), ws.partial, bias.as<float>(), x.as<float>(), lnw.as<float>(),
                                lnb.as<float>(), 1e-5f, xn.as<_Float16>(), d);
            } else {
                EpiParams e;
                e.bias = bias.as<float>(); e.resid = x.as<float>(); e.out32 = x.as<float>(); e.ldo = d;
                gemm(s, EPI_RESID_F32, R, d, K, A, K, nullptr, K, e, &ws, Wt);
            }
        };
        auto consumer = [&](int c, int mode, int N, const _Float16 * Wt, const EpiParams & e) {
            if (variant == 5)
                gemm_rows_lnx(s, mode, 0, R, N, d, x.as<float>(), lnw.as<float>(), lnb.as<float>(), 1e-5f, Wt, e);
            else if (ln_prologue(c))
                gemm_rows_ln(s, mode, R, N, d, x.as<float>(), lnw.as<float>(), lnb.as<float>(), 1e-5f, Wt, e, variant == 2);
            else
                gemm(s, mode, R, N, d, xn.as<_Float16>(), d, nullptr, d, e, &ws, Wt);
        };
        auto chain = [&]() {
            for (int l = 0; l < n_layers; ++l) {
                const LW & L = lw[l];
                EpiParams e1;
                e1.bias = bias.as<float>(); e1.bias2 = bias.as<float>(); e1.scale = 0.35f;
                e1.out16 = q.as<_Float16>(); e1.ldo = d; e1.out16b = kc.as<_Float16>(); e1.out16c = vc.as<_Float16>();
                e1.d = d; e1.row_off = rowoff.as<int64_t>(); e1.Tpad = cells * 64;
                consumer(0, EPI_QKV_DEC, 3 * d, L.qkv.as<_Float16>(), e1);
                resid(0, ao.as<_Float16>(), L.o.as<_Float16>(), d);
                EpiParams e2;
                e2.bias = bias.as<float>(); e2.out16 = q.as<_Float16>(); e2.ldo = d;
                consumer(1, EPI_F16, d, L.cq.as<_Float16>(), e2);
                resid(1, ao.as<_Float16>(), L.co.as<_Float16>(), d);
                EpiParams e3;
                e3.bias = bias4.as<float>(); e3.gelu_tab = gt.as<uint16_t>(); e3.out16 = h.as<_Float16>(); e3.ldo = 4 * d;
                consumer(2, EPI_GELU_F16, 4 * d, L.m0.as<_Float16>(), e3);
                resid(2, h.as<_Float16>(), L.m1.as<_Float16>(), 4 * d);
            }
        };
        OWK_HIP_CHECK(hipStreamSynchronize(s));
        hipGraph_t g = nullptr;
        hipGraphExec_t ex = nullptr;
        OWK_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        chain();
        OWK_HIP_CHECK(hipStreamEndCapture(s, &g));
        OWK_HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
        (void) hipGraphDestroy(g);
        for (int i = 0; i < 2; ++i) OWK_HIP_CHECK(hipGraphLaunch(ex, s));
        hipEvent_t e0, e1;
        OWK_HIP_CHECK(hipEventCreate(&e0));
        OWK_HIP_CHECK(hipEventCreate(&e1));
        OWK_HIP_CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; ++i) OWK_HIP_CHECK(hipGraphLaunch(ex, s));
        OWK_HIP_CHECK(hipEventRecord(e1, s));
        OWK_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        OWK_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void) hipEventDestroy(e0);
        (void) hipEventDestroy(e1);
        (void) hipGraphExecDestroy(ex);
        OWK_HIP_CHECK(hipStreamDestroy(s));
        return 1e3 * ms / iters / n_layers;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_decode_chain: %s\n", ex.what());
        return -1;
    }
}

// K-quant formats (kquant.h): the model's path for every shape -- host expansion to the virtual
// blocks, Q8_K activation rows (quantize_q8k_f16), gemm_q16 over the virtual K. q_out: the virtual
// activation row values [M][kq_kx] as int8 (the bsums of layout 0 saturate: only q is checked),
// d_out: the Q8_K d of every row and super-block [M][K/256]
static int debug_gemm_kquant(int device, int fmt, int M, int N, int K, const float * a, const uint8_t * w_blocks,
                             float * out, int8_t * q_out, float * d_out) {
    OWK_HIP_CHECK(hipSetDevice(device));
    hipStream_t s;
    OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int kx = kq_kx(fmt, K), nkb = kx / 32, nsb = K / 256;
    const int npad = (N + 255) / 256 * 256, mpad = (M + 255) / 256 * 256;
    std::vector<uint16_t> wi((size_t) N * kx);
    std::vector<float> dwt((size_t) nkb * npad);
    kq_expand_host(fmt, w_blocks, N, K, wi.data(), dwt.data(), npad);
    DevBuf da, dwi, ddw, q16, q16d, dout;
    da.alloc((size_t) M * K * 4);
    dwi.alloc(wi.size() * 2);
    ddw.alloc(dwt.size() * 4);
    q16.alloc((size_t) M * kx * 2);
    q16d.alloc((size_t) nkb * mpad * 4);
    dout.alloc((size_t) M * N * 4);
    OWK_HIP_CHECK(hipMemcpy(da.ptr, a, (size_t) M * K * 4, hipMemcpyHostToDevice));
    OWK_HIP_CHECK(hipMemcpy(dwi.ptr, wi.data(), wi.size() * 2, hipMemcpyHostToDevice));
    OWK_HIP_CHECK(hipMemcpy(ddw.ptr, dwt.data(), dwt.size() * 4, hipMemcpyHostToDevice));
    Q5W w;
    w.fmt = fmt;
    w.wi = dwi.as<_Float16>();
    w.dwt = ddw.as<float>();
    w.npad = npad;
    w.kx = kx;
    quantize_q8k_f16(s, da.as<float>(), nullptr, K, M, K, fmt, q16.as<_Float16>(), q16d.as<float>(), mpad);
    EpiParams ep;
    ep.out32 = dout.as<float>();
    ep.ldo = N;
    gemm_q16(s, EPI_F32, M, N, kx, q16.as<_Float16>(), q16d.as<float>(), mpad, w, ep);
    OWK_HIP_CHECK(hipStreamSynchronize(s));
    OWK_HIP_CHECK(hipMemcpy(out, dout.ptr, (size_t) M * N * 4, hipMemcpyDeviceToHost));
    if (q_out) {
        std::vector<_Float16> h((size_t) M * kx);
        OWK_HIP_CHECK(hipMemcpy(h.data(), q16.ptr, h.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h.size(); ++i) q_out[i] = (int8_t) std::max(-128.0f, std::min(127.0f, (float) h[i]));
    }
    if (d_out) {
        std::vector<float> h((size_t) nkb * mpad);
        OWK_HIP_CHECK(hipMemcpy(h.data(), q16d.ptr, h.size() * 4, hipMemcpyDeviceToHost));
        const int per = nkb / nsb;
        for (int r = 0; r < M; ++r) {
            const int t = r & 127, pr = (r & ~127) | (t & 64) | ((t & 15) << 2) | ((t >> 4) & 3);
            for (int sb = 0; sb < nsb; ++sb) d_out[(size_t) r * nsb + sb] = h[(size_t) sb * per * mpad + pr];
        }
    }
    OWK_HIP_CHECK(hipStreamDestroy(s));
    return 0;
}

// host-only K-quant decoding (tests/test_kquant.py, CPU): N rows of ggml blocks -> the virtual-block
// expansion (wi [N][kx] f16 bits, dwt [kx/32][N]) and / or the reference's f32 row dequantization
int owk_debug_kquant(int fmt, int N, int K, const uint8_t * w_blocks, uint16_t * wi, float * dwt, float * deq) {
    try {
        if (!qf_is_k(fmt) || N <= 0 || K % 256) throw std::runtime_error("bad format or shape");
        if (wi || dwt) {
            const int kx = kq_kx(fmt, K);
            std::vector<uint16_t> w((size_t) N * kx);
            std::vector<float> d((size_t) (kx / 32) * N);
            kq_expand_host(fmt, w_blocks, N, K, w.data(), d.data(), N);
            if (wi) memcpy(wi, w.data(), w.size() * 2);
            if (dwt) memcpy(dwt, d.data(), d.size() * 4);
        }
        if (deq) {
            const size_t rb = (size_t) K / 256 * kq_block_bytes(fmt);
            for (int n = 0; n < N; ++n) kq_dequant_row_host(fmt, w_blocks + n * rb, K, deq + (size_t) n * K);
        }
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_kquant: %s\n", ex.what());
        return -1;
    }
    return 0;
}

int owk_debug_gemm_quant(int device, int fmt, int M, int N, int K, const float * a, const uint8_t * w_blocks,
                         float * out, int8_t * q_out, float * d_out) {
    return owk_debug_gemm_quant2(device, fmt, M, N, K, a, w_blocks, out, q_out, d_out, 0);
}

int owk_debug_gemm_quant2(int device, int fmt, int M, int N, int K, const float * a, const uint8_t * w_blocks,
                          float * out, int8_t * q_out, float * d_out, int use_q16) {
    try {
        if (qf_is_k(fmt)) return debug_gemm_kquant(device, fmt, M, N, K, a, w_blocks, out, q_out, d_out);
        if (fmt < QF_Q5_0 || fmt > QF_Q5_1 || K % 32) throw std::runtime_error("bad format or K");
        OWK_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const int nb = K / 32;
        const size_t nbk = (size_t) N * nb;
        std::vector<uint8_t> qs(nbk * qf_qs_bytes(fmt));
        std::vector<uint32_t> qh(nbk);
        std::vector<uint16_t> dd(nbk), mm(nbk);
        quant_split_host(fmt, w_blocks, N, K, qs.data(), qh.data(), dd.data(), mm.data());
        DevBuf da, dqs, dqh, ddd, dmm, dout, q8, q8d;
        da.alloc((size_t) M * K * 4);
        dqs.alloc(qs.size());
        dqh.alloc(qh.size() * 4);
        ddd.alloc(dd.size() * 2);
        dmm.alloc(mm.size() * 2);
        dout.alloc((size_t) M * N * 4);
        q8.alloc((size_t) M * K);
        q8d.alloc((size_t) M * nb * 4);
        OWK_HIP_CHECK(hipMemcpy(da.ptr, a, (size_t) M * K * 4, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(dqs.ptr, qs.data(), qs.size(), hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(dqh.ptr, qh.data(), qh.size() * 4, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(ddd.ptr, dd.data(), dd.size() * 2, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(dmm.ptr, mm.data(), mm.size() * 2, hipMemcpyHostToDevice));
        Q5W w;
        w.fmt = fmt;
        w.qs = dqs.as<uint8_t>();
        w.qh = qf_has_qh(fmt) ? dqh.as<uint32_t>() : nullptr;
        w.d = ddd.as<_Float16>();
        w.m = qf_has_m(fmt) ? dmm.as<_Float16>() : nullptr;
        // the tiled copy a model keeps for its decode-step matrices (decode-row GEMM path)
        std::vector<uint8_t> tl(quant_tiled_bytes(fmt, N, K));
        quant_tile_host(fmt, qs.data(), qh.data(), dd.data(), mm.data(), N, K, tl.data());
        DevBuf dtl;
        dtl.alloc(tl.size());
        OWK_HIP_CHECK(hipMemcpy(dtl.ptr, tl.data(), tl.size(), hipMemcpyHostToDevice));
        w.tiled = dtl.as<uint8_t>();
        quantize_q8(s, da.as<float>(), nullptr, K, M, K, q8.as<int8_t>(), q8d.as<float>());
        EpiParams ep;
        ep.out32 = dout.as<float>();
        ep.ldo = N;
        DevBuf wi, dwt, q16, q16d;
        if (use_q16 == 1) {
            // the large-tile path of the encoder: expanded weights, f16 Q8_0 integers, gemm_q16
            w.npad = (N + 255) / 256 * 256;
            wi.alloc((size_t) N * K * 2);
            dwt.alloc((size_t) nb * w.npad * 4);
            quant_expand_f16(s, w, N, K, wi.as<_Float16>(), dwt.as<float>(), w.npad);
            w.wi = wi.as<_Float16>();
            w.dwt = dwt.as<float>();
            if (!gemm_q16_applies(w, M, N, K)) throw std::runtime_error("gemm_q16 does not apply to this shape");
            const int mpad = (M + 255) / 256 * 256;
            q16.alloc((size_t) M * K * 2);
            q16d.alloc((size_t) nb * mpad * 4);
            quantize_q8_f16(s, da.as<float>(), nullptr, K, M, K, q16.as<_Float16>(), q16d.as<float>(), mpad);
            gemm_q16(s, EPI_F32, M, N, K, q16.as<_Float16>(), q16d.as<float>(), mpad, w, ep);
        } else if (use_q16 == 2) {
            // the MLP0 form: EPI_GELU_F16 decode rows that also write the next GEMM's Q8_0 rows. The GELU
            // table is the identity (out16 = f16(row . col)), so out is comparable with the EPI_F32 launch;
            // q_out [M][N] / d_out [M][N/32] receive the epilogue's Q8_0 rows
            if (M > 32 || N % 32) throw std::runtime_error("GELU + Q8_0 rows: M <= 32, N % 32 == 0");
            std::vector<uint16_t> tab(65536), o16((size_t) M * N);
            for (int i = 0; i < 65536; ++i) tab[i] = (uint16_t) i;
            DevBuf dtab, do16, dbias, hq, hqd;
            dtab.alloc(tab.size() * 2);
            do16.alloc(o16.size() * 2);
            dbias.alloc((size_t) N * 4);
            hq.alloc((size_t) M * N);
            hqd.alloc((size_t) M * (N / 32) * 4);
            OWK_HIP_CHECK(hipMemcpy(dtab.ptr, tab.data(), tab.size() * 2, hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemset(dbias.ptr, 0, dbias.bytes));
            EpiParams eg;
            eg.bias = dbias.as<float>();
            eg.gelu_tab = dtab.as<uint16_t>();
            eg.out16 = do16.as<_Float16>();
            eg.ldo = N;
            eg.q8 = hq.as<int8_t>();
            eg.q8d = hqd.as<float>();
            gemm_q5(s, EPI_GELU_F16, M, N, K, q8.as<int8_t>(), q8d.as<float>(), w, eg);
            OWK_HIP_CHECK(hipStreamSynchronize(s));
            OWK_HIP_CHECK(hipMemcpy(o16.data(), do16.ptr, o16.size() * 2, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < o16.size(); ++i) out[i] = f16_to_f32_host(o16[i]);
            if (q_out) OWK_HIP_CHECK(hipMemcpy(q_out, hq.ptr, (size_t) M * N, hipMemcpyDeviceToHost));
            if (d_out) OWK_HIP_CHECK(hipMemcpy(d_out, hqd.ptr, (size_t) M * (N / 32) * 4, hipMemcpyDeviceToHost));
            OWK_HIP_CHECK(hipStreamDestroy(s));
            return 0;
        } else {
            gemm_q5(s, EPI_F32, M, N, K, q8.as<int8_t>(), q8d.as<float>(), w, ep);
        }
        OWK_HIP_CHECK(hipStreamSynchronize(s));
        OWK_HIP_CHECK(hipMemcpy(out, dout.ptr, (size_t) M * N * 4, hipMemcpyDeviceToHost));
        if (q_out) OWK_HIP_CHECK(hipMemcpy(q_out, q8.ptr, (size_t) M * K, hipMemcpyDeviceToHost));
        if (d_out) OWK_HIP_CHECK(hipMemcpy(d_out, q8d.ptr, (size_t) M * nb * 4, hipMemcpyDeviceToHost));
        OWK_HIP_CHECK(hipStreamDestroy(s));
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_gemm_quant: %s\n", ex.what());
        return -1;
    }
    return 0;
}

int owk_debug_gemm_q5(int device, int M, int N, int K, const float * a, const uint8_t * w_blocks, float * out,
                      int8_t * q_out, float * d_out) {
    return owk_debug_gemm_quant(device, QF_Q5_0, M, N, K, a, w_blocks, out, q_out, d_out);
}

// one_chunk cross attention of R rows (row r over its own clip r: k, v [R][H][T][64] f16 head-major,
// q [R][H*64]) with k_attn_step, one wave (which = 1) or a loader and a math wave (2); out [R][H*64] f16.
// iters > 0: also returns the mean device time per launch in microseconds (random q/k/v if the host
// pointers are null); iters == 0 returns 0; -1 on error
double owk_debug_attn_cross(int device, int which, int R, int H, int T, int n_zero_pad, float scale, const uint16_t * q,
                            const uint16_t * k, const uint16_t * v, uint16_t * out, int iters) {
    try {
        if (R <= 0 || H <= 0 || T < 0 || n_zero_pad < 0 || (which != 1 && which != 2) || iters < 0)
            throw std::runtime_error("bad arguments");
        OWK_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const size_t nq = (size_t) R * H * 64, nkv = std::max<size_t>((size_t) R * H * T * 64, 64);
        // random inputs: timed launches rotate over 8 K/V copies, so no launch finds its K/V in the
        // 256 MB MALL from the one before (as in a decode step, where each layer's cross K/V is cold)
        const int copies = (q && k && v) ? 1 : 8;
        DevBuf dq, dk, dv, dout, drows;
        dq.alloc(nq * 2);
        dk.alloc(nkv * 2 * copies);
        dv.alloc(nkv * 2 * copies);
        dout.alloc(nq * 2);
        if (q && k && v) {
            OWK_HIP_CHECK(hipMemcpy(dq.ptr, q, nq * 2, hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemcpy(dk.ptr, k, (size_t) R * H * T * 64 * 2, hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemcpy(dv.ptr, v, (size_t) R * H * T * 64 * 2, hipMemcpyHostToDevice));
        } else {
            hipLaunchKernelGGL(k_fill_rand_f16, dim3(1024), dim3(256), 0, s, dq.as<_Float16>(), nq, 3u);
            hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, dk.as<_Float16>(), nkv * copies, 5u);
            hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, dv.as<_Float16>(), nkv * copies, 9u);
        }
        std::vector<AttnRow> rows(R);
        for (int r = 0; r < R; ++r) rows[r] = AttnRow{r, r * H * T * 64, T, -1, n_zero_pad, 0};
        drows.alloc(R * sizeof(AttnRow));
        OWK_HIP_CHECK(hipMemcpy(drows.ptr, rows.data(), R * sizeof(AttnRow), hipMemcpyHostToDevice));
        int it = 0;
        auto run = [&] {
            const size_t c = (size_t) (it++ % copies) * nkv;
            attn_cross_kernel(s, which, dq.as<_Float16>(), H * 64, dk.as<_Float16>() + c, dv.as<_Float16>() + c, T * 64,
                              (const AttnRow *) drows.ptr, R, H, scale, dout.as<_Float16>(), H * 64);
        };
        run();
        double us = 0.0;
        if (iters > 0) {
            hipEvent_t e0, e1;
            OWK_HIP_CHECK(hipEventCreate(&e0));
            OWK_HIP_CHECK(hipEventCreate(&e1));
            OWK_HIP_CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i) run();
            OWK_HIP_CHECK(hipEventRecord(e1, s));
            OWK_HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0;
            OWK_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            (void) hipEventDestroy(e0);
            (void) hipEventDestroy(e1);
            us = 1e3 * ms / iters;
        }
        OWK_HIP_CHECK(hipStreamSynchronize(s));
        if (out) OWK_HIP_CHECK(hipMemcpy(out, dout.ptr, nq * 2, hipMemcpyDeviceToHost));
        OWK_HIP_CHECK(hipStreamDestroy(s));
        return us;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_attn_cross: %s\n", ex.what());
        return -1;
    }
}

// soft_max decoder attention (flash_attn = false rows) on random q / K / V: the key-split form (split
// != 0, attn_decoder_softmax with its workspace) or the single-block kernel; R rows x H heads x T keys
// (cross layout), heads 0 .. 3 captured as DTW alignment heads. Writes out [R][H*64] f16 and cap
// [4][T][R] f32 (either may be null); returns us per call over `iters` timed calls, or -1 on error.
double owk_debug_attn_softmax(int device, int split, int R, int H, int T, uint16_t * out, float * cap_out, int iters) {
    try {
        if (R <= 0 || H < 4 || T <= 0 || iters < 0) throw std::runtime_error("bad arguments");
        OWK_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const size_t nq = (size_t) R * H * 64, nkv = (size_t) R * H * T * 64;
        DevBuf dq, dk, dv, dout, drows, damap, dcap, dws;
        dq.alloc(nq * 2);
        dk.alloc(nkv * 2);
        dv.alloc(nkv * 2);
        dout.alloc(nq * 2);
        hipLaunchKernelGGL(k_fill_rand_f16, dim3(1024), dim3(256), 0, s, dq.as<_Float16>(), nq, 3u);
        hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, dk.as<_Float16>(), nkv, 5u);
        hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, dv.as<_Float16>(), nkv, 9u);
        std::vector<AttnRow> rows(R);
        for (int r = 0; r < R; ++r) rows[r] = AttnRow{r, r * H * T * 64, T, -1, 0, 2};
        drows.alloc(R * sizeof(AttnRow));
        OWK_HIP_CHECK(hipMemcpy(drows.ptr, rows.data(), R * sizeof(AttnRow), hipMemcpyHostToDevice));
        std::vector<int> amap(H, -1);
        for (int h = 0; h < 4; ++h) amap[h] = h;
        damap.alloc(H * sizeof(int));
        OWK_HIP_CHECK(hipMemcpy(damap.ptr, amap.data(), H * sizeof(int), hipMemcpyHostToDevice));
        dcap.alloc((size_t) 4 * T * R * 4);
        if (split == 1) {
            dws.alloc(attn_softmax_ws_floats(R, H) * 4);
            OWK_HIP_CHECK(hipMemsetAsync(dws.ptr, 0, dws.bytes, s));
        }
        // split: 0 single-block kernel at the engine's width, 1 key-split form, 256 / 1024 single-block at
        // that width
        auto run = [&] {
            attn_softmax_force_nt = split >= 256 ? split : 0;
            attn_decoder_softmax(s, dq.as<_Float16>(), H * 64, dk.as<_Float16>(), dv.as<_Float16>(), 64, T * 64,
                                 (const AttnRow *) drows.ptr, R, nullptr, H, 0.125f, T, dout.as<_Float16>(), H * 64,
                                 damap.as<int>(), dcap.as<float>(), R, nullptr, split == 1 ? dws.as<float>() : nullptr,
                                 split == 1 ? dws.bytes / 4 : 0);
            attn_softmax_force_nt = 0;
        };
        run();
        double us = 0.0;
        if (iters > 0) {
            hipEvent_t e0, e1;
            OWK_HIP_CHECK(hipEventCreate(&e0));
            OWK_HIP_CHECK(hipEventCreate(&e1));
            OWK_HIP_CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i) run();
            OWK_HIP_CHECK(hipEventRecord(e1, s));
            OWK_HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0;
            OWK_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            (void) hipEventDestroy(e0);
            (void) hipEventDestroy(e1);
            us = 1e3 * ms / iters;
        }
        OWK_HIP_CHECK(hipStreamSynchronize(s));
        if (out) OWK_HIP_CHECK(hipMemcpy(out, dout.ptr, nq * 2, hipMemcpyDeviceToHost));
        if (cap_out) OWK_HIP_CHECK(hipMemcpy(cap_out, dcap.ptr, (size_t) 4 * T * R * 4, hipMemcpyDeviceToHost));
        OWK_HIP_CHECK(hipStreamDestroy(s));
        return us;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_attn_softmax: %s\n", ex.what());
        return -1;
    }
}

// one large-tile GEMM epilogue mode through the 128x128 kernel (per-element epilogue) and the
// 256x256 ring kernel (C^T tiles, 16-byte vector epilogue) on the same random operands, bias,
// residual, positional rows and the real GELU table; returns the max |difference| over every
// output the mode writes (f32 and f16 images), or -1 on error. d / T: EPI_QKV_ENC / EPI_KV_CROSS /
// EPI_CONV2 shape parameters (N = 3d / 2d / d).
double owk_debug_gemm_epi_diff(int device, int mode, int M, int N, int K, int d, int T) {
    // 0x800: the 8-phase kernel against the 128x128 one; 0x1000 / 0x2000: the 64x64 / 32x32 ring tile
    const int large = (mode & 0x1000) ? GEMM_MID_FORCED : (mode & 0x2000) ? GEMM_MID32_FORCED : 8;
    mode &= 0xFF;
    try {
        OWK_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const int Tpad = (T + 63) / 64 * 64;
        const int clips = T > 0 ? (M + T - 1) / T : 1;
        const size_t n32 = (size_t) M * N, n16 = std::max((size_t) M * N, (size_t) clips * d * Tpad);
        DevBuf da, dw, bias, bias2, pos, gt, res[2], o32[2], o16[3][2];
        da.alloc((size_t) M * K * 2);
        dw.alloc((size_t) N * K * 2);
        bias.alloc((size_t) N * 4);
        bias2.alloc((size_t) N * 4);
        pos.alloc((size_t) std::max(T, 1) * N * 4);
        gt.alloc(65536 * 2);
        OWK_HIP_CHECK(hipMemcpy(gt.ptr, gelu_table_host().data(), 65536 * 2, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, da.as<_Float16>(), (size_t) M * K, 1u);
        hipLaunchKernelGGL(k_fill_rand_f16, dim3(4096), dim3(256), 0, s, dw.as<_Float16>(), (size_t) N * K, 7u);
        std::vector<float> hb(N), hb2(N), hp((size_t) std::max(T, 1) * N), hr(n32);
        uint32_t st = 12345u;
        auto rnd = [&] { st = st * 1664525u + 1013904223u; return (float) ((st >> 8) & 0xFFFF) / 65536.0f - 0.5f; };
        for (auto & v : hb) v = rnd();
        for (auto & v : hb2) v = rnd();
        for (auto & v : hp) v = rnd();
        for (auto & v : hr) v = rnd();
        OWK_HIP_CHECK(hipMemcpy(bias.ptr, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(bias2.ptr, hb2.data(), hb2.size() * 4, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(pos.ptr, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> out32[2];
        std::vector<uint16_t> out16[3][2];
        for (int k = 0; k < 2; ++k) {
            res[k].alloc(n32 * 4);
            o32[k].alloc(n32 * 4);
            OWK_HIP_CHECK(hipMemcpy(res[k].ptr, hr.data(), n32 * 4, hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemset(o32[k].ptr, 0, n32 * 4));
            for (int j = 0; j < 3; ++j) {
                o16[j][k].alloc(n16 * 2);
                OWK_HIP_CHECK(hipMemset(o16[j][k].ptr, 0, n16 * 2));
            }
            EpiParams ep;
            ep.bias = bias.as<float>();
            ep.bias2 = bias2.as<float>();
            ep.scale = 0.35f;
            ep.resid = res[k].as<float>();
            ep.out32 = o32[k].as<float>();
            ep.out16 = o16[0][k].as<_Float16>();
            ep.out16b = o16[1][k].as<_Float16>();
            ep.out16c = o16[2][k].as<_Float16>();
            ep.ldo = N;
            ep.d = d;
            ep.T = T;
            ep.Tpad = Tpad;
            ep.pos = pos.as<float>();
            ep.gelu_tab = gt.as<uint16_t>();
            if (mode == EPI_RESID_F32 || mode == EPI_HALF_RESID) ep.out32 = res[k].as<float>();  // in place, as the engine
            GemmOverride ov(k == 0 ? 0 : large);
            gemm_f16(s, mode, M, N, K, da.as<_Float16>(), K, dw.as<_Float16>(), K, ep);
            OWK_HIP_CHECK(hipStreamSynchronize(s));
            out32[k].resize(n32);
            OWK_HIP_CHECK(hipMemcpy(out32[k].data(), ep.out32, n32 * 4, hipMemcpyDeviceToHost));
            for (int j = 0; j < 3; ++j) {
                out16[j][k].resize(n16);
                OWK_HIP_CHECK(hipMemcpy(out16[j][k].data(), o16[j][k].ptr, n16 * 2, hipMemcpyDeviceToHost));
            }
        }
        double mx = 0.0;
        for (size_t i = 0; i < n32; ++i) mx = std::max(mx, (double) std::fabs(out32[0][i] - out32[1][i]));
        for (int j = 0; j < 3; ++j)
            for (size_t i = 0; i < n16; ++i) {
                const _Float16 a = __builtin_bit_cast(_Float16, out16[j][0][i]), b = __builtin_bit_cast(_Float16, out16[j][1][i]);
                mx = std::max(mx, (double) std::fabs((float) a - (float) b));
            }
        OWK_HIP_CHECK(hipStreamDestroy(s));
        return mx;
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_gemm_epi_diff: %s\n", ex.what());
        return -1;
    }
}

int owk_debug_gemm(int device, int M, int N, int K, const uint16_t * a, const uint16_t * w, float * out) {
    try {
        OWK_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        DevBuf da, dw, dout, part;
        da.alloc((size_t) M * K * 2);
        dw.alloc((size_t) N * K * 2);
        dout.alloc((size_t) M * N * 4);
        OWK_HIP_CHECK(hipMemcpy(da.ptr, a, (size_t) M * K * 2, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(dw.ptr, w, (size_t) N * K * 2, hipMemcpyHostToDevice));
        GemmWs ws;
        const size_t fl = gemm_ws_floats(N, K);
        part.alloc(std::max<size_t>(fl, 1) * 4);
        ws.partial = part.as<float>();
        ws.partial_floats = fl;
        EpiParams ep;
        ep.out32 = dout.as<float>();
        ep.ldo = N;
        DevBuf dwt;
        dwt.alloc(tiled_weight_elems(N, K) * 2);
        tile_weights(s, dw.as<_Float16>(), N, K, dwt.as<_Float16>());
        gemm(s, EPI_F32, M, N, K, da.as<_Float16>(), K, dw.as<_Float16>(), K, ep, &ws, dwt.as<_Float16>());
        // a second launch on the same workspace (results must not depend on its history)
        gemm(s, EPI_F32, M, N, K, da.as<_Float16>(), K, dw.as<_Float16>(), K, ep, &ws, dwt.as<_Float16>());
        OWK_HIP_CHECK(hipStreamSynchronize(s));
        OWK_HIP_CHECK(hipMemcpy(out, dout.ptr, (size_t) M * N * 4, hipMemcpyDeviceToHost));
        OWK_HIP_CHECK(hipStreamDestroy(s));
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_gemm: %s\n", ex.what());
        return -1;
    }
    return 0;
}

// The decoder's LayerNorm-prologue GEMM (gemm_rows_ln) against the two-launch form it replaces
// (layernorm_f16 -> f16 rows -> decode-row GEMM), EPI_F16 with bias b (may be null) and scale 1:
// x [M][K] f32, lnw / lnb [K], w [N][K] f16 bits; out_fused / out_ref [M][N] f16 bits. Also the
// residual epilogue over the whole K (EPI_RESID_F32 with K = 4 N, the mlp.2 shape) against the
// split-K partial + resid_layernorm finish: resid [M][N] f32 in, out_resid_* [M][N] f32 (may be null).
int owk_debug_gemm_rows_ln(int device, int M, int N, int K, const float * x, const float * lnw, const float * lnb,
                           const float * b, const uint16_t * w, uint16_t * out_fused, uint16_t * out_ref,
                           const uint16_t * w2, const float * resid, float * out_resid_full, float * out_resid_split) {
    try {
        OWK_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        DevBuf dx, dlw, dlb, db, dw, dwt, dxn, o1, o2, part;
        dx.alloc((size_t) M * K * 4);
        dlw.alloc((size_t) K * 4);
        dlb.alloc((size_t) K * 4);
        db.alloc((size_t) N * 4);
        dw.alloc((size_t) N * K * 2);
        dwt.alloc(tiled_weight_elems(N, K) * 2);
        dxn.alloc((size_t) M * K * 2);
        o1.alloc((size_t) M * N * 2);
        o2.alloc((size_t) M * N * 2);
        OWK_HIP_CHECK(hipMemcpy(dx.ptr, x, (size_t) M * K * 4, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(dlw.ptr, lnw, (size_t) K * 4, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(dlb.ptr, lnb, (size_t) K * 4, hipMemcpyHostToDevice));
        if (b) OWK_HIP_CHECK(hipMemcpy(db.ptr, b, (size_t) N * 4, hipMemcpyHostToDevice));
        OWK_HIP_CHECK(hipMemcpy(dw.ptr, w, (size_t) N * K * 2, hipMemcpyHostToDevice));
        tile_weights(s, dw.as<_Float16>(), N, K, dwt.as<_Float16>());
        EpiParams ep;
        ep.bias = b ? db.as<float>() : nullptr;
        ep.ldo = N;
        ep.out16 = o1.as<_Float16>();
        gemm_rows_ln(s, EPI_F16, M, N, K, dx.as<float>(), dlw.as<float>(), dlb.as<float>(), 1e-5f, dwt.as<_Float16>(), ep);
        layernorm_f16(s, dx.as<float>(), M, K, dlw.as<float>(), dlb.as<float>(), 1e-5f, dxn.as<_Float16>(), K, nullptr,
                      nullptr, nullptr, nullptr);
        ep.out16 = o2.as<_Float16>();
        GemmWs ws;
        const size_t fl = std::max(gemm_ws_floats(N, K), gemm_partial_floats(N, 4 * N));
        part.alloc(std::max<size_t>(fl, 1) * 4);
        ws.partial = part.as<float>();
        ws.partial_floats = fl;
        gemm(s, EPI_F16, M, N, K, dxn.as<_Float16>(), K, dw.as<_Float16>(), K, ep, &ws, dwt.as<_Float16>());
        if (w2 && resid) {
            // mlp.2 shape: [M][4N] f16 activations (the LayerNorm rows of x reused as data) x [N][4N]
            const int K2 = 4 * N;
            DevBuf dw2, dw2t, da2, r1, r2;
            dw2.alloc((size_t) N * K2 * 2);
            dw2t.alloc(tiled_weight_elems(N, K2) * 2);
            da2.alloc((size_t) M * K2 * 2);
            r1.alloc((size_t) M * N * 4);
            r2.alloc((size_t) M * N * 4);
            OWK_HIP_CHECK(hipMemcpy(dw2.ptr, w2, (size_t) N * K2 * 2, hipMemcpyHostToDevice));
            tile_weights(s, dw2.as<_Float16>(), N, K2, dw2t.as<_Float16>());
            std::vector<uint16_t> a2((size_t) M * K2);
            for (size_t i = 0; i < a2.size(); ++i) a2[i] = w2[(i * 7919) % ((size_t) N * K2)];
            OWK_HIP_CHECK(hipMemcpy(da2.ptr, a2.data(), a2.size() * 2, hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemcpy(r1.ptr, resid, (size_t) M * N * 4, hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemcpy(r2.ptr, resid, (size_t) M * N * 4, hipMemcpyHostToDevice));
            EpiParams e2;
            e2.bias = db.as<float>();
            e2.resid = r1.as<float>();
            e2.out32 = r1.as<float>();
            e2.ldo = N;
            gemm(s, EPI_RESID_F32, M, N, K2, da2.as<_Float16>(), K2, dw2.as<_Float16>(), K2, e2, &ws, dw2t.as<_Float16>());
            EpiParams e3;
            gemm(s, EPI_PARTIAL, M, N, K2, da2.as<_Float16>(), K2, nullptr, K2, e3, &ws, dw2t.as<_Float16>());
            resid_layernorm(s, M, N, gemm_partial_splits(K2), ws.partial, db.as<float>(), r2.as<float>(), nullptr,
                            nullptr, 1e-5f, nullptr, N);
            OWK_HIP_CHECK(hipStreamSynchronize(s));
            if (out_resid_full) OWK_HIP_CHECK(hipMemcpy(out_resid_full, r1.ptr, (size_t) M * N * 4, hipMemcpyDeviceToHost));
            if (out_resid_split) OWK_HIP_CHECK(hipMemcpy(out_resid_split, r2.ptr, (size_t) M * N * 4, hipMemcpyDeviceToHost));
        }
        OWK_HIP_CHECK(hipStreamSynchronize(s));
        OWK_HIP_CHECK(hipMemcpy(out_fused, o1.ptr, (size_t) M * N * 2, hipMemcpyDeviceToHost));
        OWK_HIP_CHECK(hipMemcpy(out_ref, o2.ptr, (size_t) M * N * 2, hipMemcpyDeviceToHost));
        OWK_HIP_CHECK(hipStreamDestroy(s));
    } catch (const std::exception & ex) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_debug_gemm_rows_ln: %s\n", ex.what());
        return -1;
    }
    return 0;
}

// test hook: decode passes of at most n rows take the whole-K chain (engine.cpp; 0 = never); returns
// the previous limit. Both chains must give the same bits (tests/test_gpu_kernels.py).
int owk_debug_set_whole_k_rows(int n) { return set_whole_k_rows(n); }

}  // extern "C"
