// ggml-bin model loader for the MI355X engine.
//
// Reads exactly the file format of the reference loader (whisper_model_load,
// ref src/whisper.cpp:1485-1956; tensor names src/whisper-arch.h:42-106) and packs
// the weights for the GEMM kernels in one device allocation:
//   - attention q/k/v weights concatenated into one [3d][d] matrix per layer (one GEMM)
//   - cross-attention k/v concatenated into [2d][d] per decoder layer
//   - conv1 weight [d][n_mels*3] zero-padded along K to a multiple of 64
// plus device constants: the f16 GELU table, mel filterbank, DFT twiddles, Hann window.
#include "model.h"
#include "kernels.h"
#include "kquant.h"

#include <cmath>
#include <cstdarg>
#include <cstring>
#include <memory>
#include <mutex>
#include <regex>

namespace owk {

static ggml_log_callback g_log_cb = nullptr;
static void * g_log_ud = nullptr;

void set_log_callback(ggml_log_callback cb, void * ud) {
    g_log_cb = cb;
    g_log_ud = ud;
}

void log_msg(ggml_log_level level, const char * fmt, ...) {
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (g_log_cb) {
        g_log_cb(level, buf, g_log_ud);
    } else if (level != GGML_LOG_LEVEL_DEBUG) {  // whisper_log_callback_default (ref whisper.cpp:9028-9038)
        fputs(buf, stderr);
        fflush(stderr);
    }
}

const std::map<std::string, std::pair<int, std::string>> & languages() {
    static const char * tab[][2] = {
        {"en", "english"}, {"zh", "chinese"}, {"de", "german"}, {"es", "spanish"}, {"ru", "russian"},
        {"ko", "korean"}, {"fr", "french"}, {"ja", "japanese"}, {"pt", "portuguese"}, {"tr", "turkish"},
        {"pl", "polish"}, {"ca", "catalan"}, {"nl", "dutch"}, {"ar", "arabic"}, {"sv", "swedish"},
        {"it", "italian"}, {"id", "indonesian"}, {"hi", "hindi"}, {"fi", "finnish"}, {"vi", "vietnamese"},
        {"he", "hebrew"}, {"uk", "ukrainian"}, {"el", "greek"}, {"ms", "malay"}, {"cs", "czech"},
        {"ro", "romanian"}, {"da", "danish"}, {"hu", "hungarian"}, {"ta", "tamil"}, {"no", "norwegian"},
        {"th", "thai"}, {"ur", "urdu"}, {"hr", "croatian"}, {"bg", "bulgarian"}, {"lt", "lithuanian"},
        {"la", "latin"}, {"mi", "maori"}, {"ml", "malayalam"}, {"cy", "welsh"}, {"sk", "slovak"},
        {"te", "telugu"}, {"fa", "persian"}, {"lv", "latvian"}, {"bn", "bengali"}, {"sr", "serbian"},
        {"az", "azerbaijani"}, {"sl", "slovenian"}, {"kn", "kannada"}, {"et", "estonian"}, {"mk", "macedonian"},
        {"br", "breton"}, {"eu", "basque"}, {"is", "icelandic"}, {"hy", "armenian"}, {"ne", "nepali"},
        {"mn", "mongolian"}, {"bs", "bosnian"}, {"kk", "kazakh"}, {"sq", "albanian"}, {"sw", "swahili"},
        {"gl", "galician"}, {"mr", "marathi"}, {"pa", "punjabi"}, {"si", "sinhala"}, {"km", "khmer"},
        {"sn", "shona"}, {"yo", "yoruba"}, {"so", "somali"}, {"af", "afrikaans"}, {"oc", "occitan"},
        {"ka", "georgian"}, {"be", "belarusian"}, {"tg", "tajik"}, {"sd", "sindhi"}, {"gu", "gujarati"},
        {"am", "amharic"}, {"yi", "yiddish"}, {"lo", "lao"}, {"uz", "uzbek"}, {"fo", "faroese"},
        {"ht", "haitian creole"}, {"ps", "pashto"}, {"tk", "turkmen"}, {"nn", "nynorsk"}, {"mt", "maltese"},
        {"sa", "sanskrit"}, {"lb", "luxembourgish"}, {"my", "myanmar"}, {"bo", "tibetan"}, {"tl", "tagalog"},
        {"mg", "malagasy"}, {"as", "assamese"}, {"tt", "tatar"}, {"haw", "hawaiian"}, {"ln", "lingala"},
        {"ha", "hausa"}, {"ba", "bashkir"}, {"jw", "javanese"}, {"su", "sundanese"}, {"yue", "cantonese"},
    };
    static std::map<std::string, std::pair<int, std::string>> m;
    static std::once_flag once;
    std::call_once(once, [] {
        for (int i = 0; i < (int) (sizeof(tab) / sizeof(tab[0])); ++i) m[tab[i][0]] = {i, tab[i][1]};
    });
    return m;
}

// ---------------------------------------------------------------------------------
// GELU table: ggml_table_gelu_f16[i] = fp16(gelu_f32(fp32(i))) with
// gelu_f32(x) = 0.5*x*(1 + tanh(sqrt(2/pi)*x*(1 + 0.044715*x^2)))  (ggml-cpu/vec.h:975-977).
// The reference build (gcc, GNU mode, FMA ISA) contracts 1 + a*x*x into one fma; the
// same contraction is written explicitly here (pinned by tests/test_oracle_pin.py).
// ---------------------------------------------------------------------------------
static void build_gelu_table(std::vector<uint16_t> & tab) {
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    tab.resize(65536);
    for (int i = 0; i < 65536; ++i) {
        const float x = f16_to_f32_host((uint16_t) i);
        const float inner = fmaf(GELU_COEF_A * x, x, 1.0f);
        const float g = 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * inner));
        tab[i] = f32_to_f16_host(g);
    }
}

const std::vector<uint16_t> & gelu_table_host() {
    static std::vector<uint16_t> tab;
    static std::once_flag once;
    std::call_once(once, [] { build_gelu_table(tab); });
    return tab;
}

namespace {

struct Reader {
    whisper_model_loader * l;
    bool ok = true;
    void read(void * dst, size_t n) {
        if (!ok) return;
        if (l->read(l->context, dst, n) != n) ok = false;
    }
    template <typename T> T get() {
        T v{};
        read(&v, sizeof(T));
        return v;
    }
};

struct TensorSpec {
    std::string name;
    std::vector<int64_t> ne;  // ggml order (ne[0] innermost)
    bool f16;                 // expected storage type in an F16 model
};

std::vector<TensorSpec> expected_tensors(const HParams & hp) {
    const int64_t d = hp.n_audio_state, dt = hp.n_text_state;
    std::vector<TensorSpec> t;
    auto add = [&](const std::string & n, std::vector<int64_t> ne, bool f16) { t.push_back({n, ne, f16}); };
    add("encoder.positional_embedding", {d, hp.n_audio_ctx}, false);
    add("encoder.conv1.weight", {3, hp.n_mels, d}, true);
    add("encoder.conv1.bias", {1, d}, false);
    add("encoder.conv2.weight", {3, d, d}, true);
    add("encoder.conv2.bias", {1, d}, false);
    add("encoder.ln_post.weight", {d}, false);
    add("encoder.ln_post.bias", {d}, false);
    for (int i = 0; i < hp.n_audio_layer; ++i) {
        const std::string p = "encoder.blocks." + std::to_string(i) + ".";
        add(p + "mlp_ln.weight", {d}, false);
        add(p + "mlp_ln.bias", {d}, false);
        add(p + "mlp.0.weight", {d, 4 * d}, true);
        add(p + "mlp.0.bias", {4 * d}, false);
        add(p + "mlp.2.weight", {4 * d, d}, true);
        add(p + "mlp.2.bias", {d}, false);
        add(p + "attn_ln.weight", {d}, false);
        add(p + "attn_ln.bias", {d}, false);
        add(p + "attn.query.weight", {d, d}, true);
        add(p + "attn.query.bias", {d}, false);
        add(p + "attn.key.weight", {d, d}, true);
        add(p + "attn.value.weight", {d, d}, true);
        add(p + "attn.value.bias", {d}, false);
        add(p + "attn.out.weight", {d, d}, true);
        add(p + "attn.out.bias", {d}, false);
    }
    add("decoder.positional_embedding", {dt, hp.n_text_ctx}, false);
    add("decoder.token_embedding.weight", {dt, hp.n_vocab}, true);
    add("decoder.ln.weight", {dt}, false);
    add("decoder.ln.bias", {dt}, false);
    for (int i = 0; i < hp.n_text_layer; ++i) {
        const std::string p = "decoder.blocks." + std::to_string(i) + ".";
        add(p + "mlp_ln.weight", {dt}, false);
        add(p + "mlp_ln.bias", {dt}, false);
        add(p + "mlp.0.weight", {dt, 4 * dt}, true);
        add(p + "mlp.0.bias", {4 * dt}, false);
        add(p + "mlp.2.weight", {4 * dt, dt}, true);
        add(p + "mlp.2.bias", {dt}, false);
        for (const char * a : {"attn", "cross_attn"}) {
            const std::string q = p + a;
            add(q + "_ln.weight", {dt}, false);
            add(q + "_ln.bias", {dt}, false);
            add(q + ".query.weight", {dt, dt}, true);
            add(q + ".query.bias", {dt}, false);
            add(q + ".key.weight", {dt, dt}, true);
            add(q + ".value.weight", {dt, dt}, true);
            add(q + ".value.bias", {dt}, false);
            add(q + ".out.weight", {dt, dt}, true);
            add(q + ".out.bias", {dt}, false);
        }
    }
    return t;
}

struct HostTensor {
    std::vector<uint8_t> data;  // raw bytes as stored
    bool f16 = false;
    bool q5 = false;            // block_q5_0 rows
    bool loaded = false;
    int64_t nelem = 0;
};

} // namespace

Model * load_model(whisper_model_loader * loader, int device, std::string & err, bool vocab_only) {
    Reader r{loader};
    auto m = std::make_unique<Model>();
    m->device = device;
    HParams & hp = m->hp;

    if (r.get<uint32_t>() != 0x67676d6c) { err = "invalid model data (bad magic)"; return nullptr; }
    hp.n_vocab = r.get<int32_t>();
    hp.n_audio_ctx = r.get<int32_t>();
    hp.n_audio_state = r.get<int32_t>();
    hp.n_audio_head = r.get<int32_t>();
    hp.n_audio_layer = r.get<int32_t>();
    hp.n_text_ctx = r.get<int32_t>();
    hp.n_text_state = r.get<int32_t>();
    hp.n_text_head = r.get<int32_t>();
    hp.n_text_layer = r.get<int32_t>();
    hp.n_mels = r.get<int32_t>();
    hp.ftype = r.get<int32_t>();
    if (!r.ok) { err = "truncated header"; return nullptr; }
    if (hp.n_audio_state != hp.n_text_state || hp.n_audio_state % 64 || hp.n_audio_state / hp.n_audio_head != 64 ||
        hp.n_text_state / hp.n_text_head != 64) {
        err = "unsupported hyper-parameters (head dim must be 64)";
        return nullptr;
    }
    switch (hp.n_audio_layer) {
        case 4: m->type = MODEL_TINY; break;
        case 6: m->type = MODEL_BASE; break;
        case 12: m->type = MODEL_SMALL; break;
        case 24: m->type = MODEL_MEDIUM; break;
        case 32: m->type = MODEL_LARGE; break;
        default: m->type = MODEL_UNKNOWN;
    }
    const int qntvr = hp.ftype / 1000;
    (void) qntvr;
    hp.ftype %= 1000;
    // GGML_FTYPE_MOSTLY_F16 (1), MOSTLY_Q4_0 (2), MOSTLY_Q4_1 (3), MOSTLY_Q8_0 (7), MOSTLY_Q5_0 (8),
    // MOSTLY_Q5_1 (9) (ggml.h:440-450)
    switch (hp.ftype) {
        case 1: break;
        case 2: m->qfmt = QF_Q4_0; break;
        case 3: m->qfmt = QF_Q4_1; break;
        case 7: m->qfmt = QF_Q8_0; break;
        case 8: m->qfmt = QF_Q5_0; break;
        case 9: m->qfmt = QF_Q5_1; break;
        // MOSTLY_Q2_K .. Q6_K (10-14): 256-weight super-blocks x Q8_K activations (kquant.h)
        case 10: m->qfmt = QF_Q2_K; break;
        case 11: m->qfmt = QF_Q3_K; break;
        case 12: m->qfmt = QF_Q4_K; break;
        case 13: m->qfmt = QF_Q5_K; break;
        case 14: m->qfmt = QF_Q6_K; break;
        default:
            err = "unsupported ftype " + std::to_string(hp.ftype) +
                  " (this engine build loads F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0 and Q2_K-Q6_K models)";
            return nullptr;
    }
    m->q5 = hp.ftype != 1;  // quantized weights x Q8_0 / Q8_1 / Q8_K activations
    m->kq = qf_is_k(m->qfmt) && m->q5;

    // mel filters
    m->n_filters_mel = r.get<int32_t>();
    m->n_filters_fft = r.get<int32_t>();
    if (m->n_filters_fft != 201 || m->n_filters_mel <= 0 || m->n_filters_mel > 512) { err = "bad mel filters"; return nullptr; }
    m->filters.resize((size_t) m->n_filters_mel * m->n_filters_fft);
    r.read(m->filters.data(), m->filters.size() * sizeof(float));

    // vocab (ref 1589-1675)
    Vocab & v = m->vocab;
    const int32_t n_vocab_file = r.get<int32_t>();
    if (!r.ok || n_vocab_file < 0 || n_vocab_file > hp.n_vocab) { err = "bad vocab"; return nullptr; }
    v.id_to_token.resize(std::max<int>(hp.n_vocab, n_vocab_file));
    std::string word;
    for (int i = 0; i < n_vocab_file; ++i) {
        const uint32_t len = r.get<uint32_t>();
        if (!r.ok || len > (1u << 20)) { err = "bad vocab entry"; return nullptr; }
        word.assign(len, '\0');
        if (len) r.read(&word[0], len);
        v.token_to_id[word] = i;
        v.id_to_token[i] = word;
    }
    v.n_vocab = hp.n_vocab;
    if (v.is_multilingual()) {
        v.eot++;
        v.sot++;
        const int dt = v.num_languages() - 98;
        v.translate += dt; v.transcribe += dt; v.solm += dt; v.prev += dt; v.nosp += dt; v.not_ += dt; v.beg += dt;
    }
    if (n_vocab_file < hp.n_vocab) {
        // reverse map of language ids for the synthesized "[_LANG_xx]" names
        std::vector<std::string> lang_code(200);
        for (const auto & kv : languages()) lang_code[kv.second.first] = kv.first;
        for (int i = n_vocab_file; i < hp.n_vocab; ++i) {
            if (i > v.beg) word = "[_TT_" + std::to_string(i - v.beg) + "]";
            else if (i == v.eot) word = "[_EOT_]";
            else if (i == v.sot) word = "[_SOT_]";
            else if (i == v.translate) word = "[_TRANSLATE_]";
            else if (i == v.transcribe) word = "[_TRANSCRIBE_]";
            else if (i == v.solm) word = "[_SOLM_]";
            else if (i == v.prev) word = "[_PREV_]";
            else if (i == v.nosp) word = "[_NOSP_]";
            else if (i == v.not_) word = "[_NOT_]";
            else if (i == v.beg) word = "[_BEG_]";
            else if (i > v.sot && i <= v.sot + v.num_languages()) {
                const int lid = i - v.sot - 1;
                word = "[_LANG_" + (lid < (int) lang_code.size() ? lang_code[lid] : std::string("")) + "]";
            } else word = "[_extra_token_" + std::to_string(i) + "]";
            v.token_to_id[word] = i;
            v.id_to_token[i] = word;
        }
    }
    if (!r.ok) { err = "truncated vocab"; return nullptr; }
    if (vocab_only) return m.release();

    // tensors
    const auto specs = expected_tensors(hp);
    std::map<std::string, size_t> idx;
    for (size_t i = 0; i < specs.size(); ++i) idx[specs[i].name] = i;
    std::vector<HostTensor> ht(specs.size());
    int n_loaded = 0;
    for (;;) {
        int32_t n_dims = 0, name_len = 0, ttype = 0;
        r.read(&n_dims, 4);
        r.read(&name_len, 4);
        r.read(&ttype, 4);
        if (!r.ok || loader->eof(loader->context)) break;
        if (n_dims < 1 || n_dims > 4 || name_len <= 0 || name_len > 512) { err = "bad tensor header"; return nullptr; }
        int64_t ne[4] = {1, 1, 1, 1}, nel = 1;
        for (int i = 0; i < n_dims; ++i) { ne[i] = r.get<int32_t>(); nel *= ne[i]; }
        std::string name(name_len, '\0');
        r.read(&name[0], name_len);
        auto it = idx.find(name);
        if (it == idx.end()) { err = "unknown tensor '" + name + "' in model file"; return nullptr; }
        const TensorSpec & sp = specs[it->second];
        int64_t expect = 1;
        for (auto e : sp.ne) expect *= e;
        for (size_t i = 0; i < sp.ne.size(); ++i)
            if (ne[i] != sp.ne[i]) { err = "tensor '" + name + "' has wrong shape in model file"; return nullptr; }
        if (nel != expect) { err = "tensor '" + name + "' has wrong size in model file"; return nullptr; }
        // quantized models: every 2-D weight is of the model's block type (whisper-quantize)
        const bool want_q5 = m->q5 && sp.f16 && sp.ne.size() == 2;
        const int qtype = !m->q5 ? -1 : m->kq ? kq_ggml_type(m->qfmt) : qf_ggml_type(m->qfmt);
        const int qblk = m->kq ? 256 : 32, qbytes = !m->q5 ? 0 : m->kq ? kq_block_bytes(m->qfmt) : qf_block_bytes(m->qfmt);
        if (want_q5 ? ttype != qtype : (ttype != 0 && ttype != 1)) {
            err = "tensor '" + name + "': unsupported type " + std::to_string(ttype);
            return nullptr;
        }
        if (sp.f16 && !want_q5 && ttype != 1) { err = "tensor '" + name + "': expected F16 weights"; return nullptr; }
        if (want_q5 && sp.ne[0] % qblk) {
            err = "tensor '" + name + "': row length not a multiple of " + std::to_string(qblk);
            return nullptr;
        }
        HostTensor & t = ht[it->second];
        t.f16 = ttype == 1;
        t.q5 = want_q5;
        t.nelem = nel;
        t.data.resize(want_q5 ? (size_t) nel / qblk * qbytes : (size_t) nel * (t.f16 ? 2 : 4));
        r.read(t.data.data(), t.data.size());
        if (!r.ok) { err = "truncated tensor data for '" + name + "'"; return nullptr; }
        t.loaded = true;
        ++n_loaded;
    }
    m->n_loaded = n_loaded;
    if (n_loaded == 0) {
        log_msg(GGML_LOG_LEVEL_WARN, "whisper_model_load: WARN no tensors loaded from model file - assuming empty model for testing\n");
    } else if (n_loaded != (int) specs.size()) {
        err = "not all tensors loaded from model file - expected " + std::to_string(specs.size()) + ", got " +
              std::to_string(n_loaded);
        return nullptr;
    }

    // ---- device packing ----
    OWK_HIP_CHECK(hipSetDevice(device));
    const int64_t d = hp.n_audio_state;
    m->kpad_conv1 = (int) (((3 * hp.n_mels) + 63) / 64 * 64);

    // layout plan: (offset, bytes) per packed item, 256-byte aligned
    size_t off = 0;
    auto reserve = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t) 255; return o; };
    const auto & S = specs;
    auto bytes_of = [&](const std::string & n) {
        const TensorSpec & sp = S[idx.at(n)];
        int64_t e = 1;
        for (auto x : sp.ne) e *= x;
        return (size_t) e * (sp.f16 ? 2 : 4);
    };
    std::map<std::string, size_t> place;  // simple tensors -> offset
    for (const auto & sp : S) place[sp.name] = 0;
    // packed matrices
    const size_t o_conv1 = reserve((size_t) d * m->kpad_conv1 * 2);
    std::vector<size_t> o_enc_qkv(hp.n_audio_layer), o_dec_qkv(hp.n_text_layer), o_dec_ckv(hp.n_text_layer);
    if (!m->q5) {
        for (int i = 0; i < hp.n_audio_layer; ++i) o_enc_qkv[i] = reserve((size_t) 3 * d * d * 2);
        for (int i = 0; i < hp.n_text_layer; ++i) {
            o_dec_qkv[i] = reserve((size_t) 3 * d * d * 2);
            o_dec_ckv[i] = reserve((size_t) 2 * d * d * 2);
        }
    }
    auto is_q5 = [&](const std::string & n) {
        const TensorSpec & sp = S[idx.at(n)];
        return m->q5 && sp.f16 && sp.ne.size() == 2;
    };
    for (auto & kv : place) {
        const std::string & n = kv.first;
        const bool packed = n == "encoder.conv1.weight" ||
                            (n.find(".key.weight") != std::string::npos) ||
                            (n.find(".value.weight") != std::string::npos) ||
                            (n.find("attn.query.weight") != std::string::npos && n.find("cross_attn") == std::string::npos);
        kv.second = (packed || is_q5(n)) ? (size_t) -1 : reserve(bytes_of(n));
    }
    const size_t o_gelu = reserve(65536 * 2);
    const size_t o_filt = reserve(m->filters.size() * 4);
    const size_t o_tw = reserve(800 * 8);
    const size_t o_hann = reserve(400 * 4);
    const int n_filt = (int) (m->filters.size() / 201);
    const size_t o_rng = reserve((size_t) n_filt * 2 * 4);

    m->blob.alloc(off);
    OWK_HIP_CHECK(hipMemset(m->blob.ptr, 0, off));
    char * base = (char *) m->blob.ptr;
    auto up = [&](size_t o, const void * src, size_t n) { OWK_HIP_CHECK(hipMemcpy(base + o, src, n, hipMemcpyHostToDevice)); };
    auto host = [&](const std::string & n) -> const HostTensor & { return ht[idx.at(n)]; };

    if (n_loaded > 0) {
        for (const auto & kv : place)
            if (kv.second != (size_t) -1) up(kv.second, host(kv.first).data.data(), host(kv.first).data.size());
        // conv1 [d][n_mels][3] -> [d][kpad]
        {
            const HostTensor & t = host("encoder.conv1.weight");
            std::vector<uint16_t> p((size_t) d * m->kpad_conv1, 0);
            const uint16_t * src = (const uint16_t *) t.data.data();
            for (int64_t o = 0; o < d; ++o)
                memcpy(&p[(size_t) o * m->kpad_conv1], src + (size_t) o * 3 * hp.n_mels, (size_t) 3 * hp.n_mels * 2);
            up(o_conv1, p.data(), p.size() * 2);
        }
        auto cat = [&](size_t o, std::initializer_list<std::string> parts) {
            size_t at = o;
            for (const auto & n : parts) {
                const HostTensor & t = host(n);
                up(at, t.data.data(), t.data.size());
                at += t.data.size();
            }
        };
        for (int i = 0; i < hp.n_audio_layer && !m->q5; ++i) {
            const std::string p = "encoder.blocks." + std::to_string(i) + ".attn.";
            cat(o_enc_qkv[i], {p + "query.weight", p + "key.weight", p + "value.weight"});
        }
        for (int i = 0; i < hp.n_text_layer && !m->q5; ++i) {
            const std::string p = "decoder.blocks." + std::to_string(i) + ".";
            cat(o_dec_qkv[i], {p + "attn.query.weight", p + "attn.key.weight", p + "attn.value.weight"});
            cat(o_dec_ckv[i], {p + "cross_attn.key.weight", p + "cross_attn.value.weight"});
        }
    }
    up(o_gelu, gelu_table_host().data(), 65536 * 2);
    up(o_filt, m->filters.data(), m->filters.size() * 4);
    {
        // twiddles for the 400-point DFT (double) and the periodic Hann window computed like
        // whisper_global_cache::fill_hann_window (whisper.cpp:3023-3031): float cosf of a
        // double argument, 0.5*(1-c) in double, stored as float.
        std::vector<double> tw(800);
        for (int i = 0; i < 400; ++i) {
            const double th = 2.0 * M_PI * i / 400.0;
            tw[i] = cos(th);
            tw[400 + i] = sin(th);
        }
        up(o_tw, tw.data(), tw.size() * 8);
        std::vector<float> hann(400);
        for (int i = 0; i < 400; ++i) hann[i] = (float) (0.5 * (1.0 - cosf((float) ((2.0 * M_PI * i) / (400 + 0)))));
        up(o_hann, hann.data(), hann.size() * 4);
        // each mel filter's nonzero bin range [lo, hi): the projection skips the zero weights around it
        // (power * 0 adds an exact 0 to the double sum, so the result is unchanged)
        std::vector<int> rng((size_t) n_filt * 2);
        for (int f = 0; f < n_filt; ++f) {
            const float * fr = m->filters.data() + (size_t) f * 201;
            int lo = 0, hi = 201;
            while (lo < hi && fr[lo] == 0.0f) ++lo;
            while (hi > lo && fr[hi - 1] == 0.0f) --hi;
            rng[2 * f] = lo;
            rng[2 * f + 1] = hi;
        }
        up(o_rng, rng.data(), rng.size() * 4);
    }

    auto F = [&](const std::string & n) { return (const float *) (base + place.at(n)); };
    auto H = [&](const std::string & n) -> const _Float16 * {
        return place.at(n) == (size_t) -1 ? nullptr : (const _Float16 *) (base + place.at(n));
    };
    // Q5_0 matrices: split block arrays (kernels.h Q5W), row groups concatenated like the F16 packs
    std::map<std::string, Q5W> q5m;
    if (m->kq && n_loaded > 0) {
        // K-quants: every 2-D linear (row groups concatenated like the F16 packs) as the virtual-block
        // f16 integers + scales of kquant.h, the one layout every GEMM shape runs on (gemm_q16)
        std::vector<std::vector<std::string>> groups;
        groups.push_back({"decoder.token_embedding.weight"});
        for (int i = 0; i < hp.n_audio_layer; ++i) {
            const std::string p = "encoder.blocks." + std::to_string(i) + ".";
            groups.push_back({p + "attn.query.weight", p + "attn.key.weight", p + "attn.value.weight"});
            for (const char * n : {"attn.out.weight", "mlp.0.weight", "mlp.2.weight"}) groups.push_back({p + n});
        }
        for (int i = 0; i < hp.n_text_layer; ++i) {
            const std::string p = "decoder.blocks." + std::to_string(i) + ".";
            groups.push_back({p + "attn.query.weight", p + "attn.key.weight", p + "attn.value.weight"});
            groups.push_back({p + "cross_attn.key.weight", p + "cross_attn.value.weight"});
            for (const char * n : {"attn.out.weight", "cross_attn.query.weight", "cross_attn.out.weight", "mlp.0.weight",
                                   "mlp.2.weight"})
                groups.push_back({p + n});
        }
        const int f = m->qfmt;
        auto al = [](size_t b) { return (b + 255) & ~(size_t) 255; };
        struct KPlan { int N, K, kx, npad; size_t wi, dwt; };
        std::vector<KPlan> kp;
        size_t tot = 0;
        for (const auto & gr : groups) {
            KPlan pl{0, (int) S[idx.at(gr[0])].ne[0], 0, 0, 0, 0};
            for (const auto & n : gr) pl.N += (int) S[idx.at(n)].ne[1];
            pl.kx = kq_kx(f, pl.K);
            pl.npad = (pl.N + 255) / 256 * 256;
            pl.wi = tot;
            tot += al((size_t) pl.N * pl.kx * 2);
            pl.dwt = tot;
            tot += al((size_t) (pl.kx / 32) * pl.npad * 4);
            kp.push_back(pl);
        }
        m->q16blob.alloc(tot);
        char * b16 = (char *) m->q16blob.ptr;
        for (size_t gi = 0; gi < groups.size(); ++gi) {
            const KPlan & pl = kp[gi];
            std::vector<uint8_t> raw;
            for (const auto & n : groups[gi]) raw.insert(raw.end(), host(n).data.begin(), host(n).data.end());
            std::vector<uint16_t> wi((size_t) pl.N * pl.kx);
            std::vector<float> dwt((size_t) (pl.kx / 32) * pl.npad);
            kq_expand_host(f, raw.data(), pl.N, pl.K, wi.data(), dwt.data(), pl.npad);
            OWK_HIP_CHECK(hipMemcpy(b16 + pl.wi, wi.data(), wi.size() * 2, hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemcpy(b16 + pl.dwt, dwt.data(), dwt.size() * 4, hipMemcpyHostToDevice));
            Q5W w;
            w.fmt = f;
            w.wi = (const _Float16 *) (b16 + pl.wi);
            w.dwt = (const float *) (b16 + pl.dwt);
            w.npad = pl.npad;
            w.kx = pl.kx;
            q5m[groups[gi][0]] = w;
        }
        // token embedding rows for get_rows: the reference dequantizes them to f32 (ggml get_rows)
        {
            const HostTensor & t = host("decoder.token_embedding.weight");
            const int nv = (int) hp.n_vocab, dd = (int) d;
            const size_t rb = (size_t) dd / 256 * kq_block_bytes(f);
            std::vector<float> te((size_t) nv * dd);
            for (int v = 0; v < nv; ++v) kq_dequant_row_host(f, t.data.data() + (size_t) v * rb, dd, te.data() + (size_t) v * dd);
            m->te32.alloc(te.size() * 4);
            OWK_HIP_CHECK(hipMemcpy(m->te32.ptr, te.data(), te.size() * 4, hipMemcpyHostToDevice));
        }
    }
    if (m->q5 && !m->kq && n_loaded > 0) {
        std::vector<std::vector<std::string>> groups;
        groups.push_back({"decoder.token_embedding.weight"});
        const size_t n_dec_first = 0;  // token embedding: a decode (logits) matrix too
        for (int i = 0; i < hp.n_audio_layer; ++i) {
            const std::string p = "encoder.blocks." + std::to_string(i) + ".";
            groups.push_back({p + "attn.query.weight", p + "attn.key.weight", p + "attn.value.weight"});
            for (const char * n : {"attn.out.weight", "mlp.0.weight", "mlp.2.weight"}) groups.push_back({p + n});
        }
        for (int i = 0; i < hp.n_text_layer; ++i) {
            const std::string p = "decoder.blocks." + std::to_string(i) + ".";
            groups.push_back({p + "attn.query.weight", p + "attn.key.weight", p + "attn.value.weight"});
            groups.push_back({p + "cross_attn.key.weight", p + "cross_attn.value.weight"});
            for (const char * n : {"attn.out.weight", "cross_attn.query.weight", "cross_attn.out.weight", "mlp.0.weight",
                                   "mlp.2.weight"})
                groups.push_back({p + n});
        }
        const size_t n_enc_groups = 1 + 4 * (size_t) hp.n_audio_layer;  // groups [1, n_enc_groups): encoder
        size_t qoff = 0;
        struct Plan { size_t qs, qh, d, m, tiled; int N, K; };
        std::vector<Plan> plans;
        for (size_t gi = 0; gi < groups.size(); ++gi) {
            const auto & gr = groups[gi];
            int N = 0;
            const int K = (int) S[idx.at(gr[0])].ne[0];
            for (const auto & n : gr) N += (int) S[idx.at(n)].ne[1];
            Plan pl{0, 0, 0, 0, (size_t) -1, N, K};
            auto res = [&](size_t bytes) { size_t o = qoff; qoff += (bytes + 255) & ~(size_t) 255; return o; };
            const int f = m->qfmt;
            pl.qs = res((size_t) N * (K / 32) * qf_qs_bytes(f));
            pl.qh = qf_has_qh(f) ? res((size_t) N * (K / 32) * 4) : 0;
            pl.d = res((size_t) N * (K / 32) * 2);
            pl.m = qf_has_m(f) ? res((size_t) N * (K / 32) * 2) : 0;
            // decode-step matrices also get the column-tiled copy the decode-row GEMM streams
            if (gi == n_dec_first || gi >= n_enc_groups) pl.tiled = res(quant_tiled_bytes(f, N, K));
            plans.push_back(pl);
        }
        m->q5blob.alloc(qoff);
        char * qb = (char *) m->q5blob.ptr;
        const int f = m->qfmt;
        for (size_t gi = 0; gi < groups.size(); ++gi) {
            const Plan & pl = plans[gi];
            const size_t nbk = (size_t) pl.N * (pl.K / 32);
            std::vector<uint8_t> qs(nbk * qf_qs_bytes(f));
            std::vector<uint32_t> qh(qf_has_qh(f) ? nbk : 0);
            std::vector<uint16_t> dd(nbk), mm(qf_has_m(f) ? nbk : 0);
            size_t row = 0;
            for (const auto & n : groups[gi]) {
                const HostTensor & t = host(n);
                const int rows = (int) S[idx.at(n)].ne[1];
                const size_t b0 = row * (pl.K / 32);
                quant_split_host(f, t.data.data(), rows, pl.K, qs.data() + b0 * qf_qs_bytes(f),
                                 qh.empty() ? nullptr : qh.data() + b0, dd.data() + b0, mm.empty() ? nullptr : mm.data() + b0);
                row += rows;
            }
            OWK_HIP_CHECK(hipMemcpy(qb + pl.qs, qs.data(), qs.size(), hipMemcpyHostToDevice));
            OWK_HIP_CHECK(hipMemcpy(qb + pl.d, dd.data(), dd.size() * 2, hipMemcpyHostToDevice));
            if (!qh.empty()) OWK_HIP_CHECK(hipMemcpy(qb + pl.qh, qh.data(), qh.size() * 4, hipMemcpyHostToDevice));
            if (!mm.empty()) OWK_HIP_CHECK(hipMemcpy(qb + pl.m, mm.data(), mm.size() * 2, hipMemcpyHostToDevice));
            Q5W w;
            w.fmt = f;
            w.qs = (const uint8_t *) (qb + pl.qs);
            w.d = (const _Float16 *) (qb + pl.d);
            if (!qh.empty()) w.qh = (const uint32_t *) (qb + pl.qh);
            if (!mm.empty()) w.m = (const _Float16 *) (qb + pl.m);
            if (pl.tiled != (size_t) -1) {
                std::vector<uint8_t> tl(quant_tiled_bytes(f, pl.N, pl.K));
                quant_tile_host(f, qs.data(), qh.empty() ? nullptr : qh.data(), dd.data(), mm.empty() ? nullptr : mm.data(),
                                pl.N, pl.K, tl.data());
                OWK_HIP_CHECK(hipMemcpy(qb + pl.tiled, tl.data(), tl.size(), hipMemcpyHostToDevice));
                w.tiled = (const uint8_t *) (qb + pl.tiled);
            }
            q5m[groups[gi][0]] = w;
        }
        // symmetric formats: the encoder and cross-K/V matrices (M >= 2048 rows at batch) also as exact
        // f16 integers + transposed scales for the f16 MFMA ring kernel (gemm_q16); large-v3: 1.4 GB
        if (!qf_has_m(f)) {
            std::vector<size_t> sel;
            size_t tot = 0;
            auto al = [](size_t b) { return (b + 255) & ~(size_t) 255; };
            for (size_t gi = 1; gi < groups.size(); ++gi) {
                if (gi >= n_enc_groups && groups[gi][0].find("cross_attn.key") == std::string::npos) continue;
                const Plan & pl = plans[gi];
                const int npad = (pl.N + 255) / 256 * 256;
                tot += al((size_t) pl.N * pl.K * 2) + al((size_t) (pl.K / 32) * npad * 4);
                sel.push_back(gi);
            }
            m->q16blob.alloc(tot);
            char * b16 = (char *) m->q16blob.ptr;
            size_t o = 0;
            for (size_t gi : sel) {
                const Plan & pl = plans[gi];
                Q5W & w = q5m[groups[gi][0]];
                w.npad = (pl.N + 255) / 256 * 256;
                w.wi = (const _Float16 *) (b16 + o);
                o += al((size_t) pl.N * pl.K * 2);
                w.dwt = (const float *) (b16 + o);
                o += al((size_t) (pl.K / 32) * w.npad * 4);
                quant_expand_f16(nullptr, w, pl.N, pl.K, (_Float16 *) w.wi, (float *) w.dwt, w.npad);
            }
            OWK_HIP_CHECK(hipDeviceSynchronize());
        }
    }
    auto Q = [&](const std::string & n) { auto it = q5m.find(n); return it == q5m.end() ? Q5W() : it->second; };
    m->conv1_w = (const _Float16 *) (base + o_conv1);
    m->conv1_b = F("encoder.conv1.bias");
    m->conv2_w = H("encoder.conv2.weight");
    m->conv2_b = F("encoder.conv2.bias");
    m->e_pe = F("encoder.positional_embedding");
    m->e_ln_w = F("encoder.ln_post.weight");
    m->e_ln_b = F("encoder.ln_post.bias");
    m->enc.resize(hp.n_audio_layer);
    for (int i = 0; i < hp.n_audio_layer; ++i) {
        const std::string p = "encoder.blocks." + std::to_string(i) + ".";
        EncLayerW & L = m->enc[i];
        L.attn_ln_w = F(p + "attn_ln.weight"); L.attn_ln_b = F(p + "attn_ln.bias");
        L.mlp_ln_w = F(p + "mlp_ln.weight"); L.mlp_ln_b = F(p + "mlp_ln.bias");
        L.w_qkv = (const _Float16 *) (base + o_enc_qkv[i]);
        L.b_q = F(p + "attn.query.bias"); L.b_v = F(p + "attn.value.bias");
        L.w_o = H(p + "attn.out.weight"); L.b_o = F(p + "attn.out.bias");
        L.w_mlp0 = H(p + "mlp.0.weight"); L.b_mlp0 = F(p + "mlp.0.bias");
        L.w_mlp1 = H(p + "mlp.2.weight"); L.b_mlp1 = F(p + "mlp.2.bias");
        if (m->q5) {
            L.w_qkv = nullptr;
            L.q_qkv = Q(p + "attn.query.weight");
            L.q_o = Q(p + "attn.out.weight");
            L.q_mlp0 = Q(p + "mlp.0.weight");
            L.q_mlp1 = Q(p + "mlp.2.weight");
        }
    }
    m->d_te = H("decoder.token_embedding.weight");
    m->q_te = Q("decoder.token_embedding.weight");
    m->d_pe = F("decoder.positional_embedding");
    m->d_ln_w = F("decoder.ln.weight");
    m->d_ln_b = F("decoder.ln.bias");
    m->dec.resize(hp.n_text_layer);
    for (int i = 0; i < hp.n_text_layer; ++i) {
        const std::string p = "decoder.blocks." + std::to_string(i) + ".";
        DecLayerW & L = m->dec[i];
        L.attn_ln_w = F(p + "attn_ln.weight"); L.attn_ln_b = F(p + "attn_ln.bias");
        L.cross_ln_w = F(p + "cross_attn_ln.weight"); L.cross_ln_b = F(p + "cross_attn_ln.bias");
        L.mlp_ln_w = F(p + "mlp_ln.weight"); L.mlp_ln_b = F(p + "mlp_ln.bias");
        L.w_qkv = (const _Float16 *) (base + o_dec_qkv[i]);
        L.b_q = F(p + "attn.query.bias"); L.b_v = F(p + "attn.value.bias");
        L.w_o = H(p + "attn.out.weight"); L.b_o = F(p + "attn.out.bias");
        L.cw_q = H(p + "cross_attn.query.weight"); L.cb_q = F(p + "cross_attn.query.bias");
        L.cw_kv = (const _Float16 *) (base + o_dec_ckv[i]);
        L.cb_v = F(p + "cross_attn.value.bias");
        L.cw_o = H(p + "cross_attn.out.weight"); L.cb_o = F(p + "cross_attn.out.bias");
        L.w_mlp0 = H(p + "mlp.0.weight"); L.b_mlp0 = F(p + "mlp.0.bias");
        L.w_mlp1 = H(p + "mlp.2.weight"); L.b_mlp1 = F(p + "mlp.2.bias");
        if (m->q5) {
            L.w_qkv = nullptr;
            L.cw_kv = nullptr;
            L.q_qkv = Q(p + "attn.query.weight");
            L.q_ckv = Q(p + "cross_attn.key.weight");
            L.q_o = Q(p + "attn.out.weight");
            L.q_cq = Q(p + "cross_attn.query.weight");
            L.q_co = Q(p + "cross_attn.out.weight");
            L.q_mlp0 = Q(p + "mlp.0.weight");
            L.q_mlp1 = Q(p + "mlp.2.weight");
        }
    }
    if (!m->q5) {
        // decoder weights re-laid out for the decode-row GEMM (an extra 1.6 GB for large-v3;
        // HBM holds both layouts comfortably, the row-major one still feeds prefills)
        const int d = hp.n_text_state;
        size_t tot = tiled_weight_elems(hp.n_vocab, d);
        const size_t per_layer = tiled_weight_elems(3 * d, d) + 3 * tiled_weight_elems(d, d) +
                                 tiled_weight_elems(4 * d, d) + tiled_weight_elems(d, 4 * d);
        tot += per_layer * hp.n_text_layer;
        m->tiled.alloc(tot * 2);
        _Float16 * t = m->tiled.as<_Float16>();
        size_t at = 0;
        auto tile = [&](const _Float16 * W, int N, int K) {
            _Float16 * out = t + at;
            tile_weights(nullptr, W, N, K, out);
            at += tiled_weight_elems(N, K);
            return (const _Float16 *) out;
        };
        for (int i = 0; i < hp.n_text_layer; ++i) {
            DecLayerW & L = m->dec[i];
            L.t_qkv = tile(L.w_qkv, 3 * d, d);
            L.t_o = tile(L.w_o, d, d);
            L.t_cq = tile(L.cw_q, d, d);
            L.t_co = tile(L.cw_o, d, d);
            L.t_mlp0 = tile(L.w_mlp0, 4 * d, d);
            L.t_mlp1 = tile(L.w_mlp1, d, 4 * d);
        }
        m->d_te_t = tile(m->d_te, hp.n_vocab, d);
        OWK_HIP_CHECK(hipDeviceSynchronize());
    }
    m->gelu_tab = (const uint16_t *) (base + o_gelu);
    m->mel_filters = (const float *) (base + o_filt);
    m->twiddle = (const double *) (base + o_tw);
    m->hann = (const float *) (base + o_hann);
    m->mel_rng = (const int *) (base + o_rng);
    return m.release();
}

std::vector<int> tokenize_text(const Vocab & v, const std::string & text) {
    // words: the GPT-2 pre-tokenizer regex in std::regex form, matched in the classic "C" locale
    // (bytes >= 0x80 are neither alpha nor digit), exactly as ref whisper.cpp:3276-3288
    std::vector<std::string> words;
    {
        std::string str = text;
        static const std::regex re(
            R"('s|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+)");
        std::smatch m;
        while (std::regex_search(str, m, re)) {
            for (auto x : m) words.push_back(x);
            str = m.suffix();
        }
    }
    // each word: repeatedly the longest vocabulary entry starting at i; a byte no entry starts
    // with is dropped with the reference's "unknown token" error
    std::vector<int> res;
    for (const auto & w : words) {
        const int n = (int) w.size();
        for (int i = 0; i < n;) {
            int j = n;
            for (; j > i; --j) {
                auto it = v.token_to_id.find(w.substr(i, j - i));
                if (it != v.token_to_id.end()) {
                    res.push_back(it->second);
                    break;
                }
            }
            if (j > i) {
                i = j;
            } else {
                log_msg(GGML_LOG_LEVEL_ERROR, "unknown token\n");
                ++i;
            }
        }
    }
    return res;
}

} // namespace owk
