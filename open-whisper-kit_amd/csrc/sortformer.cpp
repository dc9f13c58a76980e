// Streaming-SortFormer diarizer on MI355X: the C ABI of include/sortformer.h.
//
// Re-statement of /root/reference streaming-sortformer/src/sortformer.cpp ("ref:<line>"):
// the neural path (log-mel, conv2d subsampling, 17 conformer layers with relative-position
// attention, 512->192 projection, 18 post-LN transformer layers, speaker head) runs on the
// GPU (k_sortformer.hip + the MFMA GEMM of k_gemm.hip, weights resident in HBM); the
// streaming bookkeeping (chunking, FIFO, AOSC speaker-cache compression with
// std::nth_element, silence profile, feed/flush mel buffering) runs on the host exactly as
// the reference does, since its tie order is part of the result.
#include "sortformer.h"
#include "owk_sortformer.h"

#include "kquant.h"
#include "sf_kernels.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

using namespace owk;

namespace {

constexpr int N_SPK = 4;
constexpr int TF_D = 192, TF_H = 8, TF_DH = 24, TF_FF = 768;
constexpr int CONF_H = 8, CONF_DH = 64, CONF_K = 9;

bool sf_verbose() {
    static const bool v = getenv("OWK_SF_VERBOSE") && atoi(getenv("OWK_SF_VERBOSE")) > 0;
    return v;
}
#define SF_LOG(...)                                \
    do {                                           \
        if (sf_verbose()) fprintf(stderr, __VA_ARGS__); \
    } while (0)

// ---------------------------------------------------------------------------------
// GGUF v3 reader (the subset sortformer_init uses, ref:287-626 via ggml's gguf.cpp)
// ---------------------------------------------------------------------------------
struct GgufTensor {
    std::vector<int64_t> ne;
    int type = 0;  // ggml type: 0 F32, 1 F16, or a quantized block type (qfmt >= 0)
    int qfmt = -1; // QFmt of a quantized tensor (sortformer-quantize writes Q8_0 / Q4_K / Q5_K)
    const uint8_t * data = nullptr;
    size_t nbytes = 0;
};

// ggml type id -> QFmt (kernels.h) of the block formats the quantized GEMMs take; -1 otherwise
int gguf_qfmt(int t) {
    switch (t) {
        case 2: return QF_Q4_0;
        case 3: return QF_Q4_1;
        case 6: return QF_Q5_0;
        case 7: return QF_Q5_1;
        case 8: return QF_Q8_0;
        case 10: return QF_Q2_K;
        case 11: return QF_Q3_K;
        case 12: return QF_Q4_K;
        case 13: return QF_Q5_K;
        case 14: return QF_Q6_K;
        default: return -1;
    }
}

struct Gguf {
    std::vector<uint8_t> file;
    std::map<std::string, uint64_t> u32;
    std::map<std::string, float> f32;
    std::map<std::string, GgufTensor> tensors;

    bool load(const char * path, std::string & err) {
        FILE * f = fopen(path, "rb");
        if (!f) { err = "cannot open"; return false; }
        fseek(f, 0, SEEK_END);
        const long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        file.resize(n > 0 ? (size_t) n : 0);
        const size_t got = fread(file.data(), 1, file.size(), f);
        fclose(f);
        if (got != file.size()) { err = "short read"; return false; }
        size_t off = 0;
        auto need = [&](size_t k) { if (off + k > file.size()) throw std::runtime_error("truncated GGUF"); };
        auto rd = [&](void * dst, size_t k) { need(k); memcpy(dst, file.data() + off, k); off += k; };
        auto rd_u32 = [&]() { uint32_t v; rd(&v, 4); return v; };
        auto rd_u64 = [&]() { uint64_t v; rd(&v, 8); return v; };
        auto rd_str = [&]() { const uint64_t len = rd_u64(); need(len); std::string s((const char *) file.data() + off, len); off += len; return s; };
        try {
            char magic[4];
            rd(magic, 4);
            if (memcmp(magic, "GGUF", 4) != 0) { err = "bad magic"; return false; }
            const uint32_t version = rd_u32();
            if (version < 2) { err = "unsupported GGUF version"; return false; }
            const uint64_t n_tensors = rd_u64(), n_kv = rd_u64();
            static const size_t type_size[13] = {1, 1, 2, 2, 4, 4, 4, 1, 0, 0, 8, 8, 8};
            uint64_t alignment = 32;
            std::function<void(int)> skip = [&](int t) {
                if (t == 8) { (void) rd_str(); return; }
                if (t == 9) {
                    const int et = (int) rd_u32();
                    const uint64_t cnt = rd_u64();
                    for (uint64_t i = 0; i < cnt; ++i) skip(et);
                    return;
                }
                if (t < 0 || t > 12) throw std::runtime_error("bad GGUF value type");
                need(type_size[t]);
                off += type_size[t];
            };
            for (uint64_t i = 0; i < n_kv; ++i) {
                const std::string key = rd_str();
                const int t = (int) rd_u32();
                if (t == 4) {
                    u32[key] = rd_u32();
                    if (key == "general.alignment") alignment = u32[key];
                } else if (t == 6) {
                    float v; rd(&v, 4); f32[key] = v;
                } else {
                    skip(t);
                }
            }
            struct Info { std::string name; std::vector<int64_t> ne; int type; uint64_t off; };
            std::vector<Info> infos(n_tensors);
            for (auto & ti : infos) {
                ti.name = rd_str();
                const uint32_t nd = rd_u32();
                if (nd > 4) throw std::runtime_error("tensor rank > 4");
                ti.ne.resize(nd);
                for (auto & e : ti.ne) e = (int64_t) rd_u64();
                ti.type = (int) rd_u32();
                ti.off = rd_u64();
            }
            const size_t data0 = (off + alignment - 1) / alignment * alignment;
            for (auto & ti : infos) {
                size_t n = 1;
                for (auto e : ti.ne) n *= (size_t) e;
                GgufTensor t;
                t.ne = ti.ne;
                t.type = ti.type;
                if (ti.type == 0 || ti.type == 1) {
                    t.nbytes = n * (ti.type == 0 ? 4 : 2);
                } else {
                    // quantized rows (ggml_quantize_chunk blocks along ne[0])
                    t.qfmt = gguf_qfmt(ti.type);
                    if (t.qfmt < 0 || ti.ne.empty())
                        throw std::runtime_error("tensor " + ti.name + ": unsupported GGUF tensor type " + std::to_string(ti.type));
                    const int qk = qf_is_k(t.qfmt) ? 256 : 32;
                    if (ti.ne[0] % qk) throw std::runtime_error("tensor " + ti.name + ": row not a whole number of blocks");
                    t.nbytes = n / qk * (qf_is_k(t.qfmt) ? kq_block_bytes(t.qfmt) : qf_block_bytes(t.qfmt));
                }
                if (data0 + ti.off + t.nbytes > file.size()) throw std::runtime_error("tensor data out of file");
                t.data = file.data() + data0 + ti.off;
                tensors[ti.name] = t;
            }
        } catch (const std::exception & e) {
            err = e.what();
            return false;
        }
        return true;
    }
    const GgufTensor * get(const std::string & name) const {
        auto it = tensors.find(name);
        return it == tensors.end() ? nullptr : &it->second;
    }
};

// ---------------------------------------------------------------------------------
// device weight blob
// ---------------------------------------------------------------------------------
struct Blob {
    std::vector<uint8_t> host;
    size_t add(const void * p, size_t n) {
        const size_t off = (host.size() + 255) / 256 * 256;
        host.resize(off + n);
        if (p) memcpy(host.data() + off, p, n);
        return off;
    }
    template <typename V> size_t addv(const V & v) { return add(v.data(), v.size() * sizeof(v[0])); }
};

// one linear's weights: F16 [N][K] in the weight blob, or a quantized GGUF tensor (the reference's
// sortformer-quantize output, streaming-sortformer/tools/quantize.cpp:52-90) kept as the block arrays
// of kernels.h's Q5W -- 32-block formats split (qs / qh / d / m) plus the exact-f16 integer image the
// large-tile kernel reads, K-quants as the virtual-block image of kquant.h -- in the quantized blob
struct Lin {
    size_t off = (size_t) -1;  // F16 weights (blob offset); -1: quantized
    int fmt = -1, N = 0, K = 0, kx = 0, npad = 0;
    size_t qs = 0, qh = 0, d = 0, m = 0, wi = 0, dwt = 0;  // quantized blob offsets
    Q5W q;                                                 // resolved after the upload
    bool quant() const { return fmt >= 0; }
};
struct ConfLayer {
    size_t ln_ff1_w, ln_ff1_b, ff1_up_b, ff1_dn_b;
    size_t ln_sa_w, ln_sa_b, qkv_b, out_b, pbu, pbv;
    size_t ln_cv_w, ln_cv_b, pw1_b, dw, dw_b, pw2_b;
    size_t ln_ff2_w, ln_ff2_b, ff2_up_b, ff2_dn_b;
    size_t ln_out_w, ln_out_b;
    Lin ff1_up, ff1_dn, qkv, out, pos, pw1, pw2, ff2_up, ff2_dn;
};
struct TransLayer {
    size_t qkv_b, out_b, ln1_w, ln1_b, up_b, dn_b, ln2_w, ln2_b;
    Lin qkv, out, up, dn;
};

// streaming configuration / state (ref:1652-1727)
struct StreamConfig {
    int chunk_len = 188, fifo_len = 0, spkcache_len = 188, spkcache_update_period = 188;
    int chunk_left_context = 1, chunk_right_context = 1;
    int spkcache_sil_frames_per_spk = 3;
    float sil_threshold = 0.2f, pred_score_threshold = 0.25f, scores_boost_latest = 0.05f;
    float strong_boost_rate = 0.75f, weak_boost_rate = 1.5f, min_pos_scores_rate = 0.5f;
    int max_index = 99999;
};

struct StreamState {
    std::vector<float> spkcache, spkcache_preds;
    int spkcache_len = 0;
    bool spkcache_preds_valid = false;
    std::vector<float> fifo, fifo_preds;
    int fifo_len = 0;
    std::vector<float> mean_sil_emb;
    int n_sil_frames = 0;
    explicit StreamState(int d = 512) : mean_sil_emb(d, 0.0f) {}
};

}  // namespace

struct sortformer_context {
    sortformer_params params{};
    int device = 0;
    hipStream_t stream = nullptr;

    int n_mels = 128, n_fft = 512, hop = 160, win_length = 400, sample_rate = 16000;
    int d_model = 512, subsampling = 8, n_conf = 17, n_trans = 18, c_sub = 256;

    DevBuf w;  // weight blob
    size_t fb, win512, tw;
    size_t c0_w, c0_b, c2_w, c2_b, c3_w, c3_b, c5_w, c5_b, c6_w, c6_b, pre_out_b;
    Lin pre_out;
    std::vector<ConfLayer> conf;
    Lin proj;
    size_t proj_b;
    std::vector<TransLayer> trans;
    Lin hid, spk;
    size_t hid_b, spk_b;
    DevBuf qw;          // quantized linears (Lin::qs .. dwt)
    bool quant = false; // any linear quantized: producers also keep their f32 outputs

    // position-embedding cache (ref:140-142, 1127-1136): f16 table of the current n_pos
    int pos_T = 0;  // positions pos_T-1 .. -(pos_T-1) in pos16 / pos32
    DevBuf pos16;
    // every conformer layer's linear_pos weight stacked [n_conf * d][d] (F16 models): one GEMM of the
    // position table gives all layers' projections (a pass's 17 launches in one)
    DevBuf pos_all;

    // scratch (grown on demand)
    DevBuf s_pcm, s_mel, s_c1, s_c2, s_c3, s_c4, s_flat, s_pre;
    DevBuf s_x, s_y, s_xn, s_h, s_qkv, s_P, s_ao, s_cv, s_g, s_t32, s_t16, s_pred;
    // quantized models: f32 activations (LayerNorm rows, SiLU / ReLU outputs, attention outputs,
    // the position table) and the Q8 operand buffers of the quantized GEMMs
    DevBuf s_xn32, s_h32, s_ao32, pos32, s_q8, s_q8d, s_q16, s_q16d;

    template <typename T> T * wp(size_t off) const { return (T *) ((uint8_t *) w.ptr + off); }
    float * f(size_t off) const { return wp<float>(off); }
    _Float16 * h(size_t off) const { return wp<_Float16>(off); }

    ~sortformer_context() {
        if (stream) (void) hipStreamDestroy(stream);
    }
};

struct sortformer_stream_state {
    sortformer_context * ctx = nullptr;  // not owned (ref:2677)
    StreamConfig cfg;
    StreamState st;
    std::vector<float> audio_overlap;
    std::vector<float> mel_buffer;
    int mel_buffer_frames = 0;
    int64_t total_samples_fed = 0;
    int64_t total_frames_output = 0;
};

namespace {

// ---------------------------------------------------------------------------------
// model load
// ---------------------------------------------------------------------------------
void load_weights(sortformer_context * ctx, const Gguf & g) {
    Blob blob;
    auto T = [&](const std::string & name) -> const GgufTensor & {
        const GgufTensor * t = g.get(name);
        if (!t) throw std::runtime_error("tensor '" + name + "' not found");
        return *t;
    };
    auto as_f32 = [&](const GgufTensor & t) {
        if (t.qfmt >= 0) throw std::runtime_error("quantized GGUF tensor where F32/F16 is expected");
        size_t n = t.nbytes / (t.type == 0 ? 4 : 2);
        std::vector<float> v(n);
        if (t.type == 0) memcpy(v.data(), t.data, t.nbytes);
        else for (size_t i = 0; i < n; ++i) v[i] = f16_to_f32_host(((const uint16_t *) t.data)[i]);
        return v;
    };
    auto as_f16 = [&](const GgufTensor & t) {
        if (t.qfmt >= 0) throw std::runtime_error("quantized GGUF tensor where F32/F16 is expected");
        size_t n = t.nbytes / (t.type == 0 ? 4 : 2);
        std::vector<uint16_t> v(n);
        if (t.type == 1) memcpy(v.data(), t.data, t.nbytes);
        else for (size_t i = 0; i < n; ++i) v[i] = f32_to_f16_host(((const float *) t.data)[i]);
        return v;
    };
    Blob qb;
    // a linear's weights (several GGUF tensors packed along the output rows, like q/k/v): F16 in the
    // blob, or the quantized tensors' blocks (every part of one type) as Lin's arrays in qb. K is the
    // product of all dims but the last (the 1x1 conv weights [1][K][N] reshape to 2-D, ref:1240-1241)
    auto Lcat = [&](std::initializer_list<std::string> names) {
        Lin L;
        std::vector<const GgufTensor *> ts;
        for (auto & n : names) ts.push_back(&T(n));
        auto kdim = [](const GgufTensor & t) {
            int64_t k = 1;
            for (size_t i = 0; i + 1 < t.ne.size(); ++i) k *= t.ne[i];
            return k;
        };
        const int64_t K = kdim(*ts[0]);
        int64_t N = 0;
        for (auto * t : ts) {
            if (t->ne.size() < 2 || kdim(*t) != K) throw std::runtime_error("linear weight shape mismatch");
            if (t->qfmt != ts[0]->qfmt) throw std::runtime_error("packed linear weights of mixed types");
            N += t->ne.back();
        }
        L.N = (int) N;
        L.K = (int) K;
        if (ts[0]->qfmt < 0) {
            std::vector<uint16_t> all;
            for (auto * t : ts) { auto v = as_f16(*t); all.insert(all.end(), v.begin(), v.end()); }
            L.off = blob.addv(all);
            return L;
        }
        const int q = L.fmt = ts[0]->qfmt;
        std::vector<uint8_t> raw;
        for (auto * t : ts) raw.insert(raw.end(), t->data, t->data + t->nbytes);
        L.npad = (L.N + 255) / 256 * 256;
        if (qf_is_k(q)) {
            // the virtual-block f16 integers + scales every GEMM shape runs on (gemm_q16, kquant.h)
            L.kx = kq_kx(q, L.K);
            std::vector<uint16_t> wi((size_t) L.N * L.kx);
            std::vector<float> dwt((size_t) (L.kx / 32) * L.npad);
            kq_expand_host(q, raw.data(), L.N, L.K, wi.data(), dwt.data(), L.npad);
            L.wi = qb.addv(wi);
            L.dwt = qb.addv(dwt);
        } else {
            const size_t nbk = (size_t) L.N * (L.K / 32);
            std::vector<uint8_t> qs(nbk * qf_qs_bytes(q));
            std::vector<uint32_t> qh(qf_has_qh(q) ? nbk : 0);
            std::vector<uint16_t> dd(nbk), mm(qf_has_m(q) ? nbk : 0);
            quant_split_host(q, raw.data(), L.N, L.K, qs.data(), qh.empty() ? nullptr : qh.data(), dd.data(),
                             mm.empty() ? nullptr : mm.data());
            L.qs = qb.addv(qs);
            L.d = qb.addv(dd);
            if (!qh.empty()) L.qh = qb.addv(qh);
            if (!mm.empty()) L.m = qb.addv(mm);
            if (!qf_has_m(q)) {  // symmetric formats: exact-f16 integer image for the large-tile kernel
                L.wi = qb.add(nullptr, (size_t) L.N * L.K * 2);
                L.dwt = qb.add(nullptr, (size_t) (L.K / 32) * L.npad * 4);
            }
        }
        ctx->quant = true;
        return L;
    };
    auto Lw = [&](const std::string & name) { return Lcat({name}); };
    auto F = [&](const std::string & name) { auto v = as_f32(T(name)); return blob.add(v.data(), v.size() * 4); };
    auto Fcat = [&](std::initializer_list<std::string> names) {
        std::vector<float> all;
        for (auto & n : names) { auto v = as_f32(T(n)); all.insert(all.end(), v.begin(), v.end()); }
        return blob.add(all.data(), all.size() * 4);
    };

    // mel front-end tensors (ref:329-366) + FFT twiddles as the reference recurrence makes them
    {
        const GgufTensor & fbt = T("preprocessor.featurizer.fb");
        if (fbt.ne.size() < 2 || fbt.ne[0] != ctx->n_fft / 2 + 1 || fbt.ne[1] != ctx->n_mels)
            throw std::runtime_error("unexpected fb shape");
        ctx->fb = F("preprocessor.featurizer.fb");
        const GgufTensor & wt = T("preprocessor.featurizer.window");
        if (wt.ne.empty() || wt.ne[0] != ctx->win_length) throw std::runtime_error("unexpected window shape");
        auto wv = as_f32(wt);
        std::vector<float> w512(ctx->n_fft, 0.0f);
        const int wpad = (ctx->n_fft - ctx->win_length) / 2;  // centre the window (ref:813-817)
        for (int i = 0; i < ctx->win_length; ++i) w512[wpad + i] = wv[i];
        ctx->win512 = blob.add(w512.data(), w512.size() * 4);
        std::vector<float> tw;
        for (int len = 2; len <= ctx->n_fft; len *= 2) {  // ref:229-262
            const float angle = -2.0f * (float) M_PI / (float) len;
            const float w_re = cosf(angle), w_im = sinf(angle);
            float tr = 1.0f, ti = 0.0f;
            for (int k = 0; k < len / 2; ++k) {
                tw.push_back(tr);
                tw.push_back(ti);
                const float nr = tr * w_re - ti * w_im;
                const float ni = tr * w_im + ti * w_re;
                tr = nr;
                ti = ni;
            }
        }
        ctx->tw = blob.add(tw.data(), tw.size() * 4);
    }
    // pre-encoder: conv kernels cast to F32 (ref:971-977), out linear F16
    const std::string pe = "encoder.pre_encode.";
    ctx->c0_w = F(pe + "conv.0.weight"); ctx->c0_b = F(pe + "conv.0.bias");
    ctx->c2_w = F(pe + "conv.2.weight"); ctx->c2_b = F(pe + "conv.2.bias");
    ctx->c3_w = F(pe + "conv.3.weight"); ctx->c3_b = F(pe + "conv.3.bias");
    ctx->c5_w = F(pe + "conv.5.weight"); ctx->c5_b = F(pe + "conv.5.bias");
    ctx->c6_w = F(pe + "conv.6.weight"); ctx->c6_b = F(pe + "conv.6.bias");
    {
        const GgufTensor & ow = T(pe + "out.weight");
        if (ow.ne.size() != 2 || ow.ne[1] != ctx->d_model || ow.ne[0] != (int64_t) ctx->c_sub * (ctx->n_mels / 8))
            throw std::runtime_error("unexpected pre_encode.out shape");
    }
    ctx->pre_out = Lw(pe + "out.weight"); ctx->pre_out_b = F(pe + "out.bias");

    ctx->conf.resize(ctx->n_conf);
    for (int i = 0; i < ctx->n_conf; ++i) {
        const std::string p = "encoder.layers." + std::to_string(i) + ".";
        ConfLayer & L = ctx->conf[i];
        L.ln_ff1_w = F(p + "norm_feed_forward1.weight"); L.ln_ff1_b = F(p + "norm_feed_forward1.bias");
        L.ff1_up = Lw(p + "feed_forward1.linear1.weight"); L.ff1_up_b = F(p + "feed_forward1.linear1.bias");
        L.ff1_dn = Lw(p + "feed_forward1.linear2.weight"); L.ff1_dn_b = F(p + "feed_forward1.linear2.bias");
        L.ln_sa_w = F(p + "norm_self_att.weight"); L.ln_sa_b = F(p + "norm_self_att.bias");
        L.qkv = Lcat({p + "self_attn.linear_q.weight", p + "self_attn.linear_k.weight", p + "self_attn.linear_v.weight"});
        L.qkv_b = Fcat({p + "self_attn.linear_q.bias", p + "self_attn.linear_k.bias", p + "self_attn.linear_v.bias"});
        L.out = Lw(p + "self_attn.linear_out.weight"); L.out_b = F(p + "self_attn.linear_out.bias");
        L.pos = Lw(p + "self_attn.linear_pos.weight");
        L.pbu = F(p + "self_attn.pos_bias_u"); L.pbv = F(p + "self_attn.pos_bias_v");
        L.ln_cv_w = F(p + "norm_conv.weight"); L.ln_cv_b = F(p + "norm_conv.bias");
        L.pw1 = Lw(p + "conv.pointwise_conv1.weight"); L.pw1_b = F(p + "conv.pointwise_conv1.bias");
        L.dw = F(p + "conv.depthwise_conv.weight"); L.dw_b = F(p + "conv.depthwise_conv.bias");
        L.pw2 = Lw(p + "conv.pointwise_conv2.weight"); L.pw2_b = F(p + "conv.pointwise_conv2.bias");
        L.ln_ff2_w = F(p + "norm_feed_forward2.weight"); L.ln_ff2_b = F(p + "norm_feed_forward2.bias");
        L.ff2_up = Lw(p + "feed_forward2.linear1.weight"); L.ff2_up_b = F(p + "feed_forward2.linear1.bias");
        L.ff2_dn = Lw(p + "feed_forward2.linear2.weight"); L.ff2_dn_b = F(p + "feed_forward2.linear2.bias");
        L.ln_out_w = F(p + "norm_out.weight"); L.ln_out_b = F(p + "norm_out.bias");
    }
    ctx->proj = Lw("sortformer_modules.encoder_proj.weight");
    ctx->proj_b = F("sortformer_modules.encoder_proj.bias");
    ctx->trans.resize(ctx->n_trans);
    for (int i = 0; i < ctx->n_trans; ++i) {
        const std::string p = "transformer_encoder.layers." + std::to_string(i) + ".";
        TransLayer & L = ctx->trans[i];
        L.qkv = Lcat({p + "first_sub_layer.query_net.weight", p + "first_sub_layer.key_net.weight",
                      p + "first_sub_layer.value_net.weight"});
        L.qkv_b = Fcat({p + "first_sub_layer.query_net.bias", p + "first_sub_layer.key_net.bias",
                        p + "first_sub_layer.value_net.bias"});
        L.out = Lw(p + "first_sub_layer.out_projection.weight"); L.out_b = F(p + "first_sub_layer.out_projection.bias");
        L.ln1_w = F(p + "layer_norm_1.weight"); L.ln1_b = F(p + "layer_norm_1.bias");
        L.up = Lw(p + "second_sub_layer.dense_in.weight"); L.up_b = F(p + "second_sub_layer.dense_in.bias");
        L.dn = Lw(p + "second_sub_layer.dense_out.weight"); L.dn_b = F(p + "second_sub_layer.dense_out.bias");
        L.ln2_w = F(p + "layer_norm_2.weight"); L.ln2_b = F(p + "layer_norm_2.bias");
    }
    ctx->hid = Lw("sortformer_modules.first_hidden_to_hidden.weight");
    ctx->hid_b = F("sortformer_modules.first_hidden_to_hidden.bias");
    ctx->spk = Lw("sortformer_modules.single_hidden_to_spks.weight");
    ctx->spk_b = F("sortformer_modules.single_hidden_to_spks.bias");

    ctx->w.alloc(blob.host.size());
    OWK_HIP_CHECK(hipMemcpy(ctx->w.ptr, blob.host.data(), blob.host.size(), hipMemcpyHostToDevice));
    if (ctx->quant) {
        ctx->qw.alloc(qb.host.size());
        OWK_HIP_CHECK(hipMemcpy(ctx->qw.ptr, qb.host.data(), qb.host.size(), hipMemcpyHostToDevice));
        uint8_t * base = (uint8_t *) ctx->qw.ptr;
        auto resolve = [&](Lin & L) {
            if (!L.quant()) return;
            Q5W & q = L.q;
            q.fmt = L.fmt;
            q.npad = L.npad;
            q.kx = L.kx;
            q.wi = L.wi || qf_is_k(L.fmt) ? (const _Float16 *) (base + L.wi) : nullptr;
            q.dwt = q.wi ? (const float *) (base + L.dwt) : nullptr;
            if (!qf_is_k(L.fmt)) {
                q.qs = base + L.qs;
                q.d = (const _Float16 *) (base + L.d);
                if (qf_has_qh(L.fmt)) q.qh = (const uint32_t *) (base + L.qh);
                if (qf_has_m(L.fmt)) q.m = (const _Float16 *) (base + L.m);
                if (q.wi) quant_expand_f16(ctx->stream, q, L.N, L.K, (_Float16 *) q.wi, (float *) q.dwt, q.npad);
            }
        };
        resolve(ctx->pre_out);
        resolve(ctx->proj);
        resolve(ctx->hid);
        resolve(ctx->spk);
        for (auto & L : ctx->conf)
            for (Lin * l : {&L.ff1_up, &L.ff1_dn, &L.qkv, &L.out, &L.pos, &L.pw1, &L.pw2, &L.ff2_up, &L.ff2_dn}) resolve(*l);
        for (auto & L : ctx->trans)
            for (Lin * l : {&L.qkv, &L.out, &L.up, &L.dn}) resolve(*l);
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        SF_LOG("sortformer_init: %.1f MB of quantized linears\n", qb.host.size() / 1e6);
    }
    bool all_f16 = !ctx->conf.empty();
    for (const auto & L : ctx->conf) all_f16 = all_f16 && !L.pos.quant();
    if (all_f16) {
        const size_t dd = (size_t) ctx->d_model * ctx->d_model;
        ctx->pos_all.alloc(ctx->conf.size() * dd * 2);
        for (size_t il = 0; il < ctx->conf.size(); ++il)
            OWK_HIP_CHECK(hipMemcpyAsync(ctx->pos_all.as<_Float16>() + il * dd, ctx->h(ctx->conf[il].pos.off), dd * 2,
                                         hipMemcpyDeviceToDevice, ctx->stream));
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    }
    SF_LOG("sortformer_init: %.1f MB of weights resident on device %d\n", blob.host.size() / 1e6, ctx->device);
}

// ---------------------------------------------------------------------------------
// GPU passes
// ---------------------------------------------------------------------------------
void dev_guard(sortformer_context * ctx) { OWK_HIP_CHECK(hipSetDevice(ctx->device)); }

template <typename Tp> Tp * grow(DevBuf & b, size_t n) {
    b.alloc(n * sizeof(Tp));
    return b.as<Tp>();
}

// y = W x with the fused epilogue `mode` (the reference's ggml_mul_mat + bias / activation / residual).
// F16 weights take the f16 activation A16 (ggml converts src1 to F16, the vec_dot_type of F16).
// Quantized weights round the f32 activation A32 to the weight's vec_dot_type -- Q8_0 / Q8_1 per 32
// (x86 quantize_row_q8_0 / _q8_1) or Q8_K per 256 (quantize_row_q8_K) -- as ggml_compute_forward_mul_mat
// does for its f32 src1 (ggml-cpu.c), then the block dots: large tiles on the f16 MFMA ring kernel over
// the exact integers (gemm_q16), other shapes on the int8 MFMA kernels (gemm_q5). A32 null: the f16
// activation is quantized instead (only where the reference's operand is itself f16-exact).
void sf_lin(sortformer_context * ctx, int mode, int M, int N, int K, const _Float16 * A16, const float * A32, int lda,
            const Lin & w, const EpiParams & ep) {
    hipStream_t s = ctx->stream;
    if (M <= 0) return;
    if (w.N != N || w.K != K) throw std::runtime_error("sortformer: linear shape mismatch");
    if (!w.quant()) {
        gemm(s, mode, M, N, K, A16, lda, ctx->h(w.off), K, ep);
        return;
    }
    const Q5W & q = w.q;
    const int mpad = (M + 255) / 256 * 256;
    if (qf_is_k(q.fmt)) {
        _Float16 * q16 = grow<_Float16>(ctx->s_q16, (size_t) M * q.kx);
        float * q16d = grow<float>(ctx->s_q16d, (size_t) (q.kx / 32) * mpad);
        quantize_q8k_f16(s, A32, A32 ? nullptr : A16, lda, M, K, q.fmt, q16, q16d, mpad);
        gemm_q16(s, mode, M, N, q.kx, q16, q16d, mpad, q, ep);
    } else if (gemm_q16_applies(q, M, N, K)) {
        _Float16 * q16 = grow<_Float16>(ctx->s_q16, (size_t) M * K);
        float * q16d = grow<float>(ctx->s_q16d, (size_t) (K / 32) * mpad);
        quantize_q8_f16(s, A32, A32 ? nullptr : A16, lda, M, K, q16, q16d, mpad);
        gemm_q16(s, mode, M, N, K, q16, q16d, mpad, q, ep);
    } else {
        int8_t * qa = grow<int8_t>(ctx->s_q8, (size_t) M * K);
        float * da = grow<float>(ctx->s_q8d, (size_t) M * (K / 32));
        quantize_q8(s, A32, A32 ? nullptr : A16, lda, M, K, qa, da);
        gemm_q5(s, mode, M, N, K, qa, da, q, ep);
    }
}
// f32 copy of an activation for a quantized consumer (null when the consumer is F16)
float * f32_for(sortformer_context * ctx, const Lin & consumer, DevBuf & buf, size_t n) {
    return consumer.quant() ? grow<float>(buf, n) : nullptr;
}

struct MelDims {
    int n_frames_out, seq_len, n_compute;
};
MelDims mel_dims(const sortformer_context * ctx, int n_samples) {
    MelDims m;
    const int pad = ctx->n_fft / 2;
    const int padded_len = n_samples + 2 * pad;
    const int n_stft = 1 + (padded_len - ctx->n_fft) / ctx->hop;  // ref:821
    m.seq_len = n_samples / ctx->hop;                             // ref:825
    m.n_frames_out = n_stft;
    const int rem = m.n_frames_out % 16;                           // pad_to 16 (ref:830-834)
    if (rem) m.n_frames_out += 16 - rem;
    m.n_compute = std::min(n_stft, m.seq_len);
    return m;
}

// log-mel of host samples into ctx->s_mel [n_mels][n_frames_out] (device)
MelDims run_mel(sortformer_context * ctx, const float * samples, int n_samples) {
    const MelDims md = mel_dims(ctx, n_samples);
    float * pcm = grow<float>(ctx->s_pcm, std::max(n_samples, 1));
    OWK_HIP_CHECK(hipMemcpyAsync(pcm, samples, (size_t) n_samples * 4, hipMemcpyHostToDevice, ctx->stream));
    float * mel = grow<float>(ctx->s_mel, (size_t) ctx->n_mels * std::max(md.n_frames_out, 1));
    sf::mel(ctx->stream, pcm, n_samples, ctx->f(ctx->win512), ctx->f(ctx->tw), ctx->f(ctx->fb), ctx->n_mels, md.n_compute,
            md.n_frames_out, mel);
    return md;
}

int conv_out(int n) { return (n - 1) / 2 + 1; }  // k3 s2 p1 (ref:919-925)

// pre-encoder over mel[f][c0 .. c0+T_in) (row stride ld, device) -> ctx->s_pre [T3][d] f32
int run_preenc(sortformer_context * ctx, const float * mel, int ld, int c0, int T_in) {
    const int C = ctx->c_sub;
    const int T1 = conv_out(T_in), F1 = conv_out(ctx->n_mels);
    const int T2 = conv_out(T1), F2 = conv_out(F1);
    const int T3 = conv_out(T2), F3 = conv_out(F2);
    if (C * F3 != 4096 && C * F3 % 64 != 0) throw std::runtime_error("pre-encoder flatten width");
    hipStream_t s = ctx->stream;
    float * a1 = grow<float>(ctx->s_c1, (size_t) T1 * F1 * C);
    float * a2 = grow<float>(ctx->s_c2, (size_t) T2 * F2 * C);
    float * a3 = grow<float>(ctx->s_c3, (size_t) T2 * F2 * C);
    float * a4 = grow<float>(ctx->s_c4, (size_t) T3 * F3 * C);
    _Float16 * flat = grow<_Float16>(ctx->s_flat, (size_t) T3 * C * F3);
    float * out = grow<float>(ctx->s_pre, (size_t) T3 * ctx->d_model);
    sf::conv0(s, mel, ld, c0, T_in, ctx->n_mels, ctx->f(ctx->c0_w), ctx->f(ctx->c0_b), C, a1, T1, F1);
    sf::dwconv(s, a1, T1, F1, C, ctx->f(ctx->c2_w), ctx->f(ctx->c2_b), a2, T2, F2);
    sf::pwconv(s, a2, T2 * F2, C, ctx->f(ctx->c3_w), ctx->f(ctx->c3_b), 0, F2, a3, nullptr, 0);
    sf::dwconv(s, a3, T2, F2, C, ctx->f(ctx->c5_w), ctx->f(ctx->c5_b), a4, T3, F3);
    sf::pwconv(s, a4, T3 * F3, C, ctx->f(ctx->c6_w), ctx->f(ctx->c6_b), 1, F3, nullptr, flat, C * F3);
    EpiParams ep;
    ep.bias = ctx->f(ctx->pre_out_b);
    ep.out32 = out;
    ep.ldo = ctx->d_model;
    sf_lin(ctx, EPI_BIAS_F32, T3, ctx->d_model, C * F3, flat, nullptr, C * F3, ctx->pre_out, ep);
    return T3;
}

// NeMo relative positions T-1 .. -(T-1), interleaved sin/cos (ref:1050-1066), as F16 (the
// activation rounding of linear_pos's F16 mul_mat). A row depends only on its position, so one table
// for the longest T seen (rounded up to 64) serves every shorter T as a contiguous row range: returns
// the row of position T-1. (The reference rebuilds it per n_pos; here a streaming pass whose length
// changes no longer recomputes 0.4 M transcendentals on the host and waits for the upload.)
int ensure_pos(sortformer_context * ctx, int T) {
    if (T > ctx->pos_T) {
        const int Tc = (T + 63) / 64 * 64, n_pos = 2 * Tc - 1, d = ctx->d_model;
        std::vector<uint16_t> pe((size_t) n_pos * d);
        std::vector<float> pe32((size_t) n_pos * d);  // quantized linear_pos: the f32 table is its operand
        const int half = d / 2;
        for (int p = 0; p < n_pos; ++p) {
            const float pos = (float) (Tc - 1 - p);
            for (int j = 0; j < half; ++j) {
                const float freq = 1.0f / powf(10000.0f, (2.0f * j) / (float) d);
                const float angle = pos * freq;
                pe32[(size_t) p * d + 2 * j] = sinf(angle);
                pe32[(size_t) p * d + 2 * j + 1] = cosf(angle);
            }
        }
        for (size_t i = 0; i < pe.size(); ++i) pe[i] = f32_to_f16_host(pe32[i]);
        _Float16 * dst = grow<_Float16>(ctx->pos16, pe.size());
        OWK_HIP_CHECK(hipMemcpyAsync(dst, pe.data(), pe.size() * 2, hipMemcpyHostToDevice, ctx->stream));
        if (ctx->quant) {
            float * d32 = grow<float>(ctx->pos32, pe32.size());
            OWK_HIP_CHECK(hipMemcpyAsync(d32, pe32.data(), pe32.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        }
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));  // pe is a host temporary
        ctx->pos_T = Tc;
    }
    return ctx->pos_T - T;
}

// independent sequences stacked along the rows of one buffer: (first row, length). Row-wise
// layers (GEMMs, LayerNorms) run once over all rows -- one weight read for every stream --;
// attention and the depthwise conv run per sequence.
typedef std::vector<std::pair<int, int>> Segs;

// conformer layers 0..last over x (device f32 [T][d], already xscaled). Returns the buffer
// holding the output (f32) and fills ctx->s_xn with its f16 copy.
float * run_conformer(sortformer_context * ctx, float * x, const Segs & segs, int last) {
    int T = 0, Tmax = 0;
    for (const auto & sg : segs) {
        T += sg.second;
        Tmax = std::max(Tmax, sg.second);
    }
    const int d = ctx->d_model;
    hipStream_t s = ctx->stream;
    float * y = grow<float>(ctx->s_y, (size_t) T * d);
    _Float16 * xn = grow<_Float16>(ctx->s_xn, (size_t) T * d);
    _Float16 * hbuf = grow<_Float16>(ctx->s_h, (size_t) T * 4 * d);
    float * qkv = grow<float>(ctx->s_qkv, (size_t) T * 3 * d);
    const size_t p0 = (size_t) ensure_pos(ctx, Tmax) * d;  // table row of position Tmax-1
    // linear_pos of every layer at once when the weights are stacked: P_all [2 Tmax - 1][n_conf * d]
    const bool pos_batched = ctx->pos_all.ptr != nullptr;
    const int ldP = pos_batched ? ctx->n_conf * d : d;
    float * P = grow<float>(ctx->s_P, (size_t) (2 * Tmax - 1) * ldP);
    if (pos_batched) {
        // only the layers this call runs (0 .. last): the stacked weights are layer-major. Each P value is
        // the same MFMA chain over K = d whichever tile kernel the N of the call selects: the 64x64 ring
        // (a per-layer N = d at these M) and the 128x128 tile are bit-identical (test_gpu_kernels.py
        // test_gemm_mid_matches_128, f32 epilogue at K = 512), and M >= 2048 takes the 8-phase kernel for
        // both, whose outputs do not depend on N
        EpiParams ep;
        ep.out32 = P;
        ep.ldo = ldP;
        gemm(s, EPI_F32, 2 * Tmax - 1, (last + 1) * d, d, ctx->pos16.as<_Float16>() + p0, d, ctx->pos_all.as<_Float16>(),
             d, ep);
    }
    _Float16 * ao = grow<_Float16>(ctx->s_ao, (size_t) T * d);
    float * cv = grow<float>(ctx->s_cv, (size_t) T * 2 * d);
    _Float16 * g = grow<_Float16>(ctx->s_g, (size_t) T * d);
    const float eps = 1e-5f;
    bool ff1_done = false;  // the layer's first LayerNorm already ran with the previous layer's last
    for (int il = 0; il <= last; ++il) {
        const ConfLayer & L = ctx->conf[il];
        auto ffn = [&](size_t lnw, size_t lnb, const Lin & up, size_t upb, const Lin & dn, size_t dnb, bool ln_done) {
            float * xn32 = f32_for(ctx, up, ctx->s_xn32, (size_t) T * d);
            if (!ln_done) layernorm_f16(s, x, T, d, ctx->f(lnw), ctx->f(lnb), eps, xn, d, nullptr, xn32);
            float * h32 = f32_for(ctx, dn, ctx->s_h32, (size_t) T * 4 * d);
            EpiParams e1;
            e1.bias = ctx->f(upb); e1.out16 = hbuf; e1.out32 = h32; e1.ldo = 4 * d;
            sf_lin(ctx, EPI_SILU_F16, T, 4 * d, d, xn, xn32, d, up, e1);
            EpiParams e2;
            e2.bias = ctx->f(dnb); e2.resid = x; e2.out32 = x; e2.ldo = d;
            sf_lin(ctx, EPI_HALF_RESID, T, d, 4 * d, hbuf, h32, 4 * d, dn, e2);
        };
        // FFN1 (ref:1159-1168)
        ffn(L.ln_ff1_w, L.ln_ff1_b, L.ff1_up, L.ff1_up_b, L.ff1_dn, L.ff1_dn_b, ff1_done);
        // relative-position MHSA (ref:1170-1235)
        {
            float * xn32 = f32_for(ctx, L.qkv, ctx->s_xn32, (size_t) T * d);
            layernorm_f16(s, x, T, d, ctx->f(L.ln_sa_w), ctx->f(L.ln_sa_b), eps, xn, d, nullptr, xn32);
            EpiParams e;
            e.bias = ctx->f(L.qkv_b); e.out32 = qkv; e.ldo = 3 * d;
            sf_lin(ctx, EPI_BIAS_F32, T, 3 * d, d, xn, xn32, d, L.qkv, e);
            if (!pos_batched) {
                EpiParams ep;
                ep.out32 = P; ep.ldo = d;
                sf_lin(ctx, EPI_F32, 2 * Tmax - 1, d, d, ctx->pos16.as<_Float16>() + p0,
                       L.pos.quant() ? ctx->pos32.as<float>() + p0 : nullptr, d, L.pos, ep);
            }
            const float * Pl = pos_batched ? P + (size_t) il * d : P;
            // positions Tb-1 .. -(Tb-1) of a shorter sequence are rows Tmax-Tb .. of the table
            float * ao32 = f32_for(ctx, L.out, ctx->s_ao32, (size_t) T * d);
            for (const auto & sg : segs)
                sf::attention(s, CONF_DH, true, qkv + (size_t) sg.first * 3 * d, 3 * d, d, 2 * d, sg.second, CONF_H,
                              ctx->f(L.pbu), ctx->f(L.pbv), Pl + (size_t) (Tmax - sg.second) * ldP,
                              1.0f / sqrtf((float) CONF_DH), ao + (size_t) sg.first * d,
                              ao32 ? ao32 + (size_t) sg.first * d : nullptr, ldP);
            EpiParams eo;
            eo.bias = ctx->f(L.out_b); eo.resid = x; eo.out32 = x; eo.ldo = d;
            sf_lin(ctx, EPI_RESID_F32, T, d, d, ao, ao32, d, L.out, eo);
        }
        // conv module (ref:1237-1274); sortformer-quantize leaves the 1x1 convs F16 (their rows are
        // ne[0] = 1 wide, quantize.cpp:167-169)
        {
            float * xn32 = f32_for(ctx, L.pw1, ctx->s_xn32, (size_t) T * d);
            layernorm_f16(s, x, T, d, ctx->f(L.ln_cv_w), ctx->f(L.ln_cv_b), eps, xn, d, nullptr, xn32);
            EpiParams e;
            e.bias = ctx->f(L.pw1_b); e.out32 = cv; e.ldo = 2 * d;
            sf_lin(ctx, EPI_BIAS_F32, T, 2 * d, d, xn, xn32, d, L.pw1, e);
            for (const auto & sg : segs)
                sf::glu_dwconv(s, cv + (size_t) sg.first * 2 * d, sg.second, d, ctx->f(L.dw), CONF_K, ctx->f(L.dw_b),
                               g + (size_t) sg.first * d);
            EpiParams eo;
            eo.bias = ctx->f(L.pw2_b); eo.resid = x; eo.out32 = x; eo.ldo = d;
            sf_lin(ctx, EPI_RESID_F32, T, d, d, g, nullptr, d, L.pw2, eo);
        }
        // FFN2 (ref:1276-1285)
        ffn(L.ln_ff2_w, L.ln_ff2_b, L.ff2_up, L.ff2_up_b, L.ff2_dn, L.ff2_dn_b, false);
        // final LayerNorm (ref:1288) -> y, then swap; below the last layer the next layer's FFN1 LayerNorm
        // runs in the same launch from the f32 rows in registers (bit-identical to two launches)
        if (il < last) {
            const ConfLayer & N = ctx->conf[il + 1];
            // LN1's f16 row is read by nothing (the next layer takes the f32 y): not written
            layernorm2_f16(s, x, T, d, ctx->f(L.ln_out_w), ctx->f(L.ln_out_b), nullptr, y, ctx->f(N.ln_ff1_w),
                           ctx->f(N.ln_ff1_b), xn, f32_for(ctx, N.ff1_up, ctx->s_xn32, (size_t) T * d), eps);
            ff1_done = true;
        } else {
            layernorm_f16(s, x, T, d, ctx->f(L.ln_out_w), ctx->f(L.ln_out_b), eps, xn, d, nullptr, y);
        }
        std::swap(x, y);
    }
    // keep the output in s_x so callers find it there
    if (x != ctx->s_x.as<float>()) {
        OWK_HIP_CHECK(hipMemcpyAsync(ctx->s_x.ptr, x, (size_t) T * d * 4, hipMemcpyDeviceToDevice, s));
        x = ctx->s_x.as<float>();
    }
    return x;
}
float * run_conformer(sortformer_context * ctx, float * x, int T, int last) { return run_conformer(ctx, x, Segs{{0, T}}, last); }

// projection 512 -> 192 from the f16 copy in s_xn -> s_t32 (f32) + s_t16 (f16)
void run_projection(sortformer_context * ctx, const _Float16 * x16, int T) {
    float * o32 = grow<float>(ctx->s_t32, (size_t) T * TF_D);
    _Float16 * o16 = grow<_Float16>(ctx->s_t16, (size_t) T * TF_D);
    EpiParams e;
    e.bias = ctx->f(ctx->proj_b); e.out32 = o32; e.out16 = o16; e.ldo = TF_D;
    sf_lin(ctx, EPI_BIAS_F32, T, TF_D, ctx->d_model, x16, nullptr, ctx->d_model, ctx->proj, e);
}

// transformer layers 0..last over s_t32 / s_t16 (in place) (ref:1467-1520)
void run_transformer(sortformer_context * ctx, const Segs & segs, int last) {
    int T = 0;
    for (const auto & sg : segs) T += sg.second;
    hipStream_t s = ctx->stream;
    float * x32 = ctx->s_t32.as<float>();
    _Float16 * x16 = ctx->s_t16.as<_Float16>();
    float * y = grow<float>(ctx->s_y, (size_t) T * TF_D);
    float * qkv = grow<float>(ctx->s_qkv, (size_t) T * 3 * TF_D);
    _Float16 * ao = grow<_Float16>(ctx->s_ao, (size_t) T * TF_D);
    _Float16 * hbuf = grow<_Float16>(ctx->s_h, (size_t) T * TF_FF);
    const float eps = 1e-5f;
    for (int il = 0; il <= last; ++il) {
        const TransLayer & L = ctx->trans[il];
        // x32 holds the f32 of x16 (the projection output, then each layer's final LayerNorm)
        EpiParams e;
        e.bias = ctx->f(L.qkv_b); e.out32 = qkv; e.ldo = 3 * TF_D;
        sf_lin(ctx, EPI_BIAS_F32, T, 3 * TF_D, TF_D, x16, x32, TF_D, L.qkv, e);
        float * ao32 = f32_for(ctx, L.out, ctx->s_ao32, (size_t) T * TF_D);
        for (const auto & sg : segs)
            sf::attention(s, TF_DH, false, qkv + (size_t) sg.first * 3 * TF_D, 3 * TF_D, TF_D, 2 * TF_D, sg.second, TF_H,
                          nullptr, nullptr, nullptr, 1.0f / sqrtf((float) TF_DH), ao + (size_t) sg.first * TF_D,
                          ao32 ? ao32 + (size_t) sg.first * TF_D : nullptr);
        EpiParams eo;
        eo.bias = ctx->f(L.out_b); eo.resid = x32; eo.out32 = y; eo.ldo = TF_D;
        sf_lin(ctx, EPI_RESID_F32, T, TF_D, TF_D, ao, ao32, TF_D, L.out, eo);
        layernorm_f16(s, y, T, TF_D, ctx->f(L.ln1_w), ctx->f(L.ln1_b), eps, x16, TF_D, nullptr, x32);
        float * h32 = f32_for(ctx, L.dn, ctx->s_h32, (size_t) T * TF_FF);
        EpiParams eu;
        eu.bias = ctx->f(L.up_b); eu.out16 = hbuf; eu.out32 = h32; eu.ldo = TF_FF;
        sf_lin(ctx, EPI_RELU_F16, T, TF_FF, TF_D, x16, x32, TF_D, L.up, eu);
        EpiParams ed;
        ed.bias = ctx->f(L.dn_b); ed.resid = x32; ed.out32 = y; ed.ldo = TF_D;
        sf_lin(ctx, EPI_RESID_F32, T, TF_D, TF_FF, hbuf, h32, TF_FF, L.dn, ed);
        layernorm_f16(s, y, T, TF_D, ctx->f(L.ln2_w), ctx->f(L.ln2_b), eps, x16, TF_D, nullptr, x32);
    }
}

void run_transformer(sortformer_context * ctx, int T, int last) { run_transformer(ctx, Segs{{0, T}}, last); }

// prediction head over s_t32 -> s_pred [T][4] (ref:1597-1612)
float * run_prediction(sortformer_context * ctx, int T) {
    hipStream_t s = ctx->stream;
    _Float16 * r16 = grow<_Float16>(ctx->s_ao, (size_t) T * TF_D);
    _Float16 * h16 = grow<_Float16>(ctx->s_h, (size_t) T * TF_D);
    float * pred = grow<float>(ctx->s_pred, (size_t) T * N_SPK);
    sf::relu_f16(s, ctx->s_t32.as<float>(), (size_t) T * TF_D, r16);
    EpiParams e;
    e.bias = ctx->f(ctx->hid_b); e.out16 = h16; e.ldo = TF_D;
    sf_lin(ctx, EPI_RELU_F16, T, TF_D, TF_D, r16, nullptr, TF_D, ctx->hid, e);
    EpiParams e2;
    e2.bias = ctx->f(ctx->spk_b); e2.out32 = pred; e2.ldo = N_SPK;
    sf_lin(ctx, EPI_SIGMOID_F32, T, N_SPK, TF_D, h16, nullptr, TF_D, ctx->spk, e2);
    return pred;
}

// the full head (sortformer_compute_streaming_prediction, ref:1924-2224) of a device input
// x [T][d] (f32, not yet xscaled; overwritten) -> host preds [T][4]
void run_head(sortformer_context * ctx, const Segs & segs, std::vector<float> & preds) {
    int T = 0;
    for (const auto & sg : segs) T += sg.second;
    float * x = ctx->s_x.as<float>();
    sf::scale(ctx->stream, x, (size_t) T * ctx->d_model, sqrtf((float) ctx->d_model), x);
    run_conformer(ctx, x, segs, ctx->n_conf - 1);
    run_projection(ctx, ctx->s_xn.as<_Float16>(), T);
    run_transformer(ctx, segs, ctx->n_trans - 1);
    float * p = run_prediction(ctx, T);
    preds.resize((size_t) T * N_SPK);
    OWK_HIP_CHECK(hipMemcpyAsync(preds.data(), p, preds.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
}

void run_head(sortformer_context * ctx, int T, std::vector<float> & preds) { run_head(ctx, Segs{{0, T}}, preds); }

// ---------------------------------------------------------------------------------
// streaming bookkeeping (host, ref:1729-1920)
// ---------------------------------------------------------------------------------
void update_silence_profile(StreamState & st, const StreamConfig & cfg, const float * pop_embs,
                            const float * pop_preds, int pop_len, int d) {
    for (int t = 0; t < pop_len; ++t) {
        float ps = 0;
        for (int s = 0; s < N_SPK; ++s) ps += pop_preds[t * N_SPK + s];
        if (ps < cfg.sil_threshold) {
            st.n_sil_frames++;
            const float w_old = (float) (st.n_sil_frames - 1) / (float) st.n_sil_frames;
            const float w_new = 1.0f / (float) st.n_sil_frames;
            // the reference as built (gcc contracts w_old * m + w_new * e into one fma on x86-64-v3/v4)
            for (int k = 0; k < d; ++k) st.mean_sil_emb[k] = fmaf(w_old, st.mean_sil_emb[k], w_new * pop_embs[t * d + k]);
        }
    }
}

void boost_topk(float * scores, int n_frames, int k, float scale_factor, float offset) {
    if (k <= 0 || k > n_frames) return;
    const float boost = -scale_factor * logf(offset);
    std::vector<std::pair<float, int>> sv(n_frames);
    for (int s = 0; s < N_SPK; ++s) {
        for (int t = 0; t < n_frames; ++t) sv[t] = {scores[t * N_SPK + s], t};
        std::nth_element(sv.begin(), sv.begin() + k, sv.end(),
                         [](const std::pair<float, int> & a, const std::pair<float, int> & b) { return a.first > b.first; });
        for (int i = 0; i < k; ++i) scores[sv[i].second * N_SPK + s] += boost;
    }
}

void compress_spkcache(StreamState & st, const StreamConfig & cfg, int d) {
    const int n_frames = st.spkcache_len;
    const int target = cfg.spkcache_len;
    const int per_spk = target / N_SPK - cfg.spkcache_sil_frames_per_spk;
    const int strong_k = (int) floor(per_spk * cfg.strong_boost_rate);
    const int weak_k = (int) floor(per_spk * cfg.weak_boost_rate);
    const int min_pos_k = (int) floor(per_spk * cfg.min_pos_scores_rate);

    std::vector<float> sc((size_t) n_frames * N_SPK);
    for (int t = 0; t < n_frames; ++t) {  // log-odds importance (ref:1799-1811)
        const float * p = &st.spkcache_preds[t * N_SPK];
        float l1sum = 0;
        for (int s = 0; s < N_SPK; ++s) l1sum += logf(fmaxf(1.0f - p[s], cfg.pred_score_threshold));
        for (int s = 0; s < N_SPK; ++s) {
            const float lp = logf(fmaxf(p[s], cfg.pred_score_threshold));
            const float l1p = logf(fmaxf(1.0f - p[s], cfg.pred_score_threshold));
            sc[t * N_SPK + s] = lp - l1p + l1sum - logf(0.5f);
        }
    }
    for (int t = 0; t < n_frames; ++t)
        for (int s = 0; s < N_SPK; ++s)
            if (st.spkcache_preds[t * N_SPK + s] <= 0.5f) sc[t * N_SPK + s] = -INFINITY;
    for (int s = 0; s < N_SPK; ++s) {
        int pos = 0;
        for (int t = 0; t < n_frames; ++t) pos += sc[t * N_SPK + s] > 0;
        if (pos >= min_pos_k)
            for (int t = 0; t < n_frames; ++t)
                if (sc[t * N_SPK + s] <= 0 && st.spkcache_preds[t * N_SPK + s] > 0.5f) sc[t * N_SPK + s] = -INFINITY;
    }
    if (cfg.scores_boost_latest > 0)
        for (int t = target; t < n_frames; ++t)
            for (int s = 0; s < N_SPK; ++s)
                if (sc[t * N_SPK + s] != -INFINITY) sc[t * N_SPK + s] += cfg.scores_boost_latest;
    boost_topk(sc.data(), n_frames, strong_k, 2.0f, 0.5f);
    boost_topk(sc.data(), n_frames, std::min(weak_k, n_frames), 1.0f, 0.5f);

    const int n_sil = cfg.spkcache_sil_frames_per_spk, n_total = n_frames + n_sil;
    sc.resize((size_t) n_total * N_SPK);
    for (int t = n_frames; t < n_total; ++t)
        for (int s = 0; s < N_SPK; ++s) sc[t * N_SPK + s] = INFINITY;
    std::vector<std::pair<float, int>> flat((size_t) N_SPK * n_total);  // (spk, frame) flattening (ref:1856-1863)
    for (int s = 0; s < N_SPK; ++s)
        for (int t = 0; t < n_total; ++t) flat[s * n_total + t] = {sc[t * N_SPK + s], s * n_total + t};
    std::nth_element(flat.begin(), flat.begin() + target, flat.end(),
                     [](const std::pair<float, int> & a, const std::pair<float, int> & b) { return a.first > b.first; });
    std::vector<int> idx(target);
    for (int i = 0; i < target; ++i) idx[i] = flat[i].first == -INFINITY ? cfg.max_index : flat[i].second;
    std::sort(idx.begin(), idx.end());
    std::vector<char> disabled(target, 0);
    for (int i = 0; i < target; ++i) {
        if (idx[i] == cfg.max_index) disabled[i] = 1;
        idx[i] = idx[i] % n_total;
        if (idx[i] >= n_frames) disabled[i] = 1;
        if (disabled[i]) idx[i] = 0;
    }
    std::vector<float> embs((size_t) target * d), preds((size_t) target * N_SPK);
    for (int i = 0; i < target; ++i) {
        if (disabled[i]) {
            memcpy(&embs[(size_t) i * d], st.mean_sil_emb.data(), d * 4);
            memset(&preds[(size_t) i * N_SPK], 0, N_SPK * 4);
        } else {
            memcpy(&embs[(size_t) i * d], &st.spkcache[(size_t) idx[i] * d], d * 4);
            memcpy(&preds[(size_t) i * N_SPK], &st.spkcache_preds[(size_t) idx[i] * N_SPK], N_SPK * 4);
        }
    }
    st.spkcache = std::move(embs);
    st.spkcache_preds = std::move(preds);
    st.spkcache_len = target;
}

int validate(const StreamConfig & c) {  // ref:2226-2265
    if (c.chunk_len < 1 || c.spkcache_update_period < 1 || c.fifo_len < 0 ||
        c.spkcache_len < (1 + c.spkcache_sil_frames_per_spk) * N_SPK || c.chunk_left_context < 0 ||
        c.chunk_right_context < 0)
        return -1;
    return 0;
}

// One chunk: pre-encode mel columns [c0, c0+n) of a device mel (row stride ld), run the head
// on [spkcache | fifo | chunk], append the chunk's predictions to `out`, and (update) advance
// the FIFO / speaker cache (ref:2349-2548; flush passes update = false, ref:3161-3249).
// Returns frames appended, or -1 (flush: chunk_len_used <= 0 stops the loop -> -2).
// one chunk of one stream: rows of its head input and the host copy of its pre-encoder output
struct ChunkWork {
    int Tc = 0, lc = 0, rc = 0, used = 0, T_total = 0;
    std::vector<float> chunk;
};

int chunk_rows(const sortformer_context * ctx, int n) { return conv_out(conv_out(conv_out(n))); }

// pre-encoder of mel frames [c0, c0 + n), then the head input [spkcache | fifo | chunk] written
// to x_dst (device rows, T_total of them)
void prep_chunk(sortformer_context * ctx, StreamState & st, const float * mel, int ld, int c0, int n, int left_offset,
                int right_offset, float * x_dst, ChunkWork & w) {
    const int d = ctx->d_model, sub = ctx->subsampling;
    w.lc = (int) round((double) left_offset / sub);
    w.rc = (int) ceil((double) right_offset / sub);
    w.Tc = run_preenc(ctx, mel, ld, c0, n);
    w.used = w.Tc - w.lc - w.rc;
    w.chunk.resize((size_t) w.Tc * d);
    OWK_HIP_CHECK(hipMemcpyAsync(w.chunk.data(), ctx->s_pre.ptr, w.chunk.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    w.T_total = st.spkcache_len + st.fifo_len + w.Tc;
    float * x = x_dst;
    if (st.spkcache_len > 0)
        OWK_HIP_CHECK(hipMemcpyAsync(x, st.spkcache.data(), (size_t) st.spkcache_len * d * 4, hipMemcpyHostToDevice, ctx->stream));
    if (st.fifo_len > 0)
        OWK_HIP_CHECK(hipMemcpyAsync(x + (size_t) st.spkcache_len * d, st.fifo.data(), (size_t) st.fifo_len * d * 4,
                                     hipMemcpyHostToDevice, ctx->stream));
    OWK_HIP_CHECK(hipMemcpyAsync(x + (size_t) (st.spkcache_len + st.fifo_len) * d, ctx->s_pre.ptr, (size_t) w.Tc * d * 4,
                                 hipMemcpyDeviceToDevice, ctx->stream));
    // no sync here: the copies are stream-ordered before the head pass, whose prediction
    // read-back synchronizes the stream before post_chunk touches st or w.chunk
}

int post_chunk(const sortformer_context * ctx, const StreamConfig & cfg, StreamState & st, ChunkWork & w,
               const std::vector<float> & pred, bool update, std::vector<float> & out);

int process_chunk(sortformer_context * ctx, const StreamConfig & cfg, StreamState & st, const float * mel, int ld,
                  int c0, int n, int left_offset, int right_offset, bool update, std::vector<float> & out) {
    const int d = ctx->d_model;
    const int Tc = chunk_rows(ctx, n);
    const int lc = (int) round((double) left_offset / ctx->subsampling);
    const int rc = (int) ceil((double) right_offset / ctx->subsampling);
    if (!update && Tc - lc - rc <= 0) return -2;
    ChunkWork w;
    float * x = grow<float>(ctx->s_x, (size_t) (st.spkcache_len + st.fifo_len + Tc) * d);
    prep_chunk(ctx, st, mel, ld, c0, n, left_offset, right_offset, x, w);
    std::vector<float> pred;
    run_head(ctx, w.T_total, pred);
    return post_chunk(ctx, cfg, st, w, pred, update, out);
}

// output rows and the FIFO / speaker-cache update of one chunk from its head predictions
int post_chunk(const sortformer_context * ctx, const StreamConfig & cfg, StreamState & st, ChunkWork & w,
               const std::vector<float> & pred, bool update, std::vector<float> & out) {
    const int d = ctx->d_model;
    const int lc = w.lc, used = w.used;
    const std::vector<float> & chunk = w.chunk;
    const int ps = st.spkcache_len + st.fifo_len + lc;
    if (used > 0) out.insert(out.end(), pred.begin() + (size_t) ps * N_SPK, pred.begin() + (size_t) (ps + used) * N_SPK);
    if (!update) return std::max(used, 0);

    // FIFO / speaker-cache update (sync mode, ref:2436-2542)
    const int old_sc = st.spkcache_len, old_fifo = st.fifo_len;
    st.fifo_preds.resize((size_t) old_fifo * N_SPK);
    if (old_fifo > 0) memcpy(st.fifo_preds.data(), pred.data() + (size_t) old_sc * N_SPK, (size_t) old_fifo * N_SPK * 4);
    const int nf = old_fifo + used;
    std::vector<float> uf((size_t) std::max(nf, 0) * d), ufp((size_t) std::max(nf, 0) * N_SPK);
    if (old_fifo > 0) {
        memcpy(uf.data(), st.fifo.data(), (size_t) old_fifo * d * 4);
        memcpy(ufp.data(), st.fifo_preds.data(), (size_t) old_fifo * N_SPK * 4);
    }
    if (used > 0) {
        memcpy(uf.data() + (size_t) old_fifo * d, chunk.data() + (size_t) lc * d, (size_t) used * d * 4);
        memcpy(ufp.data() + (size_t) old_fifo * N_SPK, pred.data() + (size_t) ps * N_SPK, (size_t) used * N_SPK * 4);
    }
    if (nf > cfg.fifo_len) {
        int pop = cfg.spkcache_update_period;
        pop = std::max(pop, used - cfg.fifo_len + old_fifo);
        pop = std::min(pop, nf);
        update_silence_profile(st, cfg, uf.data(), ufp.data(), pop, d);
        const int rem = nf - pop;
        st.fifo.assign(uf.begin() + (size_t) pop * d, uf.begin() + (size_t) nf * d);
        st.fifo_preds.assign(ufp.begin() + (size_t) pop * N_SPK, ufp.begin() + (size_t) nf * N_SPK);
        st.fifo_len = rem;
        const int new_sc = old_sc + pop;
        st.spkcache.resize((size_t) new_sc * d);
        memcpy(st.spkcache.data() + (size_t) old_sc * d, uf.data(), (size_t) pop * d * 4);
        if (st.spkcache_preds_valid) {
            st.spkcache_preds.resize((size_t) new_sc * N_SPK);
            memcpy(st.spkcache_preds.data() + (size_t) old_sc * N_SPK, ufp.data(), (size_t) pop * N_SPK * 4);
        }
        st.spkcache_len = new_sc;
        if (new_sc > cfg.spkcache_len) {
            if (!st.spkcache_preds_valid) {  // first compression: cache preds from this forward pass
                st.spkcache_preds.resize((size_t) new_sc * N_SPK);
                memcpy(st.spkcache_preds.data(), pred.data(), (size_t) old_sc * N_SPK * 4);
                memcpy(st.spkcache_preds.data() + (size_t) old_sc * N_SPK, ufp.data(), (size_t) pop * N_SPK * 4);
                st.spkcache_preds_valid = true;
            }
            compress_spkcache(st, cfg, d);
        }
    } else {
        st.fifo = std::move(uf);
        st.fifo_preds = std::move(ufp);
        st.fifo_len = nf;
    }
    return used;
}

StreamConfig config_from(const sortformer_params & p) {
    StreamConfig c;
    c.chunk_len = p.chunk_len;
    c.fifo_len = p.fifo_len;
    c.spkcache_len = p.spkcache_len;
    c.spkcache_update_period = p.spkcache_update_period;
    c.chunk_left_context = p.chunk_left_context;
    c.chunk_right_context = p.right_context;
    return c;
}
StreamConfig config_from(const sortformer_stream_params & p) {
    StreamConfig c;
    c.chunk_len = p.chunk_len;
    c.fifo_len = p.fifo_len;
    c.spkcache_len = p.spkcache_len;
    c.spkcache_update_period = p.spkcache_update_period;
    c.chunk_left_context = p.left_context;
    c.chunk_right_context = p.right_context;
    return c;
}

float * malloc_copy(const float * src, size_t n) {
    float * p = (float *) malloc(std::max<size_t>(n, 1) * sizeof(float));
    if (p && n) memcpy(p, src, n * sizeof(float));
    return p;
}

}  // namespace

// =================================================================================
// C ABI
// =================================================================================
extern "C" {

struct sortformer_params sortformer_default_params(void) {  // ref:269-281
    sortformer_params p;
    p.chunk_len = 188;
    p.right_context = 1;
    p.fifo_len = 0;
    p.spkcache_len = 188;
    p.spkcache_update_period = 188;
    p.threshold = 0.5f;
    p.median_filter = 11;
    p.n_threads = 4;
    p.chunk_left_context = 1;
    return p;
}

struct sortformer_context * sortformer_init(const char * model_path, struct sortformer_params params) {
    if (!model_path) return nullptr;
    std::unique_ptr<sortformer_context> ctx(new sortformer_context());
    try {
        int n_dev = 0;
        if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev <= 0) {
            fprintf(stderr, "sortformer_init: no HIP device\n");
            return nullptr;
        }
        OWK_HIP_CHECK(hipGetDevice(&ctx->device));
        Gguf g;
        std::string err;
        if (!g.load(model_path, err)) {
            fprintf(stderr, "sortformer_init: failed to open GGUF file '%s': %s\n", model_path, err.c_str());
            return nullptr;
        }
        auto u = [&](const char * k) -> int {
            auto it = g.u32.find(k);
            if (it == g.u32.end()) throw std::runtime_error(std::string("key '") + k + "' not found");
            return (int) it->second;
        };
        ctx->params = params;
        ctx->n_mels = u("sortformer.mel.n_mels");
        ctx->n_fft = u("sortformer.mel.n_fft");
        ctx->hop = u("sortformer.mel.hop_length");
        ctx->win_length = u("sortformer.mel.win_length");
        ctx->sample_rate = u("sortformer.mel.sample_rate");
        ctx->d_model = u("sortformer.encoder.d_model");
        ctx->subsampling = u("sortformer.encoder.subsampling_factor");
        if (ctx->n_fft != 512 || ctx->n_mels != 128 || ctx->hop != 160 || ctx->d_model != 512 || ctx->subsampling != 8)
            throw std::runtime_error("unsupported SortFormer hyper-parameters");
        ctx->n_conf = 17;  // fixed by the reference (ref:31, 87)
        ctx->n_trans = 18;
        dev_guard(ctx.get());
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        load_weights(ctx.get(), g);
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_init: %s\n", e.what());
        return nullptr;
    }
    return ctx.release();
}

void sortformer_free(struct sortformer_context * ctx) { delete ctx; }

int sortformer_load_wav(const char * path, float ** samples_out) {  // ref:652-773
    if (!path || !samples_out) return -1;
    FILE * f = fopen(path, "rb");
    if (!f) return -1;
    auto fail = [&]() { fclose(f); return -1; };
    char id[4];
    uint32_t sz;
    if (fread(id, 1, 4, f) != 4 || memcmp(id, "RIFF", 4) != 0) return fail();
    if (fread(&sz, 4, 1, f) != 1) return fail();
    if (fread(id, 1, 4, f) != 4 || memcmp(id, "WAVE", 4) != 0) return fail();
    uint16_t fmt = 0, ch = 0, bits = 0;
    uint32_t sr = 0, data_size = 0;
    bool have_fmt = false, have_data = false;
    while (!have_data) {
        if (fread(id, 1, 4, f) != 4 || fread(&sz, 4, 1, f) != 1) break;
        if (memcmp(id, "fmt ", 4) == 0) {
            if (sz < 16) return fail();
            if (fread(&fmt, 2, 1, f) != 1 || fread(&ch, 2, 1, f) != 1 || fread(&sr, 4, 1, f) != 1) return fail();
            fseek(f, 6, SEEK_CUR);
            if (fread(&bits, 2, 1, f) != 1) return fail();
            if (sz > 16) fseek(f, sz - 16, SEEK_CUR);
            have_fmt = true;
        } else if (memcmp(id, "data", 4) == 0) {
            data_size = sz;
            have_data = true;
        } else {
            fseek(f, sz, SEEK_CUR);
        }
    }
    if (!have_fmt || !have_data || fmt != 1 || ch != 1 || sr != 16000 || bits != 16) return fail();
    const int n = (int) (data_size / 2);
    std::vector<int16_t> raw(n);
    if ((int) fread(raw.data(), 2, n, f) != n) return fail();
    fclose(f);
    float * out = (float *) malloc((size_t) std::max(n, 1) * sizeof(float));
    if (!out) return -1;
    for (int i = 0; i < n; ++i) out[i] = (float) raw[i] / 32768.0f;
    *samples_out = out;
    return n;
}

int sortformer_compute_mel(struct sortformer_context * ctx, const float * samples, int n_samples, float ** mel_out,
                           int * n_mels_out, int * seq_len_out) {
    if (!ctx || !samples || n_samples <= 0 || !mel_out || !n_mels_out) return -1;
    try {
        dev_guard(ctx);
        const MelDims md = run_mel(ctx, samples, n_samples);
        const size_t n = (size_t) ctx->n_mels * md.n_frames_out;
        float * out = (float *) malloc(std::max<size_t>(n, 1) * 4);
        if (!out) return -1;
        OWK_HIP_CHECK(hipMemcpyAsync(out, ctx->s_mel.ptr, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        *mel_out = out;
        *n_mels_out = ctx->n_mels;
        if (seq_len_out) *seq_len_out = md.seq_len;
        return md.n_frames_out;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_compute_mel: %s\n", e.what());
        return -1;
    }
}

int sortformer_compute_preenc(struct sortformer_context * ctx, const float * mel_data, int n_mels, int n_mel_frames,
                              int seq_len, float ** preenc_out, int * d_model_out) {
    if (!ctx || !mel_data || !preenc_out || !d_model_out) return -1;
    if (n_mels != ctx->n_mels || seq_len <= 0 || seq_len > n_mel_frames) return -1;
    try {
        dev_guard(ctx);
        float * mel = grow<float>(ctx->s_mel, (size_t) n_mels * n_mel_frames);
        OWK_HIP_CHECK(hipMemcpyAsync(mel, mel_data, (size_t) n_mels * n_mel_frames * 4, hipMemcpyHostToDevice, ctx->stream));
        const int T = run_preenc(ctx, mel, n_mel_frames, 0, seq_len);
        std::vector<float> h((size_t) T * ctx->d_model);
        OWK_HIP_CHECK(hipMemcpyAsync(h.data(), ctx->s_pre.ptr, h.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        *preenc_out = malloc_copy(h.data(), h.size());
        *d_model_out = ctx->d_model;
        return T;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_compute_preenc: %s\n", e.what());
        return -1;
    }
}

int sortformer_compute_conformer(struct sortformer_context * ctx, const float * preenc_data, int T, int d_model,
                                 int target_layer, float ** conf_out) {
    if (!ctx || !preenc_data || !conf_out || T <= 0 || d_model != ctx->d_model) return -1;
    if (target_layer < 0 || target_layer >= ctx->n_conf) return -1;
    try {
        dev_guard(ctx);
        float * x = grow<float>(ctx->s_x, (size_t) T * d_model);
        OWK_HIP_CHECK(hipMemcpyAsync(x, preenc_data, (size_t) T * d_model * 4, hipMemcpyHostToDevice, ctx->stream));
        sf::scale(ctx->stream, x, (size_t) T * d_model, sqrtf((float) d_model), x);
        float * out = run_conformer(ctx, x, T, target_layer);
        std::vector<float> h((size_t) T * d_model);
        OWK_HIP_CHECK(hipMemcpyAsync(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        *conf_out = malloc_copy(h.data(), h.size());
        return T;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_compute_conformer: %s\n", e.what());
        return -1;
    }
}

int sortformer_compute_projection(struct sortformer_context * ctx, const float * conf_data, int T, int d_model_in,
                                  float ** proj_out, int * d_model_out_ptr) {
    if (!ctx || !conf_data || !proj_out || !d_model_out_ptr || T <= 0 || d_model_in != ctx->d_model) return -1;
    try {
        dev_guard(ctx);
        float * x = grow<float>(ctx->s_x, (size_t) T * d_model_in);
        _Float16 * x16 = grow<_Float16>(ctx->s_xn, (size_t) T * d_model_in);
        OWK_HIP_CHECK(hipMemcpyAsync(x, conf_data, (size_t) T * d_model_in * 4, hipMemcpyHostToDevice, ctx->stream));
        sf::to_f16(ctx->stream, x, (size_t) T * d_model_in, x16);
        run_projection(ctx, x16, T);
        std::vector<float> h((size_t) T * TF_D);
        OWK_HIP_CHECK(hipMemcpyAsync(h.data(), ctx->s_t32.ptr, h.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        *proj_out = malloc_copy(h.data(), h.size());
        *d_model_out_ptr = TF_D;
        return T;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_compute_projection: %s\n", e.what());
        return -1;
    }
}

int sortformer_compute_transformer(struct sortformer_context * ctx, const float * proj_data, int T, int d_model,
                                   int target_layer, float ** trans_out) {
    if (!ctx || !proj_data || !trans_out || T <= 0 || d_model != TF_D) return -1;
    if (target_layer < 0 || target_layer >= ctx->n_trans) return -1;
    try {
        dev_guard(ctx);
        float * x32 = grow<float>(ctx->s_t32, (size_t) T * TF_D);
        _Float16 * x16 = grow<_Float16>(ctx->s_t16, (size_t) T * TF_D);
        OWK_HIP_CHECK(hipMemcpyAsync(x32, proj_data, (size_t) T * TF_D * 4, hipMemcpyHostToDevice, ctx->stream));
        sf::to_f16(ctx->stream, x32, (size_t) T * TF_D, x16);
        run_transformer(ctx, T, target_layer);
        std::vector<float> h((size_t) T * TF_D);
        OWK_HIP_CHECK(hipMemcpyAsync(h.data(), ctx->s_t32.ptr, h.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        *trans_out = malloc_copy(h.data(), h.size());
        return T;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_compute_transformer: %s\n", e.what());
        return -1;
    }
}

int sortformer_compute_prediction(struct sortformer_context * ctx, const float * trans_data, int T, int d_model,
                                  float ** pred_out) {
    if (!ctx || !trans_data || !pred_out || T <= 0 || d_model != TF_D) return -1;
    try {
        dev_guard(ctx);
        float * x32 = grow<float>(ctx->s_t32, (size_t) T * TF_D);
        OWK_HIP_CHECK(hipMemcpyAsync(x32, trans_data, (size_t) T * TF_D * 4, hipMemcpyHostToDevice, ctx->stream));
        float * p = run_prediction(ctx, T);
        std::vector<float> h((size_t) T * N_SPK);
        OWK_HIP_CHECK(hipMemcpyAsync(h.data(), p, h.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        *pred_out = malloc_copy(h.data(), h.size());
        return T;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_compute_prediction: %s\n", e.what());
        return -1;
    }
}

int sortformer_diarize(struct sortformer_context * ctx, const float * audio_samples, int n_samples, float * probs_out,
                       int n_frames_max) {
    if (!ctx || !audio_samples || n_samples <= 0 || !probs_out || n_frames_max <= 0) return -1;
    const StreamConfig cfg = config_from(ctx->params);
    if (validate(cfg) != 0) return -1;
    try {
        dev_guard(ctx);
        // the whole-clip mel stays on the device; chunks read column windows of it
        const MelDims md = run_mel(ctx, audio_samples, n_samples);
        const float * mel = ctx->s_mel.as<float>();
        StreamState st(ctx->d_model);
        const int feat_len = md.seq_len, sub = ctx->subsampling;
        std::vector<float> total;
        for (int stt = 0; stt < feat_len;) {  // chunk loop (ref:2328-2549)
            const int end = std::min(stt + cfg.chunk_len * sub, feat_len);
            const int lo = std::min(cfg.chunk_left_context * sub, stt);
            const int ro = std::min(cfg.chunk_right_context * sub, feat_len - end);
            process_chunk(ctx, cfg, st, mel, md.n_frames_out, stt - lo, end + ro - (stt - lo), lo, ro,
                          true, total);
            stt = end;
        }
        const int n_frames = (int) (total.size() / N_SPK);
        const int n_out = std::min(n_frames, n_frames_max);
        memcpy(probs_out, total.data(), (size_t) n_out * N_SPK * 4);
        return n_out;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_diarize: %s\n", e.what());
        return -1;
    }
}

int sortformer_to_rttm(const float * probs, int n_frames, float threshold, int median_filter, const char * filename,
                       char * rttm_out, int rttm_out_size) {  // ref:2593-2669
    if (!probs || n_frames <= 0 || !rttm_out || rttm_out_size <= 0) return -1;
    std::string name = filename ? filename : "unknown";
    const size_t slash = name.find_last_of("/\\");
    if (slash != std::string::npos) name = name.substr(slash + 1);
    const size_t dot = name.rfind('.');
    if (dot != std::string::npos) name = name.substr(0, dot);
    std::vector<uint8_t> bin((size_t) n_frames * N_SPK);
    for (size_t i = 0; i < bin.size(); ++i) bin[i] = probs[i] > threshold ? 1 : 0;
    if (median_filter > 1) {  // binary majority filter, zero padded (ref:2572-2591)
        const int half = median_filter / 2;
        std::vector<uint8_t> col(n_frames);
        for (int s = 0; s < N_SPK; ++s) {
            for (int t = 0; t < n_frames; ++t) col[t] = bin[(size_t) t * N_SPK + s];
            for (int t = 0; t < n_frames; ++t) {
                int ones = 0;
                for (int j = t - half; j < t - half + median_filter; ++j)
                    if (j >= 0 && j < n_frames) ones += col[j];
                bin[(size_t) t * N_SPK + s] = ones * 2 > median_filter ? 1 : 0;
            }
        }
    }
    const float frame_dur = 0.08f;
    int written = 0;
    for (int s = 0; s < N_SPK; ++s) {
        int start = -1;
        for (int t = 0; t <= n_frames; ++t) {
            const bool on = t < n_frames && bin[(size_t) t * N_SPK + s];
            if (on && start < 0) {
                start = t;
            } else if (!on && start >= 0) {
                const float t0 = start * frame_dur, dur = (t - start) * frame_dur;
                const int n = snprintf(rttm_out + written, rttm_out_size - written,
                                       "SPEAKER %s 1 %.2f %.2f <NA> <NA> speaker_%d <NA> <NA>\n", name.c_str(), t0, dur, s);
                if (n < 0 || written + n >= rttm_out_size) return -1;
                written += n;
                start = -1;
            }
        }
    }
    return written;
}

struct sortformer_stream_params sortformer_stream_preset_params(enum sortformer_stream_preset preset) {
    sortformer_stream_params p;  // ref:2708-2730
    switch (preset) {
        case SORTFORMER_PRESET_LOW_LATENCY: p = {6, 7, 1, 188, 188, 144}; break;
        case SORTFORMER_PRESET_2S: p = {15, 10, 1, 100, 188, 144}; break;
        case SORTFORMER_PRESET_3S: p = {30, 7, 1, 100, 188, 100}; break;
        case SORTFORMER_PRESET_5S:
        default: p = {55, 7, 1, 100, 188, 100}; break;
    }
    return p;
}

struct sortformer_stream_state * sortformer_stream_init(struct sortformer_context * ctx,
                                                        enum sortformer_stream_preset preset) {
    return sortformer_stream_init_with_params(ctx, sortformer_stream_preset_params(preset));
}

struct sortformer_stream_state * sortformer_stream_init_with_params(struct sortformer_context * ctx,
                                                                    struct sortformer_stream_params params) {
    if (!ctx) return nullptr;
    const StreamConfig cfg = config_from(params);
    if (validate(cfg) != 0) return nullptr;
    auto * s = new sortformer_stream_state();
    s->ctx = ctx;
    s->cfg = cfg;
    s->st = StreamState(ctx->d_model);
    return s;
}

}  // extern "C"

namespace {

// the mel half of a feed (ref:2776-2890): overlap + new samples -> mel with fresh zero
// padding (the reference's feed-boundary quirk), appended to the buffered frames; the
// chunks [c0, c0 + n) with their context offsets that are complete
struct FeedPlan {
    std::vector<float> cm;  // [n_mels][tot]
    int tot = 0, stt = 0;
    struct Chunk {
        int c0, n, lo, ro;
    };
    std::vector<Chunk> chunks;
};

FeedPlan feed_plan(sortformer_stream_state * sst, const float * audio_samples, int n_samples) {
    sortformer_context * ctx = sst->ctx;
    FeedPlan fp;
    const int64_t before = sst->total_samples_fed;
    sst->total_samples_fed += n_samples;
    const int n_mels = ctx->n_mels, sub = ctx->subsampling;
    std::vector<float> audio(sst->audio_overlap);
    audio.insert(audio.end(), audio_samples, audio_samples + n_samples);
    const int total_len = (int) audio.size();
    const MelDims md = run_mel(ctx, audio.data(), total_len);
    std::vector<float> mel((size_t) n_mels * md.n_frames_out);
    OWK_HIP_CHECK(hipMemcpyAsync(mel.data(), ctx->s_mel.ptr, mel.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    OWK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const int ov = ctx->n_fft - ctx->hop;
    if (total_len > ov) sst->audio_overlap.assign(audio.end() - ov, audio.end());
    else sst->audio_overlap = audio;
    int new_frames = (int) (sst->total_samples_fed / ctx->hop) - (int) (std::max<int64_t>(before, 0) / ctx->hop);
    new_frames = std::max(0, std::min(new_frames, md.seq_len));
    const int skip = md.seq_len - new_frames;
    const int tot = sst->mel_buffer_frames + new_frames;
    fp.tot = tot;
    fp.cm.resize((size_t) n_mels * tot);
    for (int m = 0; m < n_mels; ++m) {
        if (sst->mel_buffer_frames)
            memcpy(&fp.cm[(size_t) m * tot], &sst->mel_buffer[(size_t) m * sst->mel_buffer_frames], (size_t) sst->mel_buffer_frames * 4);
        if (new_frames)
            memcpy(&fp.cm[(size_t) m * tot + sst->mel_buffer_frames], &mel[(size_t) m * md.n_frames_out + skip], (size_t) new_frames * 4);
    }
    int stt = 0;
    const int min_chunk = sst->cfg.chunk_len * sub + sst->cfg.chunk_right_context * sub;
    while (tot > 0 && stt < tot) {
        if (tot - stt < min_chunk) break;
        const int end = std::min(stt + sst->cfg.chunk_len * sub, tot);
        const int lo = std::min(sst->cfg.chunk_left_context * sub, stt);
        const int ro = std::min(sst->cfg.chunk_right_context * sub, tot - end);
        fp.chunks.push_back({stt - lo, end + ro - (stt - lo), lo, ro});
        stt = end;
    }
    fp.stt = stt;
    return fp;
}

// keep the incomplete tail frames, hand out the predictions (ref:3090-3112)
int feed_finish(sortformer_stream_state * sst, const FeedPlan & fp, const std::vector<float> & out, float * probs_out,
                int probs_out_max) {
    const int n_mels = sst->ctx->n_mels, tot = fp.tot, stt = fp.stt;
    const int rem = tot - stt;
    if (rem > 0) {
        std::vector<float> mb((size_t) n_mels * rem);
        for (int m = 0; m < n_mels; ++m) memcpy(&mb[(size_t) m * rem], &fp.cm[(size_t) m * tot + stt], (size_t) rem * 4);
        sst->mel_buffer = std::move(mb);
        sst->mel_buffer_frames = rem;
    } else {
        sst->mel_buffer.clear();
        sst->mel_buffer_frames = 0;
    }
    const int n_out = std::min((int) (out.size() / N_SPK), probs_out_max);
    if (n_out > 0) memcpy(probs_out, out.data(), (size_t) n_out * N_SPK * 4);
    sst->total_frames_output += n_out;
    return n_out;
}

} // namespace

extern "C" {

int sortformer_stream_feed(struct sortformer_stream_state * sst, const float * audio_samples, int n_samples,
                           float * probs_out, int probs_out_max) {  // ref:2776-3113
    if (!sst || !audio_samples || n_samples <= 0 || !probs_out || probs_out_max <= 0) return -1;
    sortformer_context * ctx = sst->ctx;
    try {
        dev_guard(ctx);
        FeedPlan fp = feed_plan(sst, audio_samples, n_samples);
        std::vector<float> out;
        if (!fp.chunks.empty()) {
            float * dm = grow<float>(ctx->s_mel, fp.cm.size());
            OWK_HIP_CHECK(hipMemcpyAsync(dm, fp.cm.data(), fp.cm.size() * 4, hipMemcpyHostToDevice, ctx->stream));
            for (const auto & c : fp.chunks)
                process_chunk(ctx, sst->cfg, sst->st, dm, fp.tot, c.c0, c.n, c.lo, c.ro, true, out);
        }
        return feed_finish(sst, fp, out, probs_out, probs_out_max);
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_stream_feed: %s\n", e.what());
        return -1;
    }
}

// host-only AOSC bookkeeping test hook (include/owk_sortformer.h): the silence-profile update of
// popped FIFO frames, then the speaker-cache compression, exactly as the streaming feed runs them
int owk_sortformer_debug_aosc(int d, int n_frames, const float * embs, const float * preds, const float * mean_sil,
                              int n_sil, int n_pop, const float * pop_embs, const float * pop_preds, int spkcache_len,
                              int sil_frames_per_spk, float * out_embs, float * out_preds, float * out_mean_sil) {
    StreamConfig cfg;
    cfg.spkcache_len = spkcache_len;
    cfg.spkcache_sil_frames_per_spk = sil_frames_per_spk;
    if (d <= 0 || n_frames < 0 || n_pop < 0 || n_sil < 0 || !mean_sil || !out_mean_sil || validate(cfg) != 0 ||
        (n_frames > 0 && (!embs || !preds)) || (n_pop > 0 && (!pop_embs || !pop_preds)) ||
        (n_frames > spkcache_len && (!out_embs || !out_preds)))
        return -2;
    StreamState st(d);
    st.spkcache.assign(embs, embs + (size_t) n_frames * d);
    st.spkcache_preds.assign(preds, preds + (size_t) n_frames * N_SPK);
    st.spkcache_len = n_frames;
    st.spkcache_preds_valid = true;
    st.mean_sil_emb.assign(mean_sil, mean_sil + d);
    st.n_sil_frames = n_sil;
    if (n_pop > 0) update_silence_profile(st, cfg, pop_embs, pop_preds, n_pop, d);
    std::copy(st.mean_sil_emb.begin(), st.mean_sil_emb.end(), out_mean_sil);
    if (n_frames <= spkcache_len) return -1;
    compress_spkcache(st, cfg, d);
    std::copy(st.spkcache.begin(), st.spkcache.end(), out_embs);
    std::copy(st.spkcache_preds.begin(), st.spkcache_preds.end(), out_preds);
    return st.spkcache_len;
}

// Many live streams of one context fed together (owk.h): their chunks are processed in
// rounds -- round r holds the r-th pending chunk of every stream -- and each round is ONE
// head pass over the stacked [spkcache | fifo | chunk] rows of all its streams. Per stream
// the chunk order, the AOSC bookkeeping and the outputs are those of sortformer_stream_feed.
int owk_sortformer_stream_feed_batch(struct sortformer_stream_state ** ssts, const float * const * samples,
                                     const int * n_samples, int n_streams, float * const * probs_out,
                                     const int * probs_out_max, int * n_out) {
    if (!ssts || n_streams <= 0 || !samples || !n_samples || !probs_out || !probs_out_max || !n_out) return -1;
    sortformer_context * ctx = ssts[0]->ctx;
    for (int i = 0; i < n_streams; ++i) {
        if (!ssts[i] || ssts[i]->ctx != ctx || !samples[i] || n_samples[i] <= 0 || !probs_out[i] || probs_out_max[i] <= 0)
            return -1;
        for (int j = 0; j < i; ++j)
            if (ssts[j] == ssts[i]) return -1;  // a stream's chunks are sequential: once per batch
    }
    try {
        dev_guard(ctx);
        const int d = ctx->d_model;
        std::vector<FeedPlan> plans(n_streams);
        size_t mel_tot = 0;
        std::vector<size_t> mel_off(n_streams);
        size_t rounds = 0;
        for (int i = 0; i < n_streams; ++i) {
            plans[i] = feed_plan(ssts[i], samples[i], n_samples[i]);
            mel_off[i] = mel_tot;
            mel_tot += plans[i].cm.size();
            rounds = std::max(rounds, plans[i].chunks.size());
        }
        DevBuf dmel;
        dmel.alloc(std::max<size_t>(mel_tot, 1) * 4);
        for (int i = 0; i < n_streams; ++i)
            if (!plans[i].cm.empty())
                OWK_HIP_CHECK(hipMemcpyAsync(dmel.as<float>() + mel_off[i], plans[i].cm.data(), plans[i].cm.size() * 4,
                                             hipMemcpyHostToDevice, ctx->stream));
        std::vector<std::vector<float>> outs(n_streams);
        for (size_t r = 0; r < rounds; ++r) {
            std::vector<int> who;
            Segs segs;
            int rows = 0;
            for (int i = 0; i < n_streams; ++i) {
                if (r >= plans[i].chunks.size()) continue;
                const StreamState & st = ssts[i]->st;
                const int T = st.spkcache_len + st.fifo_len + chunk_rows(ctx, plans[i].chunks[r].n);
                who.push_back(i);
                segs.push_back({rows, T});
                rows += T;
            }
            float * x = grow<float>(ctx->s_x, (size_t) rows * d);
            std::vector<ChunkWork> works(who.size());
            for (size_t k = 0; k < who.size(); ++k) {
                const int i = who[k];
                const auto & c = plans[i].chunks[r];
                prep_chunk(ctx, ssts[i]->st, dmel.as<float>() + mel_off[i], plans[i].tot, c.c0, c.n, c.lo, c.ro,
                           x + (size_t) segs[k].first * d, works[k]);
            }
            std::vector<float> pred_all;
            run_head(ctx, segs, pred_all);
            for (size_t k = 0; k < who.size(); ++k) {
                const int i = who[k];
                std::vector<float> pred(pred_all.begin() + (size_t) segs[k].first * N_SPK,
                                        pred_all.begin() + (size_t) (segs[k].first + segs[k].second) * N_SPK);
                post_chunk(ctx, ssts[i]->cfg, ssts[i]->st, works[k], pred, true, outs[i]);
            }
        }
        for (int i = 0; i < n_streams; ++i) n_out[i] = feed_finish(ssts[i], plans[i], outs[i], probs_out[i], probs_out_max[i]);
        return 0;
    } catch (const std::exception & e) {
        fprintf(stderr, "owk_sortformer_stream_feed_batch: %s\n", e.what());
        return -1;
    }
}

int sortformer_stream_flush(struct sortformer_stream_state * sst, float * probs_out, int probs_out_max) {
    if (!sst || !probs_out || probs_out_max <= 0) return 0;  // ref:3115-3264
    if (sst->mel_buffer_frames == 0 && sst->audio_overlap.empty()) return 0;
    if (sst->mel_buffer_frames == 0) return 0;
    sortformer_context * ctx = sst->ctx;
    try {
        dev_guard(ctx);
        const int tot = sst->mel_buffer_frames, sub = ctx->subsampling;
        float * dm = grow<float>(ctx->s_mel, sst->mel_buffer.size());
        OWK_HIP_CHECK(hipMemcpyAsync(dm, sst->mel_buffer.data(), sst->mel_buffer.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        std::vector<float> out;
        for (int stt = 0; stt < tot;) {
            const int end = std::min(stt + sst->cfg.chunk_len * sub, tot);
            const int lo = std::min(sst->cfg.chunk_left_context * sub, stt);
            const int ro = std::min(sst->cfg.chunk_right_context * sub, tot - end);
            const int n = end + ro - (stt - lo);
            if (n < sub) break;
            // remaining chunks run WITHOUT updating the speaker cache / FIFO (ref:3161-3249)
            if (process_chunk(ctx, sst->cfg, sst->st, dm, tot, stt - lo, n, lo, ro, false, out) == -2) break;
            stt = end;
        }
        sst->mel_buffer.clear();
        sst->mel_buffer_frames = 0;
        sst->audio_overlap.clear();
        const int n_out = std::min((int) (out.size() / N_SPK), probs_out_max);
        if (n_out > 0) memcpy(probs_out, out.data(), (size_t) n_out * N_SPK * 4);
        sst->total_frames_output += n_out;
        return n_out;
    } catch (const std::exception & e) {
        fprintf(stderr, "sortformer_stream_flush: %s\n", e.what());
        return -1;
    }
}

void sortformer_stream_reset(struct sortformer_stream_state * sst) {
    if (!sst) return;
    sst->st = StreamState(sst->ctx->d_model);
    sst->audio_overlap.clear();
    sst->mel_buffer.clear();
    sst->mel_buffer_frames = 0;
    sst->total_samples_fed = 0;
    sst->total_frames_output = 0;
}

void sortformer_stream_free(struct sortformer_stream_state * sst) { delete sst; }

}  // extern "C"
