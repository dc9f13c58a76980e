// Batch-major device engine (see engine.h).
#include "engine.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace owk {

// ------------------------------------------------------------------------------------
// profiling
// ------------------------------------------------------------------------------------
int Prof::cls_id(const char * name) {
    for (size_t i = 0; i < names.size(); ++i)
        if (names[i] == name) return (int) i;
    names.push_back(name);
    tot.emplace_back();
    return (int) names.size() - 1;
}

hipEvent_t Prof::ev() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e;
    OWK_HIP_CHECK(hipEventCreate(&e));
    return e;
}

void Prof::flush() {
    for (auto & r : pending) {
        OWK_HIP_CHECK(hipEventSynchronize(r.b));
        float ms = 0.f;
        OWK_HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
        Tot & t = tot[r.cls];
        t.ms += ms;
        t.flops += r.flops;
        t.bytes += r.bytes;
        t.n += 1;
        pool.push_back(r.a);
        pool.push_back(r.b);
    }
    pending.clear();
}

void Prof::reset() {
    flush();
    for (auto & t : tot) t = Tot{};
}

Prof::~Prof() {
    for (auto & r : pending) {
        (void) hipEventDestroy(r.a);
        (void) hipEventDestroy(r.b);
    }
    for (auto e : pool) (void) hipEventDestroy(e);
}

ProfScope::ProfScope(Prof * p_, hipStream_t s_, const char * name, double flops_, double bytes_)
    : p(p_), s(s_), flops(flops_), bytes(bytes_) {
    if (!p || !p->on) return;
    cls = p->cls_id(name);
    a = p->ev();
    OWK_HIP_CHECK(hipEventRecord(a, s));
}

ProfScope::~ProfScope() {
    if (cls < 0) return;
    hipEvent_t b = p->ev();
    (void) hipEventRecord(b, s);
    p->pending.push_back({cls, a, b, flops, bytes});
    if (p->pending.size() > 4096) p->flush();
}

// ------------------------------------------------------------------------------------
// engine
// ------------------------------------------------------------------------------------
Engine::Engine(const Model * m_, Prof * prof_) : m(m_), prof(prof_) {
    OWK_HIP_CHECK(hipSetDevice(m->device));
    OWK_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    // split-K workspace for every decoder GEMM shape (K = d or 4d; N up to n_vocab)
    const HParams & hp = m->hp;
    const int d = hp.n_text_state, nv = hp.n_vocab;
    size_t fl = 0;
    for (int N : {3 * d, d, 4 * d, nv})
        for (int K : {d, 4 * d}) fl = std::max(fl, gemm_ws_floats(N, K));
    const int tickets = (std::max(4 * d, nv) + 15) / 16;
    gws_part_.alloc(std::max<size_t>(fl, 1) * 4);
    gws_tick_.alloc((size_t) tickets * 4);
    OWK_HIP_CHECK(hipMemsetAsync(gws_tick_.ptr, 0, (size_t) tickets * 4, stream));
    gws_.partial = gws_part_.as<float>();
    gws_.partial_floats = fl;
    gws_.tickets = gws_tick_.as<int>();
    gws_.n_tickets = tickets;
}

Engine::~Engine() {
    for (auto * b : mel_) delete b;
    if (stream) (void) hipStreamDestroy(stream);
}

void Engine::sync() { OWK_HIP_CHECK(hipStreamSynchronize(stream)); }

void Engine::reserve(int slots, int cells) {
    const HParams & hp = m->hp;
    const size_t d = hp.n_text_state;
    if (slots > cap_slots) {
        sync();
        cap_slots = slots;
        const size_t n = (size_t) hp.n_text_layer * cap_slots * hp.n_audio_ctx * d * 2;
        cross_k_.alloc(n);
        cross_v_.alloc(n);
        kv_cells = 0;  // force self-KV re-allocation with the new slot count
    }
    if (cells > kv_cells) {
        sync();
        kv_cells = cells;
        const size_t n = (size_t) hp.n_text_layer * cap_slots * kv_cells * d * 2;
        self_k_.alloc(n);
        self_v_.alloc(n);
        OWK_HIP_CHECK(hipMemsetAsync(self_k_.ptr, 0, n, stream));
        OWK_HIP_CHECK(hipMemsetAsync(self_v_.ptr, 0, n, stream));
    }
    while ((int) mel_.size() < cap_slots) {
        mel_.push_back(new DevBuf());
        mel_len_.push_back(0);
    }
}

void Engine::compute_mel(const std::vector<int> & slots, const std::vector<const float *> & pcm,
                         const std::vector<int> & n_samples, bool pcm_on_device) {
    const int n = (int) slots.size();
    if (n == 0) return;
    const int n_mel = m->n_filters_mel;
    size_t total_pcm = 0;
    for (int i = 0; i < n; ++i) total_pcm += (size_t) n_samples[i];
    if (!pcm_on_device) pcm_tmp_.alloc(std::max<size_t>(total_pcm, 1) * 4);
    std::vector<MelJob> jobs(n);
    size_t at = 0;
    int max_frames = 0;
    for (int i = 0; i < n; ++i) {
        const int s = slots[i];
        const int n_len = (n_samples[i] + 480000) / 160;  // (padded - 400) / 160 with 200+200 pad
        DevBuf * b = mel_[s];
        b->alloc((size_t) n_mel * n_len * 4);
        mel_len_[s] = n_len;
        const float * src = pcm[i];
        if (!pcm_on_device) {
            OWK_HIP_CHECK(hipMemcpyAsync(pcm_tmp_.as<float>() + at, pcm[i], (size_t) n_samples[i] * 4,
                                         hipMemcpyHostToDevice, stream));
            src = pcm_tmp_.as<float>() + at;
        }
        jobs[i] = MelJob{src, n_samples[i], n_len, b->as<float>()};
        at += n_samples[i];
        max_frames = std::max(max_frames, n_len);
    }
    mel_jobs_.alloc(sizeof(MelJob) * n);
    OWK_HIP_CHECK(hipMemcpyAsync(mel_jobs_.ptr, jobs.data(), sizeof(MelJob) * n, hipMemcpyHostToDevice, stream));
    {
        ProfScope ps(prof, stream, "mel");
        mel_spectrogram(stream, mel_jobs_.as<MelJob>(), n, max_frames, m->mel_filters, n_mel, m->twiddle, m->hann);
        mel_normalize(stream, mel_jobs_.as<MelJob>(), n, n_mel);
    }
    sync();  // pcm host buffers may go away after return
}

void Engine::set_mel(int slot, const float * host, int n_len, int n_mel) {
    DevBuf * b = mel_[slot];
    b->alloc((size_t) n_mel * n_len * 4);
    mel_len_[slot] = n_len;
    OWK_HIP_CHECK(hipMemcpy(b->ptr, host, (size_t) n_mel * n_len * 4, hipMemcpyHostToDevice));
}

void Engine::download_mel(int slot, float * host) const {
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    OWK_HIP_CHECK(hipMemcpy(host, mel_[slot]->ptr, (size_t) m->n_filters_mel * mel_len_[slot] * 4, hipMemcpyDeviceToHost));
}

static double gemm_flops(double M, double N, double K) { return 2.0 * M * N * K; }

void Engine::encode(const std::vector<int> & slots, const std::vector<int> & offsets) {
    const HParams & hp = m->hp;
    const int n = (int) slots.size();
    if (n == 0) return;
    const int T = hp.n_audio_ctx, T2 = 2 * T, d = hp.n_audio_state, H = hp.n_audio_head;
    const int Tpad = (T + 63) / 64 * 64;
    const int n_ctx_pad = (T + 255) / 256 * 256;  // GGML_PAD(n_audio_ctx, 256)
    const int n_zero_pad = n_ctx_pad - T;
    const int M = n * T;
    const int kp1 = m->kpad_conv1;

    if (M > enc_rows_cap_) {
        sync();
        enc_rows_cap_ = M;
        e_a1_.alloc((size_t) n * T2 * kp1 * 2);
        e_c1_.alloc((size_t) n * T2 * d * 2);
        e_a2_.alloc((size_t) M * 3 * d * 2);
        e_x_.alloc((size_t) M * d * 4);
        e_xn_.alloc((size_t) M * d * 2);
        e_q_.alloc((size_t) M * d * 2);
        e_k_.alloc((size_t) M * d * 2);
        e_vt_.alloc((size_t) n * H * 64 * Tpad * 2);
        OWK_HIP_CHECK(hipMemsetAsync(e_vt_.ptr, 0, e_vt_.bytes, stream));  // padded key columns stay 0
        e_ao_.alloc((size_t) M * d * 2);
        e_h_.alloc((size_t) M * 4 * d * 2);
        e_enc_.alloc((size_t) M * d * 2);
        e_enc32_.alloc((size_t) M * d * 4);
    }
    e_a1_.alloc((size_t) n * T2 * kp1 * 2);

    std::vector<MelWindow> win(n);
    for (int i = 0; i < n; ++i) win[i] = MelWindow{mel_[slots[i]]->as<float>(), mel_len_[slots[i]], offsets[i]};
    e_win_.alloc(sizeof(MelWindow) * n);
    e_slotmap_.alloc(sizeof(int) * n);
    OWK_HIP_CHECK(hipMemcpyAsync(e_win_.ptr, win.data(), sizeof(MelWindow) * n, hipMemcpyHostToDevice, stream));
    OWK_HIP_CHECK(hipMemcpyAsync(e_slotmap_.ptr, slots.data(), sizeof(int) * n, hipMemcpyHostToDevice, stream));

    auto G = [&](const char * cls, int mode, int Mr, int N, int K, const _Float16 * A, int lda, const _Float16 * W,
                 const EpiParams & ep) {
        ProfScope ps(prof, stream, cls, gemm_flops(Mr, N, K), 2.0 * ((double) Mr * K + (double) N * K));
        gemm_f16(stream, mode, Mr, N, K, A, lda, W, K, ep);
    };

    // conv1 (k3 s1 p1) + GELU -> f16 ; conv2 (k3 s2 p1) + GELU + positional embedding -> f32
    {
        ProfScope ps(prof, stream, "im2col");
        conv1_im2col(stream, e_win_.as<MelWindow>(), n, hp.n_mels, T2, kp1, e_a1_.as<_Float16>());
    }
    {
        EpiParams ep;
        ep.bias = m->conv1_b;
        ep.gelu_tab = m->gelu_tab;
        ep.out16 = e_c1_.as<_Float16>();
        ep.ldo = d;
        G("gemm_conv", EPI_GELU_F16, n * T2, d, kp1, e_a1_.as<_Float16>(), kp1, m->conv1_w, ep);
    }
    {
        ProfScope ps(prof, stream, "im2col");
        conv2_im2col(stream, e_c1_.as<_Float16>(), n, T2, d, e_a2_.as<_Float16>());
    }
    {
        EpiParams ep;
        ep.bias = m->conv2_b;
        ep.gelu_tab = m->gelu_tab;
        ep.out32 = e_x_.as<float>();
        ep.ldo = d;
        ep.pos = m->e_pe;
        ep.T = T;
        G("gemm_conv", EPI_CONV2, M, d, 3 * d, e_a2_.as<_Float16>(), 3 * d, m->conv2_w, ep);
    }

    const float kq_scale = 1.0f / sqrtf((float) 64);
    for (int l = 0; l < hp.n_audio_layer; ++l) {
        const EncLayerW & L = m->enc[l];
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, e_x_.as<float>(), M, d, L.attn_ln_w, L.attn_ln_b, hp.eps, e_xn_.as<_Float16>(), d);
        }
        {
            EpiParams ep;
            ep.bias = L.b_q;
            ep.bias2 = L.b_v;
            ep.out16 = e_q_.as<_Float16>();
            ep.out16b = e_k_.as<_Float16>();
            ep.out16c = e_vt_.as<_Float16>();
            ep.d = d;
            ep.T = T;
            ep.Tpad = Tpad;
            G("gemm_enc", EPI_QKV_ENC, M, 3 * d, d, e_xn_.as<_Float16>(), d, L.w_qkv, ep);
        }
        {
            // 4*T*Tpad_kv*d flops (QK^T and PV over the 1536 reference keys)
            ProfScope ps(prof, stream, "attn_encoder", 4.0 * n * (double) T * n_ctx_pad * d,
                         2.0 * 4.0 * M * (double) d);
            attn_encoder(stream, e_q_.as<_Float16>(), e_k_.as<_Float16>(), e_vt_.as<_Float16>(), n, T, Tpad, H, kq_scale,
                         n_zero_pad, e_ao_.as<_Float16>());
        }
        {
            EpiParams ep;
            ep.bias = L.b_o;
            ep.resid = e_x_.as<float>();
            ep.out32 = e_x_.as<float>();
            ep.ldo = d;
            G("gemm_enc", EPI_RESID_F32, M, d, d, e_ao_.as<_Float16>(), d, L.w_o, ep);
        }
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, e_x_.as<float>(), M, d, L.mlp_ln_w, L.mlp_ln_b, hp.eps, e_xn_.as<_Float16>(), d);
        }
        {
            EpiParams ep;
            ep.bias = L.b_mlp0;
            ep.gelu_tab = m->gelu_tab;
            ep.out16 = e_h_.as<_Float16>();
            ep.ldo = 4 * d;
            G("gemm_enc", EPI_GELU_F16, M, 4 * d, d, e_xn_.as<_Float16>(), d, L.w_mlp0, ep);
        }
        {
            EpiParams ep;
            ep.bias = L.b_mlp1;
            ep.resid = e_x_.as<float>();
            ep.out32 = e_x_.as<float>();
            ep.ldo = d;
            G("gemm_enc", EPI_RESID_F32, M, d, 4 * d, e_h_.as<_Float16>(), 4 * d, L.w_mlp1, ep);
        }
    }
    {
        ProfScope ps(prof, stream, "layernorm");
        layernorm_f16(stream, e_x_.as<float>(), M, d, m->e_ln_w, m->e_ln_b, hp.eps, e_enc_.as<_Float16>(), d, nullptr,
                      e_enc32_.as<float>());
    }
    last_enc_n_ = n;

    // cross-attention K/V for every decoder layer (whisper_build_graph_cross, ref 2272-2346)
    const float k_scale = powf(64.0f, -0.25f);
    const size_t layer_stride = (size_t) cap_slots * T * d;
    for (int l = 0; l < hp.n_text_layer; ++l) {
        const DecLayerW & L = m->dec[l];
        EpiParams ep;
        ep.scale = k_scale;
        ep.bias2 = L.cb_v;
        ep.out16b = cross_k_.as<_Float16>() + l * layer_stride;
        ep.out16c = cross_v_.as<_Float16>() + l * layer_stride;
        ep.d = d;
        ep.T = T;
        ep.slot_map = e_slotmap_.as<int>();
        G("gemm_cross", EPI_KV_CROSS, M, 2 * d, d, e_enc_.as<_Float16>(), d, L.cw_kv, ep);
    }
}

void Engine::download_enc(int index, float * host) const {
    const HParams & hp = m->hp;
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    const size_t n = (size_t) hp.n_audio_ctx * hp.n_audio_state;
    OWK_HIP_CHECK(hipMemcpy(host, e_enc32_.as<float>() + index * n, n * 4, hipMemcpyDeviceToHost));
}

void Engine::download_cross(int slot, int layer, uint16_t * kh, uint16_t * vh) const {
    const HParams & hp = m->hp;
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    const size_t per = (size_t) hp.n_audio_ctx * hp.n_text_state;
    const size_t o = ((size_t) layer * cap_slots + slot) * per;
    OWK_HIP_CHECK(hipMemcpy(kh, cross_k_.as<_Float16>() + o, per * 2, hipMemcpyDeviceToHost));
    OWK_HIP_CHECK(hipMemcpy(vh, cross_v_.as<_Float16>() + o, per * 2, hipMemcpyDeviceToHost));
}

void Engine::decode(const std::vector<DecodeRow> & rows, const std::vector<int> & key_list, int n_logit_rows) {
    const HParams & hp = m->hp;
    const int R = (int) rows.size();
    if (R == 0) return;
    const int d = hp.n_text_state, H = hp.n_text_head, T = hp.n_audio_ctx;
    const int n_ctx_pad = (T + 255) / 256 * 256;
    const int nv = hp.n_vocab;

    if (R > dec_rows_cap_) {
        sync();
        dec_rows_cap_ = std::max(R, 64);
        const int C = dec_rows_cap_;
        d_x_.alloc((size_t) C * d * 4);
        d_xn_.alloc((size_t) C * d * 2);
        d_q_.alloc((size_t) C * d * 2);
        d_ao_.alloc((size_t) C * d * 2);
        d_h_.alloc((size_t) C * 4 * d * 2);
        d_tok_.alloc((size_t) C * 4);
        d_pos_.alloc((size_t) C * 4);
        d_rowoff_.alloc((size_t) C * 8);
        d_rows_self_.alloc(sizeof(AttnRow) * C);
        d_rows_cross_.alloc(sizeof(AttnRow) * C);
        d_lsel_.alloc((size_t) C * 4);
        d_xl_.alloc((size_t) C * d * 2);
    }
    if (n_logit_rows > 0) logits_.alloc((size_t) std::max(n_logit_rows, 1) * nv * 4);

    // host-side staging
    std::vector<int> tok(R), pos(R), lsel(std::max(n_logit_rows, 1), 0);
    std::vector<int64_t> rowoff(R);
    std::vector<AttnRow> rs(R), rc(R);
    int max_keys = 1;
    bool self_oc = false, self_tl = false, cross_oc = false, cross_tl = false;
    for (int r = 0; r < R; ++r) {
        const DecodeRow & x = rows[r];
        tok[r] = x.token;
        pos[r] = x.pos;
        rowoff[r] = ((int64_t) x.slot * kv_cells + x.cell) * d;
        rs[r] = AttnRow{r, (int) ((int64_t) x.slot * kv_cells * d), x.n_keys, x.key_off, 0, x.mode_self};
        rc[r] = AttnRow{r, (int) ((int64_t) x.slot * T * d), T, -1, n_ctx_pad - T, x.mode_cross};
        max_keys = std::max(max_keys, x.n_keys);
        (x.mode_self ? self_tl : self_oc) = true;
        (x.mode_cross ? cross_tl : cross_oc) = true;
        if (x.logit_row >= 0) lsel[x.logit_row] = r;
    }
    d_keys_.alloc(std::max<size_t>(key_list.size(), 1) * 4);
    OWK_HIP_CHECK(hipMemcpyAsync(d_tok_.ptr, tok.data(), R * 4, hipMemcpyHostToDevice, stream));
    OWK_HIP_CHECK(hipMemcpyAsync(d_pos_.ptr, pos.data(), R * 4, hipMemcpyHostToDevice, stream));
    OWK_HIP_CHECK(hipMemcpyAsync(d_rowoff_.ptr, rowoff.data(), R * 8, hipMemcpyHostToDevice, stream));
    OWK_HIP_CHECK(hipMemcpyAsync(d_rows_self_.ptr, rs.data(), sizeof(AttnRow) * R, hipMemcpyHostToDevice, stream));
    OWK_HIP_CHECK(hipMemcpyAsync(d_rows_cross_.ptr, rc.data(), sizeof(AttnRow) * R, hipMemcpyHostToDevice, stream));
    if (!key_list.empty())
        OWK_HIP_CHECK(hipMemcpyAsync(d_keys_.ptr, key_list.data(), key_list.size() * 4, hipMemcpyHostToDevice, stream));
    OWK_HIP_CHECK(hipMemcpyAsync(d_lsel_.ptr, lsel.data(), lsel.size() * 4, hipMemcpyHostToDevice, stream));

    // checks the kernels rely on (fail loudly rather than read out of bounds)
    if ((int64_t) cap_slots * std::max(kv_cells, T) * d >= (int64_t) 1 << 31)
        throw std::runtime_error("decode: KV offsets exceed 32 bits");
    for (const auto & x : rows)
        if (x.slot < 0 || x.slot >= cap_slots || x.cell < 0 || x.cell >= kv_cells || x.token < 0 || x.token >= nv ||
            x.pos < 0 || x.pos >= hp.n_text_ctx)
            throw std::runtime_error("decode: row out of range");

    auto G = [&](const char * cls, int mode, int N, int K, const _Float16 * A, const _Float16 * W, const EpiParams & ep,
                 int Mr) {
        ProfScope ps(prof, stream, Mr <= 64 ? "gemm_dec" : "gemm_dec_big", gemm_flops(Mr, N, K),
                     2.0 * ((double) Mr * K + (double) N * K));
        (void) cls;
        gemm(stream, mode, Mr, N, K, A, K, W, K, ep, &gws_);
    };

    {
        ProfScope ps(prof, stream, "embed");
        embed_tokens(stream, m->d_te, m->d_pe, d_tok_.as<int>(), d_pos_.as<int>(), R, d, d_x_.as<float>());
    }
    const float kq_scale = powf(64.0f, -0.25f);
    const size_t self_stride = (size_t) cap_slots * kv_cells * d;
    const size_t cross_stride = (size_t) cap_slots * T * d;
    for (int l = 0; l < hp.n_text_layer; ++l) {
        const DecLayerW & L = m->dec[l];
        _Float16 * Kl = self_k_.as<_Float16>() + l * self_stride;
        _Float16 * Vl = self_v_.as<_Float16>() + l * self_stride;
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, d_x_.as<float>(), R, d, L.attn_ln_w, L.attn_ln_b, hp.eps, d_xn_.as<_Float16>(), d);
        }
        {
            EpiParams ep;
            ep.bias = L.b_q;
            ep.bias2 = L.b_v;
            ep.scale = kq_scale;
            ep.out16 = d_q_.as<_Float16>();
            ep.ldo = d;
            ep.out16b = Kl;
            ep.out16c = Vl;
            ep.d = d;
            ep.row_off = d_rowoff_.as<int64_t>();
            G("qkv", EPI_QKV_DEC, 3 * d, d, d_xn_.as<_Float16>(), L.w_qkv, ep, R);
        }
        {
            ProfScope ps(prof, stream, "attn_self");
            attn_decoder(stream, d_q_.as<_Float16>(), d, Kl, Vl, d, d_rows_self_.as<AttnRow>(), R, d_keys_.as<int>(), H,
                         1.0f, max_keys, d_ao_.as<_Float16>(), d, self_oc, self_tl);
        }
        {
            EpiParams ep;
            ep.bias = L.b_o;
            ep.resid = d_x_.as<float>();
            ep.out32 = d_x_.as<float>();
            ep.ldo = d;
            G("o", EPI_RESID_F32, d, d, d_ao_.as<_Float16>(), L.w_o, ep, R);
        }
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, d_x_.as<float>(), R, d, L.cross_ln_w, L.cross_ln_b, hp.eps, d_xn_.as<_Float16>(), d);
        }
        {
            EpiParams ep;
            ep.bias = L.cb_q;
            ep.out16 = d_q_.as<_Float16>();
            ep.ldo = d;
            G("cq", EPI_F16, d, d, d_xn_.as<_Float16>(), L.cw_q, ep, R);
        }
        {
            // bytes: cross K and V of each row's clip (the HBM-bound part of a decode step)
            ProfScope ps(prof, stream, "attn_cross", 4.0 * R * (double) n_ctx_pad * d, 2.0 * 2.0 * R * (double) T * d);
            attn_decoder(stream, d_q_.as<_Float16>(), d, cross_k_.as<_Float16>() + l * cross_stride,
                         cross_v_.as<_Float16>() + l * cross_stride, d, d_rows_cross_.as<AttnRow>(), R, nullptr, H,
                         kq_scale, T, d_ao_.as<_Float16>(), d, cross_oc, cross_tl);
        }
        {
            EpiParams ep;
            ep.bias = L.cb_o;
            ep.resid = d_x_.as<float>();
            ep.out32 = d_x_.as<float>();
            ep.ldo = d;
            G("co", EPI_RESID_F32, d, d, d_ao_.as<_Float16>(), L.cw_o, ep, R);
        }
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, d_x_.as<float>(), R, d, L.mlp_ln_w, L.mlp_ln_b, hp.eps, d_xn_.as<_Float16>(), d);
        }
        {
            EpiParams ep;
            ep.bias = L.b_mlp0;
            ep.gelu_tab = m->gelu_tab;
            ep.out16 = d_h_.as<_Float16>();
            ep.ldo = 4 * d;
            G("mlp0", EPI_GELU_F16, 4 * d, d, d_xn_.as<_Float16>(), L.w_mlp0, ep, R);
        }
        {
            EpiParams ep;
            ep.bias = L.b_mlp1;
            ep.resid = d_x_.as<float>();
            ep.out32 = d_x_.as<float>();
            ep.ldo = d;
            G("mlp1", EPI_RESID_F32, d, 4 * d, d_h_.as<_Float16>(), L.w_mlp1, ep, R);
        }
    }
    if (n_logit_rows > 0) {
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, d_x_.as<float>(), n_logit_rows, d, m->d_ln_w, m->d_ln_b, hp.eps, d_xl_.as<_Float16>(),
                          d, d_lsel_.as<int>());
        }
        EpiParams ep;
        ep.out32 = logits_.as<float>();
        ep.ldo = nv;
        ProfScope ps(prof, stream, n_logit_rows <= 64 ? "gemm_logits" : "gemm_logits_big",
                     gemm_flops(n_logit_rows, nv, d), 2.0 * (double) nv * d);
        gemm(stream, EPI_F32, n_logit_rows, nv, d, d_xl_.as<_Float16>(), d, m->d_te, d, ep, &gws_);
    }
}

void Engine::logits_maxes(int n, std::vector<float> & out) {
    out.resize(n);
    if (n <= 0) return;
    lmax_.alloc((size_t) n * 4);
    logits_row_max(stream, logits_.as<float>(), n, m->hp.n_vocab, lmax_.as<float>());
    OWK_HIP_CHECK(hipMemcpyAsync(out.data(), lmax_.ptr, (size_t) n * 4, hipMemcpyDeviceToHost, stream));
    sync();
}

void Engine::row0_update(const std::vector<std::pair<int, int>> & map) {
    if (map.empty()) return;
    const int nv = m->hp.n_vocab;
    row0_.alloc((size_t) cap_slots * nv * 4);
    std::vector<int2> h(map.size());
    for (size_t i = 0; i < map.size(); ++i) h[i] = make_int2(map[i].first, map[i].second);
    map_.alloc(h.size() * sizeof(int2));
    OWK_HIP_CHECK(hipMemcpyAsync(map_.ptr, h.data(), h.size() * sizeof(int2), hipMemcpyHostToDevice, stream));
    logits_copy_rows(stream, logits_.as<float>(), nv, map_.as<int2>(), (int) h.size(), row0_.as<float>());
}

void Engine::nosp(const std::vector<std::pair<int, float>> & req, std::vector<float> & out) {
    const int n = (int) req.size();
    out.resize(n);
    if (n == 0) return;
    const int nv = m->hp.n_vocab;
    row0_.alloc((size_t) cap_slots * nv * 4);
    std::vector<int> idx(n);
    std::vector<float> mx(n);
    for (int i = 0; i < n; ++i) { idx[i] = req[i].first; mx[i] = req[i].second; }
    nosp_idx_.alloc(n * 4);
    nosp_max_.alloc(n * 4);
    nosp_out_.alloc(n * 4);
    OWK_HIP_CHECK(hipMemcpyAsync(nosp_idx_.ptr, idx.data(), n * 4, hipMemcpyHostToDevice, stream));
    OWK_HIP_CHECK(hipMemcpyAsync(nosp_max_.ptr, mx.data(), n * 4, hipMemcpyHostToDevice, stream));
    nosp_probs(stream, row0_.as<float>(), nv, nosp_idx_.as<int>(), nosp_max_.as<float>(), n, m->vocab.nosp,
               nosp_out_.as<float>());
    OWK_HIP_CHECK(hipMemcpyAsync(out.data(), nosp_out_.ptr, n * 4, hipMemcpyDeviceToHost, stream));
    sync();
}

void Engine::download_logits(int logit_row, float * host) const {
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    const int nv = m->hp.n_vocab;
    OWK_HIP_CHECK(hipMemcpy(host, logits_.as<float>() + (size_t) logit_row * nv, (size_t) nv * 4, hipMemcpyDeviceToHost));
}

void Engine::upload_logits(int logit_row, const float * host) {
    const int nv = m->hp.n_vocab;
    OWK_HIP_CHECK(hipMemcpyAsync(logits_.as<float>() + (size_t) logit_row * nv, host, (size_t) nv * 4,
                                 hipMemcpyHostToDevice, stream));
    sync();
}

void Engine::process_logits(const std::vector<LogitJob> & jobs, const VocabInfo & vi_in, std::vector<TokenOut> & out,
                            float * probs_host, float * logprobs_host) {
    const int n = (int) jobs.size();
    out.resize(n);
    if (n == 0) return;
    const int nv = m->hp.n_vocab;
    VocabInfo vi = vi_in;
    suppress_.alloc(std::max(vi.n_suppress, 1) * 4);
    if (vi.n_suppress > 0)
        OWK_HIP_CHECK(hipMemcpyAsync(suppress_.ptr, vi.suppress_list, vi.n_suppress * 4, hipMemcpyHostToDevice, stream));
    vi.suppress_list = suppress_.as<int>();
    lg_jobs_.alloc(sizeof(LogitJob) * n);
    lg_out_.alloc(sizeof(TokenOut) * n);
    OWK_HIP_CHECK(hipMemcpyAsync(lg_jobs_.ptr, jobs.data(), sizeof(LogitJob) * n, hipMemcpyHostToDevice, stream));
    float * pr = nullptr;
    float * lp = nullptr;
    if (probs_host) {
        lg_probs_.alloc((size_t) n * nv * 4);
        pr = lg_probs_.as<float>();
    }
    if (logprobs_host) {
        lg_lp_.alloc((size_t) n * nv * 4);
        lp = lg_lp_.as<float>();
    }
    {
        ProfScope ps(prof, stream, "logits_proc");
        owk::process_logits(stream, logits_.as<float>(), nv, lg_jobs_.as<LogitJob>(), n, vi, lg_out_.as<TokenOut>(), lp,
                            pr);
    }
    OWK_HIP_CHECK(hipMemcpyAsync(out.data(), lg_out_.ptr, sizeof(TokenOut) * n, hipMemcpyDeviceToHost, stream));
    if (pr) OWK_HIP_CHECK(hipMemcpyAsync(probs_host, pr, (size_t) n * nv * 4, hipMemcpyDeviceToHost, stream));
    if (lp) OWK_HIP_CHECK(hipMemcpyAsync(logprobs_host, lp, (size_t) n * nv * 4, hipMemcpyDeviceToHost, stream));
    sync();
}

} // namespace owk
