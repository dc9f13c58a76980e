// Batch-major device engine (see engine.h).
#include "engine.h"

#include <atomic>
#include "kquant.h"

#include <algorithm>
#include <map>
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
    if (!p->only.empty() && std::find(p->only.begin(), p->only.end(), name) == p->only.end()) return;
    cls = p->cls_id(name);
    a = p->ev();
    if (!p->only.empty()) {
        // selected classes: events bound to the class's own kernel dispatches (KTimer), no markers
        KTimer * kt = ktimer();
        if (kt->stop) throw std::runtime_error("prof: nested selected-class scopes");
        kt->start = a;
        kt->stop = p->ev();
        kt->launches = 0;
        return;
    }
    OWK_HIP_CHECK(hipEventRecord(a, s));
}

ProfScope::~ProfScope() {
    if (cls < 0) return;
    if (!p->only.empty()) {
        KTimer * kt = ktimer();
        const hipEvent_t b = kt->stop;
        const int n = kt->launches;
        *kt = KTimer{};
        if (n > 0) {
            p->pending.push_back({cls, a, b, flops, bytes});
        } else {  // a scope that launched nothing: no record
            p->pool.push_back(a);
            p->pool.push_back(b);
        }
    } else {
        hipEvent_t b = p->ev();
        (void) hipEventRecord(b, s);
        p->pending.push_back({cls, a, b, flops, bytes});
    }
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
    for (int K : {d, 4 * d}) fl = std::max(fl, std::max(gemm_partial_floats(d, K), q5_partial_floats(d, K)));
    gws_part_.alloc(std::max<size_t>(fl, 1) * 4);
    gws_.partial = gws_part_.as<float>();
    gws_.partial_floats = fl;
}

Engine::~Engine() {
    clear_graphs();
    for (auto * b : mel_) delete b;
    if (stream) (void) hipStreamDestroy(stream);
}

static std::atomic<int> g_whole_k_rows{kWholeKRowsDefault};
int whole_k_rows() { return g_whole_k_rows.load(std::memory_order_relaxed); }
int set_whole_k_rows(int n) { return g_whole_k_rows.exchange(n); }

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
        // captured decode graphs bake in the cache strides (kv_cells, cap_slots) and buffer
        // addresses; hipMalloc may hand back the same address, so drop them on any re-layout
        clear_graphs();
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
        mel_spectrogram(stream, mel_jobs_.as<MelJob>(), n, max_frames, m->mel_filters, m->mel_rng, n_mel, m->twiddle,
                        m->hann);
        mel_normalize(stream, mel_jobs_.as<MelJob>(), n, n_mel);
    }
    sync();  // pcm host buffers may go away after return
}

void Engine::set_mel(int slot, const float * host, int n_len, int n_mel) {
    // n_len = 0 is legal (ref whisper_set_mel_with_state copies nothing; the encoder window is
    // then all zeros -- examples/bench/bench.cpp:84 does exactly this)
    if (n_len < 0 || (n_len > 0 && !host)) throw std::runtime_error("set_mel: no data");
    DevBuf * b = mel_[slot];
    b->alloc(std::max<size_t>((size_t) n_mel * n_len * 4, 4));
    mel_len_[slot] = n_len;
    if (n_len > 0) OWK_HIP_CHECK(hipMemcpy(b->ptr, host, (size_t) n_mel * n_len * 4, hipMemcpyHostToDevice));
}

void Engine::download_mel(int slot, float * host) const {
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    OWK_HIP_CHECK(hipMemcpy(host, mel_[slot]->ptr, (size_t) m->n_filters_mel * mel_len_[slot] * 4, hipMemcpyDeviceToHost));
}

static double gemm_flops(double M, double N, double K) { return 2.0 * M * N * K; }

void Engine::linear(const char * cls, int mode, int M, int N, int K, const _Float16 * A16, const float * A32, int lda,
                    const _Float16 * W, const Q5W & q, const EpiParams & ep, const _Float16 * Wt, bool dec, bool a_q8,
                    const int8_t * qa, const float * qd) {
    if (!q) {
        ProfScope ps(prof, stream, cls, gemm_flops(M, N, K), 2.0 * ((double) M * K + (double) N * K));
        if (dec) gemm(stream, mode, M, N, K, A16, lda, W, K, ep, &gws_, Wt);
        else gemm_f16(stream, mode, M, N, K, A16, lda, W, K, ep);
        return;
    }
    // the reference rounds each activation row to Q8_0 / Q8_1 (x86 quantize_row_q8_0 / _q8_1) before
    // the block dot; bytes: the weight blocks (18-34 B per 32) + the int8 activations. a_q8: the
    // producer (LayerNorm, one_chunk attention) already wrote q8a_ / q8d_ (or qa / qd: the MLP0 epilogue's rows)
    if (qf_is_k(q.fmt)) {
        // K-quants: Q8_K rows in the virtual-block layout (kquant.h), then the f16 MFMA ring kernel
        // over the virtual K at every shape
        const int mpad = (M + 255) / 256 * 256, kx = q.kx;
        if (q16a_.bytes < (size_t) M * kx * 2 || q16d_.bytes < (size_t) (kx / 32) * mpad * 4)
            throw std::runtime_error("linear: K-quant operand buffers not reserved");
        {
            ProfScope ps(prof, stream, "quantize_q8");
            quantize_q8k_f16(stream, A32, A16, lda, M, K, q.fmt, q16a_.as<_Float16>(), q16d_.as<float>(), mpad,
                             qf_k_repacked(q.fmt) ? kq_rmul_ : nullptr);
        }
        ProfScope ps(prof, stream, cls, gemm_flops(M, N, K), (double) N * K * kq_block_bytes(q.fmt) / 256.0 + (double) M * K);
        gemm_q16(stream, mode, M, N, kx, q16a_.as<_Float16>(), q16d_.as<float>(), mpad, q, ep);
        return;
    }
    if (gemm_q16_applies(q, M, N, K)) {
        // large tiles: Q8_0 integers as exact f16 + block-major scales, the f16 MFMA ring kernel; the
        // rows are quantized from the f32 activation (A32) where the producer keeps one, as the reference
        const int mpad = (M + 255) / 256 * 256;
        if (q16a_.bytes < (size_t) M * K * 2 || q16d_.bytes < (size_t) (K / 32) * mpad * 4)
            throw std::runtime_error("linear: gemm_q16 operand buffers not reserved");
        {
            ProfScope ps(prof, stream, "quantize_q8");
            quantize_q8_f16(stream, A32, A16, lda, M, K, q16a_.as<_Float16>(), q16d_.as<float>(), mpad);
        }
        ProfScope ps(prof, stream, cls, gemm_flops(M, N, K), 2.0 * ((double) M * K + (double) N * K));
        gemm_q16(stream, mode, M, N, K, q16a_.as<_Float16>(), q16d_.as<float>(), mpad, q, ep);
        return;
    }
    if (!a_q8) {
        ProfScope ps(prof, stream, "quantize_q8");
        quantize_q8(stream, A32, A16, lda, M, K, q8a_.as<int8_t>(), q8d_.as<float>());
    }
    if (qa && !a_q8) throw std::runtime_error("linear: operand rows without a_q8");
    ProfScope ps(prof, stream, cls, gemm_flops(M, N, K), (double) N * K * qf_block_bytes(q.fmt) / 32.0 + (double) M * K);
    gemm_q5(stream, mode, M, N, K, qa ? qa : q8a_.as<int8_t>(), qd ? qd : q8d_.as<float>(), q, ep);
}

void Engine::encode(const std::vector<int> & slots, const std::vector<int> & offsets) {
    const HParams & hp = m->hp;
    const int n = (int) slots.size();
    if (n == 0) return;
    const int T = n_ctx(), T2 = 2 * T, d = hp.n_audio_state, H = hp.n_audio_head;
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
        e_ao_.alloc((size_t) M * d * 2);
        e_h_.alloc((size_t) M * 4 * d * 2);
        e_enc_.alloc((size_t) M * d * 2);
        e_enc32_.alloc((size_t) M * d * 4);
        if (m->q5) {
            e_ao32_.alloc((size_t) M * d * 4);
            e_xn32_.alloc((size_t) M * d * 4);  // f32 LayerNorm rows: gemm_q16 quantizes them like the reference
            q8a_.alloc(std::max(q8a_.bytes, (size_t) M * 4 * d));
            q8d_.alloc(std::max(q8d_.bytes, (size_t) M * 4 * d / 32 * 4));
            // gemm_q16 operands (reserved here: growing them inside linear() would free a buffer
            // queued kernels may still read)
            const size_t mpad = ((size_t) M + 255) / 256 * 256;
            const size_t kmax = m->kq ? (size_t) kq_kx(m->qfmt, 4 * d) : (size_t) 4 * d;  // K-quants: the virtual K
            q16a_.alloc(std::max(q16a_.bytes, (size_t) M * kmax * 2));
            q16d_.alloc(std::max(q16d_.bytes, kmax / 32 * mpad * 4));
        }
    }
    e_a1_.alloc((size_t) n * T2 * kp1 * 2);
    // transposed V [clip][head][64][Tpad]: key columns T..Tpad-1 must read as 0 (zeroed whenever
    // the buffer or its T changes: a reduced audio_ctx re-lays it out)
    if ((size_t) n * H * 64 * Tpad * 2 > e_vt_.bytes || vt_T_ != T) {
        sync();
        e_vt_.alloc(std::max(e_vt_.bytes, (size_t) n * H * 64 * Tpad * 2));
        OWK_HIP_CHECK(hipMemsetAsync(e_vt_.ptr, 0, e_vt_.bytes, stream));
        vt_T_ = T;
    }

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

    // K-quants with repacked reference weights: each clip's T rows are one reference matmul, whose
    // complete groups of 4 rows take the repack quantizer (kernels.h qf_k_repacked)
    kq_rmul_ = nullptr;
    if (m->kq && qf_k_repacked(m->qfmt)) {
        std::vector<uint8_t> rm((size_t) M);
        for (int i = 0; i < n; ++i)
            for (int t = 0; t < T; ++t) rm[(size_t) i * T + t] = t < T - T % 4;
        e_rmul_.alloc(rm.size());
        OWK_HIP_CHECK(hipMemcpy(e_rmul_.ptr, rm.data(), rm.size(), hipMemcpyHostToDevice));
        kq_rmul_ = e_rmul_.as<uint8_t>();
    }
    const float kq_scale = 1.0f / sqrtf((float) 64);
    for (int l = 0; l < hp.n_audio_layer; ++l) {
        const EncLayerW & L = m->enc[l];
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, e_x_.as<float>(), M, d, L.attn_ln_w, L.attn_ln_b, hp.eps, e_xn_.as<_Float16>(), d,
                          nullptr, m->q5 ? e_xn32_.as<float>() : nullptr, q8a(), q8d());
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
            linear("gemm_enc", EPI_QKV_ENC, M, 3 * d, d, e_xn_.as<_Float16>(), m->q5 ? e_xn32_.as<float>() : nullptr, d,
                   L.w_qkv, L.q_qkv, ep, nullptr, false, m->q5 && !m->kq);
        }
        {
            // 4*T*Tpad_kv*d flops (QK^T and PV over the 1536 reference keys)
            ProfScope ps(prof, stream, "attn_encoder", 4.0 * n * (double) T * n_ctx_pad * d,
                         2.0 * 4.0 * M * (double) d);
            if (flash_attn)
                attn_encoder(stream, e_q_.as<_Float16>(), e_k_.as<_Float16>(), e_vt_.as<_Float16>(), n, T, Tpad, H,
                             kq_scale, n_zero_pad, e_ao_.as<_Float16>(), m->q5 ? e_ao32_.as<float>() : nullptr);
            else  // soft_max path over exactly T keys (whisper.cpp:2163-2189)
                attn_encoder_softmax(stream, e_q_.as<_Float16>(), e_k_.as<_Float16>(), e_vt_.as<_Float16>(), n, T, Tpad,
                                     H, kq_scale, e_ao_.as<_Float16>(), m->q5 ? e_ao32_.as<float>() : nullptr);
        }
        {
            EpiParams ep;
            ep.bias = L.b_o;
            ep.resid = e_x_.as<float>();
            ep.out32 = e_x_.as<float>();
            ep.ldo = d;
            linear("gemm_enc", EPI_RESID_F32, M, d, d, e_ao_.as<_Float16>(), e_ao32_.as<float>(), d, L.w_o, L.q_o, ep);
        }
        {
            ProfScope ps(prof, stream, "layernorm");
            layernorm_f16(stream, e_x_.as<float>(), M, d, L.mlp_ln_w, L.mlp_ln_b, hp.eps, e_xn_.as<_Float16>(), d,
                          nullptr, m->q5 ? e_xn32_.as<float>() : nullptr, q8a(), q8d());
        }
        {
            EpiParams ep;
            ep.bias = L.b_mlp0;
            ep.gelu_tab = m->gelu_tab;
            ep.out16 = e_h_.as<_Float16>();
            ep.ldo = 4 * d;
            linear("gemm_enc", EPI_GELU_F16, M, 4 * d, d, e_xn_.as<_Float16>(), m->q5 ? e_xn32_.as<float>() : nullptr, d,
                   L.w_mlp0, L.q_mlp0, ep, nullptr, false, m->q5 && !m->kq);
        }
        {
            EpiParams ep;
            ep.bias = L.b_mlp1;
            ep.resid = e_x_.as<float>();
            ep.out32 = e_x_.as<float>();
            ep.ldo = d;
            // GELU outputs are F16 table values: exact as the f32 tensor the reference quantizes
            linear("gemm_enc", EPI_RESID_F32, M, d, 4 * d, e_h_.as<_Float16>(), nullptr, 4 * d, L.w_mlp1, L.q_mlp1, ep);
        }
    }
    {
        ProfScope ps(prof, stream, "layernorm");
        layernorm_f16(stream, e_x_.as<float>(), M, d, m->e_ln_w, m->e_ln_b, hp.eps, e_enc_.as<_Float16>(), d, nullptr,
                      e_enc32_.as<float>(), q8a(), q8d());
    }
    last_enc_n_ = n;

    // cross-attention K/V for every decoder layer (whisper_build_graph_cross, ref 2272-2346)
    const float k_scale = powf(64.0f, -0.25f);
    const size_t layer_stride = (size_t) cap_slots * hp.n_audio_ctx * d;  // capacity; slots of n_ctx() rows inside
    if ((uint64_t) cap_slots * T * d >= (uint64_t) 1 << 32)  // the KV_CROSS epilogue's 32-bit offsets
        throw std::runtime_error("encode: cross K/V offsets exceed 32 bits");
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
        // Q5_0: the final LayerNorm wrote the encoder output's Q8_0 rows once for all layers
        linear("gemm_cross", EPI_KV_CROSS, M, 2 * d, d, e_enc_.as<_Float16>(), m->q5 ? e_enc32_.as<float>() : nullptr, d,
               L.cw_kv, L.q_ckv, ep, nullptr, false, m->q5 && !m->kq);
    }
    kq_rmul_ = nullptr;
}

void Engine::download_enc(int index, float * host) const {
    const HParams & hp = m->hp;
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    const size_t n = (size_t) n_ctx() * hp.n_audio_state;
    OWK_HIP_CHECK(hipMemcpy(host, e_enc32_.as<float>() + index * n, n * 4, hipMemcpyDeviceToHost));
}

void Engine::download_cross(int slot, int layer, uint16_t * kh, uint16_t * vh) const {
    const HParams & hp = m->hp;
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    const int T = n_ctx(), d = hp.n_text_state, H = d / 64;
    const size_t per = (size_t) T * d;
    const size_t o = (size_t) layer * cap_slots * hp.n_audio_ctx * d + (size_t) slot * per;
    // device layout is head-major [head][t][64]; the caller gets the reference's [t][d]
    std::vector<uint16_t> tk(per), tv(per);
    OWK_HIP_CHECK(hipMemcpy(tk.data(), cross_k_.as<_Float16>() + o, per * 2, hipMemcpyDeviceToHost));
    OWK_HIP_CHECK(hipMemcpy(tv.data(), cross_v_.as<_Float16>() + o, per * 2, hipMemcpyDeviceToHost));
    for (int h = 0; h < H; ++h)
        for (int t = 0; t < T; ++t)
            for (int j = 0; j < 64; ++j) {
                kh[(size_t) t * d + h * 64 + j] = tk[((size_t) h * T + t) * 64 + j];
                vh[(size_t) t * d + h * 64 + j] = tv[((size_t) h * T + t) * 64 + j];
            }
}

// decode staging: one pinned host image + its device copy, fixed sections sized by the
// row/key capacities so the pointers captured in decode graphs stay valid
void Engine::stage_layout(int C, int KC) {
    size_t o = 0;
    auto sec = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) / 256 * 256;
        return at;
    };
    st_tok_ = sec((size_t) C * 4);
    st_pos_ = sec((size_t) C * 4);
    st_rowoff_ = sec((size_t) C * 8);
    st_rs_ = sec((size_t) C * sizeof(AttnRow));
    st_rc_ = sec((size_t) C * sizeof(AttnRow));
    st_lsel_ = sec((size_t) C * 4);
    st_rmul_ = sec((size_t) C);
    st_keys_ = sec((size_t) KC * 4);
    st_bytes_ = o;
}

void Engine::clear_graphs() {
    if (graphs_.empty()) return;
    // a replay may still be running on the stream: destroy the executables only once it has drained
    (void) hipStreamSynchronize(stream);
    for (auto & kv : graphs_) (void) hipGraphExecDestroy(kv.second);
    graphs_.clear();
}

uint64_t Engine::buffers_signature() const {
    uint64_t h = 1469598103934665603ull;
    for (const void * p : {d_x_.ptr, d_xn_.ptr, d_q_.ptr, d_ao_.ptr, d_h_.ptr, d_xl_.ptr, logits_.ptr, d_stg_.ptr,
                           q8a_.ptr, q8d_.ptr, q8h_.ptr, q8hd_.ptr, d_xn32_.ptr, d_ao32_.ptr, d_xl32_.ptr, q16a_.ptr, q16d_.ptr,
                           self_k_.ptr, self_v_.ptr, cross_k_.ptr, cross_v_.ptr, gws_part_.ptr, sm_ws_.ptr})
        h = (h ^ (uint64_t) (uintptr_t) p) * 1099511628211ull;
    return h;
}

void Engine::set_alignment_heads(const std::vector<int> & amap, int n_aheads) {
    const HParams & hp = m->hp;
    if ((int) amap.size() != hp.n_text_layer * hp.n_text_head) throw std::runtime_error("set_alignment_heads: map size");
    amap_.alloc(amap.size() * sizeof(int));
    OWK_HIP_CHECK(hipMemcpy(amap_.ptr, amap.data(), amap.size() * sizeof(int), hipMemcpyHostToDevice));
    n_ah_ = n_aheads;
}

void Engine::download_capture(int row0, int n, std::vector<float> & out) const {
    const int T = n_ctx();
    if (!cap_.ptr || row0 < 0 || row0 + n > cap_rows_) throw std::runtime_error("download_capture: no such rows");
    std::vector<float> all((size_t) n_ah_ * T * cap_rows_);
    OWK_HIP_CHECK(hipMemcpyAsync(all.data(), cap_.ptr, all.size() * 4, hipMemcpyDeviceToHost, stream));
    OWK_HIP_CHECK(hipStreamSynchronize(stream));
    out.resize((size_t) n_ah_ * T * n);
    for (size_t kj = 0; kj < (size_t) n_ah_ * T; ++kj)
        memcpy(&out[kj * n], &all[kj * cap_rows_ + row0], (size_t) n * 4);
}

void Engine::decode(const std::vector<DecodeRow> & rows, const std::vector<int> & key_list, int n_logit_rows,
                    bool capture) {
    const HParams & hp = m->hp;
    const int R = (int) rows.size();
    if (R == 0) return;
    const int d = hp.n_text_state, T = n_ctx();
    const int n_ctx_pad = (T + 255) / 256 * 256;
    const int nv = hp.n_vocab;

    const int nk = (int) key_list.size();
    if (R > dec_rows_cap_ || nk > dec_keys_cap_) {
        sync();
        if (R > dec_rows_cap_) {
            dec_rows_cap_ = std::max(R, 64);
            const int C = dec_rows_cap_;
            d_x_.alloc((size_t) C * d * 4);
            d_xn_.alloc((size_t) C * d * 2);
            d_q_.alloc((size_t) C * d * 2);
            d_ao_.alloc((size_t) C * d * 2);
            d_h_.alloc((size_t) C * 4 * d * 2);
            d_xl_.alloc((size_t) C * d * 2);
            if (m->q5) {
                d_ao32_.alloc((size_t) C * d * 4);
                q8a_.alloc(std::max(q8a_.bytes, (size_t) C * 4 * d));
                q8d_.alloc(std::max(q8d_.bytes, (size_t) C * 4 * d / 32 * 4));
                q8h_.alloc((size_t) C * 4 * d);
                q8hd_.alloc((size_t) C * 4 * d / 32 * 4);
            }
            if (m->kq) {  // f32 LayerNorm rows (quantized to Q8_K like the reference) + gemm_q16 operands
                d_xn32_.alloc((size_t) C * d * 4);
                d_xl32_.alloc((size_t) C * d * 4);
                const size_t mpad = ((size_t) C + 255) / 256 * 256, kmax = (size_t) kq_kx(m->qfmt, 4 * d);
                q16a_.alloc(std::max(q16a_.bytes, (size_t) C * kmax * 2));
                q16d_.alloc(std::max(q16d_.bytes, kmax / 32 * mpad * 4));
            }
            logits_.alloc((size_t) C * nv * 4);
        }
        dec_keys_cap_ = std::max(nk, std::max(dec_keys_cap_ * 2, 4096));
        clear_graphs();  // staging offsets and row buffers change: no captured graph stays valid
        stage_layout(dec_rows_cap_, dec_keys_cap_);
        stg_.alloc(st_bytes_);
        d_stg_.alloc(st_bytes_);
    }
    if (n_logit_rows > R) throw std::runtime_error("decode: more logit rows than rows");

    // checks the kernels rely on (fail loudly rather than read out of bounds)
    if ((int64_t) cap_slots * std::max(kv_cells, T) * d >= (int64_t) 1 << 31)
        throw std::runtime_error("decode: KV offsets exceed 32 bits");
    for (const auto & x : rows)
        if (x.slot < 0 || x.slot >= cap_slots || x.cell < 0 || x.cell >= kv_cells || x.token < 0 || x.token >= nv ||
            x.pos < 0 || x.pos >= hp.n_text_ctx || x.n_keys < 0 || x.key_off < 0 || x.key_off + x.n_keys > nk)
            throw std::runtime_error("decode: row out of range");

    // host image -> one H2D copy
    char * h = stg_.as<char>();
    int * tok = (int *) (h + st_tok_);
    int * pos = (int *) (h + st_pos_);
    int64_t * rowoff = (int64_t *) (h + st_rowoff_);
    AttnRow * rs = (AttnRow *) (h + st_rs_);
    AttnRow * rc = (AttnRow *) (h + st_rc_);
    int * lsel = (int *) (h + st_lsel_);
    DecShape sh{R, n_logit_rows, false, false, false, false, 1};
    for (int r = 0; r < R; ++r) {
        const DecodeRow & x = rows[r];
        tok[r] = x.token;
        pos[r] = x.pos;
        // self-attention cache [layer][slot][head][cell][64] (head-major: a (row, head) streams
        // its cells as one contiguous run)
        rowoff[r] = (int64_t) x.slot * kv_cells * d + (int64_t) x.cell * 64;
        rs[r] = AttnRow{r, (int) ((int64_t) x.slot * kv_cells * d), x.n_keys, x.key_off, 0, x.mode_self};
        if (x.mode_self == 0 && x.n_keys > 0) {  // one contiguous run of cells: no list needed
            const int * kl = key_list.data() + x.key_off;
            bool run = true;
            for (int i = 1; i < x.n_keys && run; ++i) run = kl[i] == kl[0] + i;
            if (run) {
                rs[r].kv_base += kl[0] * 64;
                rs[r].key_list = -1;
            }
        }
        if (x.mode_self == 0 && x.n_keys > 0 && rs[r].key_list >= 0) sh.self_list = true;
        // soft_max rows attend over exactly n_audio_ctx keys (no FA padding, whisper.cpp:2700-2712)
        rc[r] = AttnRow{r, (int) ((int64_t) x.slot * T * d), T, -1, x.mode_cross == 2 ? 0 : n_ctx_pad - T, x.mode_cross};
        sh.max_keys = std::max(sh.max_keys, x.n_keys);
        (x.mode_self == 2 ? sh.self_sm : x.mode_self ? sh.self_tl : sh.self_oc) = true;
        (x.mode_cross == 2 ? sh.cross_sm : x.mode_cross ? sh.cross_tl : sh.cross_oc) = true;
        if (x.logit_row >= 0) lsel[x.logit_row] = r;
    }
    {
        std::vector<int> slots;
        slots.reserve(R);
        for (const auto & x : rows) slots.push_back(x.slot);
        std::sort(slots.begin(), slots.end());
        sh.n_clips = (int) (std::unique(slots.begin(), slots.end()) - slots.begin());
    }
    if (m->kq && qf_k_repacked(m->qfmt)) {
        // each clip's rows of this pass are one reference decode batch (its decoders' tokens, or a
        // prompt): the rows of its complete groups of 4 take the repack quantizer
        uint8_t * rm = (uint8_t *) (h + st_rmul_);
        std::map<int, int> cnt, seen;
        for (int r = 0; r < R; ++r) cnt[rows[r].slot]++;
        for (int r = 0; r < R; ++r) {
            const int c = cnt[rows[r].slot], i = seen[rows[r].slot]++;
            rm[r] = i < c - c % 4;
        }
    }
    if (nk) memcpy(h + st_keys_, key_list.data(), (size_t) nk * 4);
    OWK_HIP_CHECK(hipMemcpyAsync(d_stg_.ptr, h, st_keys_ + (size_t) nk * 4, hipMemcpyHostToDevice, stream));
    if (sh.self_oc && sh.max_keys > attn_max_listed_keys()) throw std::runtime_error("decode: too many self-attention keys");
    if (sh.self_tl && sh.max_keys > attn_max_tiled_keys()) throw std::runtime_error("decode: too many self-attention keys");

    // soft_max cross rows take the key-split attention only in passes of <= 128 (row, head) blocks
    // (attn_decoder_softmax): its workspace (~0.8 MB per large-v3 row) is sized for those passes only
    const int sm_rows = std::max(1, 128 / hp.n_text_head);
    if (sh.cross_sm && R * hp.n_text_head <= 128 && sm_ws_.bytes < attn_softmax_ws_floats(sm_rows, hp.n_text_head) * 4) {
        sync();
        sm_ws_.alloc(attn_softmax_ws_floats(sm_rows, hp.n_text_head) * 4);
        OWK_HIP_CHECK(hipMemsetAsync(sm_ws_.ptr, 0, sm_ws_.bytes, stream));  // arrival tickets start at 0
    }
    if (capture) {
        if (!n_ah_ || !amap_.ptr) throw std::runtime_error("decode: capture without alignment heads");
        if (!sh.cross_sm) throw std::runtime_error("decode: capture needs soft_max cross attention (flash_attn = false)");
        cap_.alloc((size_t) n_ah_ * T * R * 4);
        cap_rows_ = R;
        sh.capture = true;
    }
    static const bool no_graph = getenv("OWK_NO_GRAPH") && atoi(getenv("OWK_NO_GRAPH")) != 0;
    if ((prof && prof->on) || no_graph || capture) {
        // per-kernel events, debugging, DTW: eager launches
        launch_decode(sh);
        return;
    }
    // replay captured graphs of the decoder pass (one launch instead of ~10 per layer)
    const uint64_t sig = buffers_signature();
    if (sig != graphs_sig_) {
        clear_graphs();
        graphs_sig_ = sig;
    }
    // bits 0-19 R, 20-39 n_logit_rows, 40-47 flags, 48-58 T (the cross head stride baked in)
    const uint64_t shape = ((uint64_t) sh.self_oc << 40) | ((uint64_t) sh.self_tl << 41) |
                           ((uint64_t) sh.cross_oc << 42) | ((uint64_t) sh.cross_tl << 43) |
                           ((uint64_t) sh.self_sm << 44) | ((uint64_t) sh.cross_sm << 45) |
                           ((uint64_t) sh.self_list << 46) | ((uint64_t) (R <= whole_k_rows()) << 47) |
                           ((uint64_t) T << 48);
    const uint64_t key = (uint64_t) R | ((uint64_t) n_logit_rows << 20) | shape;
    OWK_HIP_CHECK(hipGraphLaunch(graph_for(key, stream, [&]() { launch_decode(sh); }), stream));
}

hipGraphExec_t Engine::graph_for(uint64_t key, hipStream_t s, const std::function<void()> & launch) {
    auto it = graphs_.find(key);
    if (it != graphs_.end()) return it->second;
    if (graphs_.size() >= 64) clear_graphs();
    hipGraph_t g = nullptr;
    OWK_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
        launch();
    } catch (...) {
        (void) hipStreamEndCapture(s, &g);
        if (g) (void) hipGraphDestroy(g);
        throw;
    }
    OWK_HIP_CHECK(hipStreamEndCapture(s, &g));
    hipGraphExec_t ex = nullptr;
    const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void) hipGraphDestroy(g);
    OWK_HIP_CHECK(e);
    graphs_.emplace(key, ex);
    return ex;
}

void Engine::launch_decode(const DecShape & sh) {
    if (sh.R <= 32 && !m->q5) {  // F16 passes of <= 32 rows: the decode-row chain
        fused_part(sh, 0, sh.R, stream, &gws_);
        launch_logits(sh);
        return;
    }
    const HParams & hp = m->hp;
    const int R = sh.R;
    const int d = hp.n_text_state, H = hp.n_text_head, T = n_ctx();
    const int n_ctx_pad = (T + 255) / 256 * 256;
    const int nv = hp.n_vocab;
    char * dv = d_stg_.as<char>();
    const int * d_tok = (const int *) (dv + st_tok_);
    const int * d_pos = (const int *) (dv + st_pos_);
    const int64_t * d_rowoff = (const int64_t *) (dv + st_rowoff_);
    const AttnRow * d_rs = (const AttnRow *) (dv + st_rs_);
    const AttnRow * d_rc = (const AttnRow *) (dv + st_rc_);
    const int * d_lsel = (const int *) (dv + st_lsel_);
    const int * d_keys = (const int *) (dv + st_keys_);
    const int max_keys = sh.max_keys;
    const bool self_oc = sh.self_oc, self_tl = sh.self_tl, cross_oc = sh.cross_oc, cross_tl = sh.cross_tl;

    auto sm_ws = [&]() { return sm_ws_.as<float>(); };
    auto sm_ws_floats = [&]() { return sm_ws_.bytes / 4; };
    const bool q5 = m->q5;
    // A32: the f32 activation a Q5_0 GEMM quantizes (null: the f16 A is exact, e.g. GELU output)
    // a_q8: the A operand's Q8_0 rows are already in q8a_ / q8d_ (Q5_0 models; written by the
    // producing LayerNorm or one_chunk attention kernel)
    auto G = [&](const char * cls, int mode, int N, int K, const _Float16 * A, const float * A32, const _Float16 * W,
                 const _Float16 * Wt, const Q5W & q, const EpiParams & ep, int Mr, bool a_q8 = false) {
        (void) cls;
        linear(Mr <= 64 ? "gemm_dec" : "gemm_dec_big", mode, Mr, N, K, A, A32, K, W, q, ep, Wt, true, a_q8);
    };
    float * ao32 = q5 ? d_ao32_.as<float>() : nullptr;
    // Q5_0: attention passes whose rows all take the one_chunk kernel emit the Q8_0 rows
    // themselves; otherwise their f32 output is quantized by the GEMM call
    const bool kq = m->kq;  // K-quants: GEMMs quantize f32 rows to Q8_K themselves (no producer rows)
    kq_rmul_ = kq && qf_k_repacked(m->qfmt) ? (const uint8_t *) (dv + st_rmul_) : nullptr;
    const bool fq_self = q5 && !kq && self_oc && !self_tl && !sh.self_sm;
    const bool fq_cross = q5 && !kq && cross_oc && !cross_tl && !sh.cross_sm;
    float * xn32 = kq ? d_xn32_.as<float>() : nullptr;  // the f32 LayerNorm rows a K-quant GEMM quantizes

    {
        ProfScope ps(prof, stream, "embed");
        if (kq) embed_tokens_f32(stream, m->te32.as<float>(), m->d_pe, d_tok, d_pos, R, d, d_x_.as<float>());
        else if (q5) embed_tokens_q5(stream, m->q_te, m->d_pe, d_tok, d_pos, R, d, d_x_.as<float>());
        else embed_tokens(stream, m->d_te, m->d_pe, d_tok, d_pos, R, d, d_x_.as<float>());
    }
    const float kq_scale = powf(64.0f, -0.25f);
    const size_t self_stride = (size_t) cap_slots * kv_cells * d;
    const size_t cross_stride = (size_t) cap_slots * hp.n_audio_ctx * d;  // per layer (capacity)
    // one_chunk / tiled cross attention of layer l (soft_max rows: attn_decoder_softmax at the call site)
    auto cross_attn = [&](int l, const _Float16 * qv, _Float16 * o16, float * o32, int8_t * q8, float * q8d) {
        attn_decoder(stream, qv, d, cross_k_.as<_Float16>() + l * cross_stride, cross_v_.as<_Float16>() + l * cross_stride,
                     64, T * 64, d_rc, R, nullptr, H, kq_scale, T, o16, d, cross_oc, cross_tl, o32, true, q8, q8d);
    };
    auto resid_full = [&](const _Float16 * A, const float * A32, const _Float16 * W, const _Float16 * Wt,
                          const Q5W & q, int K, const float * bias, bool a_q8 = false) {
        EpiParams ep;
        ep.bias = bias;
        ep.resid = d_x_.as<float>();
        ep.out32 = d_x_.as<float>();
        ep.ldo = d;
        G("resid", EPI_RESID_F32, d, K, A, A32, W, Wt, q, ep, R, a_q8);
    };
    auto ln = [&](const float * w, const float * b) {
        ProfScope ps(prof, stream, "layernorm");
        layernorm_f16(stream, d_x_.as<float>(), R, d, w, b, hp.eps, d_xn_.as<_Float16>(), d, nullptr, xn32, q8a(),
                      q8d());
    };
    // quantized decode passes of <= 32 rows (the bench's greedy steps): the residual matmuls (attn.out,
    // cross_attn.out, mlp.2) write split-K partial tiles and resid_layernorm adds them to the residual
    // stream with bias and emits the next LayerNorm as f16 AND as Q8_0 rows (the next GEMM's operand):
    // one launch where a full-epilogue GEMM plus a LayerNorm launch were
    const bool q5p = q5 && !kq && R <= 32 && !sh.self_sm && !sh.cross_sm && !sh.capture;
    auto resid_q5p = [&](const _Float16 * A16, const float * A32, const Q5W & q, int K, const float * bias,
                         const float * lnw, const float * lnb, bool a_q8, const int8_t * qa = nullptr,
                         const float * qd = nullptr) {
        EpiParams ep;
        ep.out32 = gws_.partial;
        if (gws_.partial_floats < q5_partial_floats(d, K)) throw std::runtime_error("decode: partial workspace");
        linear("gemm_dec", EPI_PARTIAL, R, d, K, A16, A32, K, nullptr, q, ep, nullptr, true, a_q8, qa, qd);
        ProfScope ps(prof, stream, "layernorm");
        resid_layernorm(stream, R, d, q5_partial_splits(K), gws_.partial, bias, d_x_.as<float>(), lnw, lnb, hp.eps,
                        d_xn_.as<_Float16>(), d, lnw ? q8a() : nullptr, lnw ? q8d() : nullptr);
    };
    if (q5p) ln(m->dec[0].attn_ln_w, m->dec[0].attn_ln_b);  // layer 0's attn_ln (with its Q8_0 rows)
    for (int l = 0; l < hp.n_text_layer && q5p; ++l) {
        const DecLayerW & L = m->dec[l];
        const DecLayerW * nx = l + 1 < hp.n_text_layer ? &m->dec[l + 1] : nullptr;
        _Float16 * Kl = self_k_.as<_Float16>() + l * self_stride;
        _Float16 * Vl = self_v_.as<_Float16>() + l * self_stride;
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
            ep.row_off = d_rowoff;
            ep.Tpad = kv_cells * 64;
            G("qkv", EPI_QKV_DEC, 3 * d, d, d_xn_.as<_Float16>(), nullptr, L.w_qkv, L.t_qkv, L.q_qkv, ep, R, true);
        }
        {
            ProfScope ps(prof, stream, "attn_self");
            attn_decoder(stream, d_q_.as<_Float16>(), d, Kl, Vl, 64, kv_cells * 64, d_rs, R, d_keys, H, 1.0f, max_keys,
                         d_ao_.as<_Float16>(), d, self_oc, self_tl, fq_self ? nullptr : ao32, sh.self_list,
                         fq_self ? q8a() : nullptr, fq_self ? q8d() : nullptr);
        }
        resid_q5p(d_ao_.as<_Float16>(), ao32, L.q_o, d, L.b_o, L.cross_ln_w, L.cross_ln_b, fq_self);
        {
            EpiParams ep;
            ep.bias = L.cb_q;
            ep.out16 = d_q_.as<_Float16>();
            ep.ldo = d;
            G("cq", EPI_F16, d, d, d_xn_.as<_Float16>(), nullptr, L.cw_q, L.t_cq, L.q_cq, ep, R, true);
        }
        {
            ProfScope ps(prof, stream, "attn_cross", 4.0 * R * (double) n_ctx_pad * d, 2.0 * 2.0 * sh.n_clips * (double) T * d);
            cross_attn(l, d_q_.as<_Float16>(), d_ao_.as<_Float16>(), fq_cross ? nullptr : ao32, fq_cross ? q8a() : nullptr,
                       fq_cross ? q8d() : nullptr);
        }
        resid_q5p(d_ao_.as<_Float16>(), ao32, L.q_co, d, L.cb_o, L.mlp_ln_w, L.mlp_ln_b, fq_cross);
        {
            EpiParams ep;
            ep.bias = L.b_mlp0;
            ep.gelu_tab = m->gelu_tab;
            ep.out16 = d_h_.as<_Float16>();
            ep.ldo = 4 * d;
            // GELU outputs are F16 table values: exact as the f32 tensor the reference quantizes; their
            // Q8_0 rows (mlp.2's operand) come from the MLP0 epilogue
            ep.q8 = q8h_.as<int8_t>();
            ep.q8d = q8hd_.as<float>();
            G("mlp0", EPI_GELU_F16, 4 * d, d, d_xn_.as<_Float16>(), nullptr, L.w_mlp0, L.t_mlp0, L.q_mlp0, ep, R, true);
        }
        resid_q5p(d_h_.as<_Float16>(), nullptr, L.q_mlp1, 4 * d, L.b_mlp1, nx ? nx->attn_ln_w : nullptr,
                  nx ? nx->attn_ln_b : nullptr, true, q8h_.as<int8_t>(), q8hd_.as<float>());
    }
    for (int l = 0; l < hp.n_text_layer && !q5p; ++l) {
        const DecLayerW & L = m->dec[l];
        _Float16 * Kl = self_k_.as<_Float16>() + l * self_stride;
        _Float16 * Vl = self_v_.as<_Float16>() + l * self_stride;
        ln(L.attn_ln_w, L.attn_ln_b);
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
            ep.row_off = d_rowoff;
            ep.Tpad = kv_cells * 64;
            G("qkv", EPI_QKV_DEC, 3 * d, d, d_xn_.as<_Float16>(), xn32, L.w_qkv, L.t_qkv, L.q_qkv, ep, R, q5 && !kq);
        }
        {
            ProfScope ps(prof, stream, "attn_self");
            // one_chunk rows all on contiguous cell runs: the list-free kernel (see k_attn_step)
            attn_decoder(stream, d_q_.as<_Float16>(), d, Kl, Vl, 64, kv_cells * 64, d_rs, R, d_keys, H, 1.0f, max_keys,
                         d_ao_.as<_Float16>(), d, self_oc, self_tl, fq_self ? nullptr : ao32, sh.self_list,
                         fq_self ? q8a() : nullptr, fq_self ? q8d() : nullptr);
            if (sh.self_sm)  // masked soft_max with scale 1 (Q, K pre-scaled; whisper.cpp:2614-2628)
                attn_decoder_softmax(stream, d_q_.as<_Float16>(), d, Kl, Vl, 64, kv_cells * 64, d_rs, R, d_keys, H, 1.0f,
                                     max_keys,
                                     d_ao_.as<_Float16>(), d, nullptr, nullptr, 0, ao32);
        }
        resid_full(d_ao_.as<_Float16>(), ao32, L.w_o, L.t_o, L.q_o, d, L.b_o, fq_self);
        ln(L.cross_ln_w, L.cross_ln_b);
        {
            EpiParams ep;
            ep.bias = L.cb_q;
            ep.out16 = d_q_.as<_Float16>();
            ep.ldo = d;
            G("cq", EPI_F16, d, d, d_xn_.as<_Float16>(), xn32, L.cw_q, L.t_cq, L.q_cq, ep, R, q5 && !kq);
        }
        {
            // bytes: cross K and V of each row's clip (the HBM-bound part of a decode step)
            ProfScope ps(prof, stream, "attn_cross", 4.0 * R * (double) n_ctx_pad * d, 2.0 * 2.0 * sh.n_clips * (double) T * d);
            cross_attn(l, d_q_.as<_Float16>(), d_ao_.as<_Float16>(), fq_cross ? nullptr : ao32, fq_cross ? q8a() : nullptr,
                       fq_cross ? q8d() : nullptr);
            if (sh.cross_sm)  // soft_max_ext(KQ, nullptr, KQscale) over n_audio_ctx keys (whisper.cpp:2697-2738)
                attn_decoder_softmax(stream, d_q_.as<_Float16>(), d, cross_k_.as<_Float16>() + l * cross_stride,
                                     cross_v_.as<_Float16>() + l * cross_stride, 64, T * 64, d_rc, R, nullptr, H, kq_scale, T,
                                     d_ao_.as<_Float16>(), d, sh.capture ? amap_.as<int>() + l * H : nullptr,
                                     sh.capture ? cap_.as<float>() : nullptr, R, ao32, sm_ws(), sm_ws_floats());
        }
        resid_full(d_ao_.as<_Float16>(), ao32, L.cw_o, L.t_co, L.q_co, d, L.cb_o, fq_cross);
        ln(L.mlp_ln_w, L.mlp_ln_b);
        {
            EpiParams ep;
            ep.bias = L.b_mlp0;
            ep.gelu_tab = m->gelu_tab;
            ep.out16 = d_h_.as<_Float16>();
            ep.ldo = 4 * d;
            G("mlp0", EPI_GELU_F16, 4 * d, d, d_xn_.as<_Float16>(), xn32, L.w_mlp0, L.t_mlp0, L.q_mlp0, ep, R, q5 && !kq);
        }
        resid_full(d_h_.as<_Float16>(), nullptr, L.w_mlp1, L.t_mlp1, L.q_mlp1, 4 * d, L.b_mlp1);
    }
    launch_logits(sh);
}

// F16 passes of <= 32 rows: the per-layer chain of decode-row GEMMs over rows [r0, r0 + n) of the pass.
// Each residual matmul site (attn.out, cross_attn.out, mlp.2) is either
//   split: split-K partial tiles + resid_layernorm, which adds bias + residual and writes the next
//          LayerNorm's f16 rows for the next matmul (2 launches), or
//   whole-K (passes of <= whole_k_rows() rows): one launch (gemm_rows_res) adding the same partial
//          sums in the same order, bias and residual; the next matmul runs the LayerNorm in its
//          prologue (gemm_rows_lnx) with the statistics in the order of the kernel it replaces --
//          bit-identical to the split chain, so a clip's result does not depend on its pass size.
// Whole-K saves a launch per site but every block of the consumer recomputes the row statistics
// from the f32 rows, and the exact split-order reduction costs more than the launch it saves:
// 36.8 vs 32.5 us per layer at 1 row, 48.3 vs 36.3 at 8 (profiles/archive/r04h_chain_ab.txt), so it is off
// by default (whole_k_rows() = 0) and kept as a verified alternative. Earlier measured alternatives
// (profiles/archive/r02e_ab.txt, the round-3 ticket finish) lost on the launch boundary or the in-launch seam.
// soft_max rows (flash_attn = false) and DTW captures run the soft_max attention launches inside the
// same chain. Every kernel here is row-independent: the row activations / GEMM outputs are addressed
// from row r0, the attention kernels take the pass's AttnRow entries r0.. (absolute q_row) and the
// key-split soft_max workspace of those rows, so a row group's results equal the whole pass's.
void Engine::fused_part(const DecShape & sh, int r0, int n, hipStream_t s, const GemmWs * ws) {
    const HParams & hp = m->hp;
    const int d = hp.n_text_state, H = hp.n_text_head, T = n_ctx();
    const int n_ctx_pad = (T + 255) / 256 * 256;
    char * dv = d_stg_.as<char>();
    const int * d_tok = (const int *) (dv + st_tok_) + r0;
    const int * d_pos = (const int *) (dv + st_pos_) + r0;
    const int64_t * d_rowoff = (const int64_t *) (dv + st_rowoff_) + r0;
    const AttnRow * d_rs = (const AttnRow *) (dv + st_rs_) + r0;
    const AttnRow * d_rc = (const AttnRow *) (dv + st_rc_) + r0;
    const int * d_keys = (const int *) (dv + st_keys_);
    const int max_keys = sh.max_keys;
    const bool whole_k = sh.R <= whole_k_rows() && gemm_rows_exact_applies(sh.R, d);
    const float kq_scale = powf(64.0f, -0.25f);
    const size_t self_stride = (size_t) cap_slots * kv_cells * d;
    const size_t cross_stride = (size_t) cap_slots * hp.n_audio_ctx * d;
    const size_t sm_off = attn_softmax_ws_floats(r0, H);
    const bool smw_ok = sm_ws_.ptr && sm_off < sm_ws_.bytes / 4;
    float * smw = smw_ok ? sm_ws_.as<float>() + sm_off : nullptr;
    const size_t smw_floats = smw_ok ? sm_ws_.bytes / 4 - sm_off : 0;
    // row-relative operands of the matmuls / LayerNorms; attention reads q and writes its output at
    // the absolute rows (AttnRow.q_row) of the pass buffers
    float * x = d_x_.as<float>() + (size_t) r0 * d;
    _Float16 * xn = d_xn_.as<_Float16>() + (size_t) r0 * d;
    _Float16 * qb = d_q_.as<_Float16>() + (size_t) r0 * d;
    _Float16 * aob = d_ao_.as<_Float16>() + (size_t) r0 * d;
    _Float16 * hr = d_h_.as<_Float16>() + (size_t) r0 * 4 * d;
    _Float16 * q_abs = d_q_.as<_Float16>();
    _Float16 * ao_abs = d_ao_.as<_Float16>();
    {
        ProfScope ps(prof, s, "embed");
        embed_tokens(s, m->d_te, m->d_pe, d_tok, d_pos, n, d, x);
    }
    // consumer of a LayerNorm (QKV, cross-Q, mlp.0): from the f16 rows the split producer wrote, or
    // with the LayerNorm in its prologue; algorithmic bytes: weights + activation rows once
    // order: 1 for layer 0's attn_ln (layernorm_f16's statistics), 0 after a residual site (resid_layernorm's)
    auto consumer = [&](int mode, int N, const float * lnw, const float * lnb, const _Float16 * Wt,
                        const EpiParams & ep, int order) {
        if (whole_k) {
            ProfScope ps(prof, s, "gemm_dec", 2.0 * n * (double) N * d, 2.0 * (double) N * d + 4.0 * n * d);
            gemm_rows_lnx(s, mode, order, n, N, d, x, lnw, lnb, hp.eps, Wt, ep);
        } else {
            ProfScope ps(prof, s, "gemm_dec", 2.0 * n * (double) N * d, 2.0 * ((double) n * d + (double) N * d));
            gemm(s, mode, n, N, d, xn, d, nullptr, d, ep, ws, Wt);
        }
    };
    // residual matmul; lnw / lnb: the LayerNorm of the next consumer (null after the last layer)
    auto resid = [&](const _Float16 * A, const _Float16 * Wt, int K, const float * bias, const float * lnw,
                     const float * lnb) {
        if (whole_k) {
            ProfScope ps(prof, s, "gemm_dec", 2.0 * n * (double) d * K, 2.0 * ((double) n * K + (double) d * K));
            gemm_rows_res(s, n, d, K, A, Wt, bias, x);
            return;
        }
        {
            ProfScope ps(prof, s, "gemm_dec", 2.0 * n * (double) d * K, 2.0 * ((double) n * K + (double) d * K));
            gemm(s, EPI_PARTIAL, n, d, K, A, K, nullptr, K, EpiParams(), ws, Wt);
        }
        ProfScope ps(prof, s, "layernorm");
        resid_layernorm(s, n, d, gemm_partial_splits(K), ws->partial, bias, x, lnw, lnb, hp.eps, xn, d);
    };
    if (!whole_k) {  // layer 0's attn_ln of the embeddings
        ProfScope ps(prof, s, "layernorm");
        layernorm_f16(s, x, n, d, m->dec[0].attn_ln_w, m->dec[0].attn_ln_b, hp.eps, xn, d, nullptr, nullptr, nullptr,
                      nullptr);
    }
    for (int l = 0; l < hp.n_text_layer; ++l) {
        const DecLayerW & L = m->dec[l];
        const DecLayerW * nx = l + 1 < hp.n_text_layer ? &m->dec[l + 1] : nullptr;
        _Float16 * Kl = self_k_.as<_Float16>() + l * self_stride;
        _Float16 * Vl = self_v_.as<_Float16>() + l * self_stride;
        const _Float16 * Kc = cross_k_.as<_Float16>() + l * cross_stride;
        const _Float16 * Vc = cross_v_.as<_Float16>() + l * cross_stride;
        {
            EpiParams ep;
            ep.bias = L.b_q;
            ep.bias2 = L.b_v;
            ep.scale = kq_scale;
            ep.out16 = qb;
            ep.ldo = d;
            ep.out16b = Kl;
            ep.out16c = Vl;
            ep.d = d;
            ep.row_off = d_rowoff;
            ep.Tpad = kv_cells * 64;
            consumer(EPI_QKV_DEC, 3 * d, L.attn_ln_w, L.attn_ln_b, L.t_qkv, ep, l == 0 ? 1 : 0);
        }
        {
            ProfScope ps(prof, s, "attn_self");
            attn_decoder(s, q_abs, d, Kl, Vl, 64, kv_cells * 64, d_rs, n, d_keys, H, 1.0f, max_keys, ao_abs, d,
                         sh.self_oc, sh.self_tl, nullptr, sh.self_list, nullptr, nullptr);
            // flash_attn = false rows: masked soft_max (scale 1; Q, K pre-scaled), one block per (row, head):
            // at most n_text_ctx keys, so one launch beats the key-split form's three at configs[4]'s one-row
            // steps (the cross rows below, 1500 keys, take the key-split form)
            if (sh.self_sm)
                attn_decoder_softmax(s, q_abs, d, Kl, Vl, 64, kv_cells * 64, d_rs, n, d_keys, H, 1.0f, max_keys, ao_abs,
                                     d, nullptr, nullptr, 0, nullptr);
        }
        resid(aob, L.t_o, d, L.b_o, L.cross_ln_w, L.cross_ln_b);
        {
            EpiParams ep;
            ep.bias = L.cb_q;
            ep.out16 = qb;
            ep.ldo = d;
            consumer(EPI_F16, d, L.cross_ln_w, L.cross_ln_b, L.t_cq, ep, 0);
        }
        {
            ProfScope ps(prof, s, "attn_cross", 4.0 * n * (double) n_ctx_pad * d, 2.0 * 2.0 * sh.n_clips * (double) T * d);
            attn_decoder(s, q_abs, d, Kc, Vc, 64, T * 64, d_rc, n, nullptr, H, kq_scale, T, ao_abs, d, sh.cross_oc,
                         sh.cross_tl, nullptr, true, nullptr, nullptr);
            if (sh.cross_sm)  // soft_max_ext over n_audio_ctx keys (key-split), DTW capture of the alignment heads
                attn_decoder_softmax(s, q_abs, d, Kc, Vc, 64, T * 64, d_rc, n, nullptr, H, kq_scale, T, ao_abs, d,
                                     sh.capture ? amap_.as<int>() + l * H : nullptr,
                                     sh.capture ? cap_.as<float>() : nullptr, sh.R, nullptr, smw, smw_floats);
        }
        resid(aob, L.t_co, d, L.cb_o, L.mlp_ln_w, L.mlp_ln_b);
        {
            EpiParams ep;
            ep.bias = L.b_mlp0;
            ep.gelu_tab = m->gelu_tab;
            ep.out16 = hr;
            ep.ldo = 4 * d;
            consumer(EPI_GELU_F16, 4 * d, L.mlp_ln_w, L.mlp_ln_b, L.t_mlp0, ep, 0);
        }
        resid(hr, L.t_mlp1, 4 * d, L.b_mlp1, nx ? nx->attn_ln_w : nullptr, nx ? nx->attn_ln_b : nullptr);
    }
}

void Engine::launch_logits(const DecShape & sh) {
    const HParams & hp = m->hp;
    const int n_logit_rows = sh.n_logit, d = hp.n_text_state, nv = hp.n_vocab;
    if (n_logit_rows <= 0) return;
    const bool kq = m->kq;
    const int * d_lsel = (const int *) (d_stg_.as<char>() + st_lsel_);
    {
        ProfScope ps(prof, stream, "layernorm");
        layernorm_f16(stream, d_x_.as<float>(), n_logit_rows, d, m->d_ln_w, m->d_ln_b, hp.eps, d_xl_.as<_Float16>(), d,
                      d_lsel, kq ? d_xl32_.as<float>() : nullptr, q8a(), q8d());
    }
    kq_rmul_ = nullptr;  // the token embedding is not repacked (a get_rows tensor): quantize_row_q8_K
    EpiParams ep;
    ep.out32 = logits_.as<float>();
    ep.ldo = nv;
    linear(n_logit_rows <= 64 ? "gemm_logits" : "gemm_logits_big", EPI_F32, n_logit_rows, nv, d, d_xl_.as<_Float16>(),
           kq ? d_xl32_.as<float>() : nullptr, d, m->d_te, m->q_te, ep, m->d_te_t, true, m->q5 && !kq);
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

void Engine::step_post(const StepPost & post, const std::vector<LogitJob> & jobs, const VocabInfo & vi_in,
                       std::vector<TokenOut> & out, std::vector<float> & nosp_out, float * probs_host,
                       float * logprobs_host) {
    const int nv = m->hp.n_vocab;
    const int n = (int) jobs.size();
    const int nn = (int) post.nosp.size();
    out.resize(n);
    nosp_out.resize(nn);
    row0_.alloc((size_t) cap_slots * nv * 4);
    rmx_.alloc((size_t) cap_slots * RMX * 4);
    for (const auto & e : post.rowmax)
        if (e.x < 0 || e.x >= cap_slots || e.y < 0 || e.y >= RMX) throw std::runtime_error("step_post: bad row entry");
    for (const auto & e : post.nosp)
        if (e.x < 0 || e.x >= cap_slots || e.y < 1 || e.y > RMX) throw std::runtime_error("step_post: bad nosp entry");

    // one packed upload: row-max entries | row-0 map | nosp requests | jobs | suppress list
    size_t o = 0;
    auto sec = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 63) / 64 * 64;
        return at;
    };
    const size_t o_rm = sec(post.rowmax.size() * sizeof(int4)), o_r0 = sec(post.row0.size() * sizeof(int2)),
                 o_ns = sec(nn * sizeof(int2)), o_jobs = sec(n * sizeof(LogitJob)),
                 o_sup = sec((size_t) std::max(vi_in.n_suppress, 0) * 4);
    post_h_.alloc(std::max<size_t>(o, 64));
    post_d_.alloc(std::max<size_t>(o, 64));
    char * h = post_h_.as<char>();
    if (!post.rowmax.empty()) memcpy(h + o_rm, post.rowmax.data(), post.rowmax.size() * sizeof(int4));
    if (!post.row0.empty()) memcpy(h + o_r0, post.row0.data(), post.row0.size() * sizeof(int2));
    if (nn) memcpy(h + o_ns, post.nosp.data(), nn * sizeof(int2));
    if (n) memcpy(h + o_jobs, jobs.data(), n * sizeof(LogitJob));
    if (vi_in.n_suppress > 0) memcpy(h + o_sup, vi_in.suppress_list, (size_t) vi_in.n_suppress * 4);
    char * dv = post_d_.as<char>();
    if (o) OWK_HIP_CHECK(hipMemcpyAsync(dv, h, o, hipMemcpyHostToDevice, stream));

    // results: token records | nosp probs
    const size_t r_tok = 0, r_ns = ((size_t) n * sizeof(TokenOut) + 63) / 64 * 64;
    const size_t r_bytes = r_ns + (size_t) nn * 4;
    post_out_h_.alloc(std::max<size_t>(r_bytes, 64));
    post_out_d_.alloc(std::max<size_t>(r_bytes, 64));
    {
        ProfScope ps(prof, stream, "logits_proc");
        rowmax_update(stream, logits_.as<float>(), nv, (const int4 *) (dv + o_rm), (int) post.rowmax.size(),
                      rmx_.as<float>(), RMX);
        logits_copy_rows(stream, logits_.as<float>(), nv, (const int2 *) (dv + o_r0), (int) post.row0.size(),
                         row0_.as<float>());
        nosp_probs(stream, row0_.as<float>(), nv, (const int2 *) (dv + o_ns), nn, rmx_.as<float>(), RMX,
                   m->vocab.nosp, (float *) (post_out_d_.as<char>() + r_ns));
        if (n) {
            VocabInfo vi = vi_in;
            vi.suppress_list = (const int *) (dv + o_sup);
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
            bool any_nosp = false;
            for (const LogitJob & j : jobs) any_nosp |= (j.flags & 256) != 0;  // LF_NEED_NOSP
            lg_ws_.alloc(process_logits_ws_bytes(n));
            owk::process_logits(stream, logits_.as<float>(), nv, (const LogitJob *) (dv + o_jobs), n, vi,
                                (TokenOut *) (post_out_d_.as<char>() + r_tok), lp, pr, any_nosp, lg_ws_.ptr,
                                lg_ws_.bytes);
            if (pr) OWK_HIP_CHECK(hipMemcpyAsync(probs_host, pr, (size_t) n * nv * 4, hipMemcpyDeviceToHost, stream));
            if (lp) OWK_HIP_CHECK(hipMemcpyAsync(logprobs_host, lp, (size_t) n * nv * 4, hipMemcpyDeviceToHost, stream));
        }
    }
    if (r_bytes) OWK_HIP_CHECK(hipMemcpyAsync(post_out_h_.ptr, post_out_d_.ptr, r_bytes, hipMemcpyDeviceToHost, stream));
    sync();
    if (n) memcpy(out.data(), post_out_h_.as<char>() + r_tok, (size_t) n * sizeof(TokenOut));
    if (nn) memcpy(nosp_out.data(), post_out_h_.as<char>() + r_ns, (size_t) nn * 4);
}

void Engine::save_logits_state(int slot, int n_rows, std::vector<float> & rowmax, std::vector<float> & row0) {
    const int nv = m->hp.n_vocab;
    sync();
    rowmax.resize(std::min(n_rows, RMX));
    row0.resize(nv);
    if (!rmx_.ptr || !row0_.ptr || slot >= cap_slots) {
        std::fill(rowmax.begin(), rowmax.end(), 0.0f);
        std::fill(row0.begin(), row0.end(), 0.0f);
        return;
    }
    if (!rowmax.empty())
        OWK_HIP_CHECK(hipMemcpy(rowmax.data(), rmx_.as<float>() + (size_t) slot * RMX, rowmax.size() * 4,
                                hipMemcpyDeviceToHost));
    OWK_HIP_CHECK(hipMemcpy(row0.data(), row0_.as<float>() + (size_t) slot * nv, (size_t) nv * 4, hipMemcpyDeviceToHost));
}

void Engine::load_logits_state(int slot, const std::vector<float> & rowmax, const std::vector<float> & row0) {
    const int nv = m->hp.n_vocab;
    row0_.alloc((size_t) cap_slots * nv * 4);
    rmx_.alloc((size_t) cap_slots * RMX * 4);
    if (slot >= cap_slots) throw std::runtime_error("load_logits_state: slot out of range");
    if (!rowmax.empty())
        OWK_HIP_CHECK(hipMemcpyAsync(rmx_.as<float>() + (size_t) slot * RMX, rowmax.data(),
                                     std::min<size_t>(rowmax.size(), RMX) * 4, hipMemcpyHostToDevice, stream));
    if ((int) row0.size() == nv)
        OWK_HIP_CHECK(hipMemcpyAsync(row0_.as<float>() + (size_t) slot * nv, row0.data(), (size_t) nv * 4,
                                     hipMemcpyHostToDevice, stream));
    else
        OWK_HIP_CHECK(hipMemsetAsync(row0_.as<float>() + (size_t) slot * nv, 0, (size_t) nv * 4, stream));
    sync();
}

} // namespace owk
