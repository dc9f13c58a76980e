// Streaming-SortFormer kernels for gfx950: NeMo log-mel front-end, conv2d subsampling
// pre-encoder, relative-position / plain multi-head attention and the conformer conv module.
//
// The dense linears of the conformer / transformer / head run on the MFMA GEMM of
// k_gemm.hip. Everything here reproduces ggml CPU f32 numerics of the reference graph
// (/root/reference streaming-sortformer/src/sortformer.cpp, cited "ref:<line>"):
// one rounding per ggml op, reference operand order inside each sum (built with
// -ffp-contract=off); only f32 dot-product association differs from the SIMD CPU code.
#include "sf_kernels.h"

namespace owk {
namespace sf {

// ---------------------------------------------------------------------------------
// log-mel (ref:779-894): one block per frame, 512-point radix-2 FFT in LDS.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sf_mel(const float * __restrict__ pcm, int n, const float * __restrict__ win,
                                                const float2 * __restrict__ tw, const float * __restrict__ fb,
                                                int n_mels, int n_compute, int n_frames_out, float * __restrict__ mel) {
    __shared__ float2 buf[512];
    __shared__ float pw[257];
    const int fr = blockIdx.x, tid = threadIdx.x;
    if (fr >= n_compute) {  // frames past seq_len stay zero (calloc, ref:840, 888)
        for (int m = tid; m < n_mels; m += 256) mel[(size_t) m * n_frames_out + fr] = 0.0f;
        return;
    }
    const int off = fr * 160;
    for (int j = tid; j < 512; j += 256) {
        const int i = off + j - 256;  // constant zero pad of n_fft/2 (ref:807-811)
        float x = 0.0f;
        if (i >= 0 && i < n) x = i == 0 ? pcm[0] : pcm[i] - 0.97f * pcm[i - 1];  // pre-emphasis (ref:800-805)
        const float v = win[j] * x;
        buf[__brev((unsigned) j) >> 23] = make_float2(v, 0.0f);  // bit-reversal permutation (ref:218-227)
    }
    __syncthreads();
    int twoff = 0;
    for (int len = 2; len <= 512; len <<= 1) {  // butterfly stages (ref:229-262)
        const int half = len >> 1;
        const int g = tid / half, k = tid - g * half;
        const int ia = g * len + k, ib = ia + half;
        const float2 w = tw[twoff + k];
        const float2 a = buf[ia], b = buf[ib];
        const float tr = w.x * b.x - w.y * b.y;
        const float ti = w.x * b.y + w.y * b.x;
        buf[ia] = make_float2(a.x + tr, a.y + ti);
        buf[ib] = make_float2(a.x - tr, a.y - ti);
        __syncthreads();
        twoff += half;
    }
    for (int k = tid; k < 257; k += 256) {
        const float2 c = buf[k];
        pw[k] = c.x * c.x + c.y * c.y;
    }
    __syncthreads();
    for (int m = tid; m < n_mels; m += 256) {  // mel = fb . P in float, ln(. + 2^-24) (ref:863-873)
        const float * row = fb + (size_t) m * 257;
        float sum = 0.0f;
        for (int k = 0; k < 257; ++k) sum += row[k] * pw[k];
        mel[(size_t) m * n_frames_out + fr] = logf(sum + 5.9604644775390625e-08f);
    }
}

void mel(hipStream_t s, const float * pcm, int n_samples, const float * win512, const float * tw, const float * fb,
         int n_mels, int n_compute, int n_frames_out, float * out) {
    if (n_frames_out <= 0) return;
    OWK_LAUNCH(k_sf_mel, dim3(n_frames_out), dim3(256), 0, s, pcm, n_samples, win512, (const float2 *) tw, fb,
                       n_mels, n_compute, n_frames_out, out);
}

// ---------------------------------------------------------------------------------
// pre-encoder (ref:900-1044)
// ---------------------------------------------------------------------------------
// Conv2d(1 -> C, 3x3, s2, p1): im2col order (ic, ky = time, kx = freq) (ops.cpp:6563+),
// then + bias (ggml_add), ReLU. One thread per output channel, 8 freq bins per block.
__global__ __launch_bounds__(256) void k_sf_conv0(const float * __restrict__ mel, int ld, int c0, int T_in, int n_mels,
                                                  const float * __restrict__ w, const float * __restrict__ b, int C,
                                                  float * __restrict__ out, int F1) {
    const int t = blockIdx.x, f0 = blockIdx.y * 8, c = threadIdx.x;
    if (c >= C) return;
    float wk[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) wk[i] = w[c * 9 + i];
    const float bc = b[c];
    for (int f = f0; f < min(f0 + 8, F1); ++f) {
        float sum = 0.0f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const int ti = 2 * t - 1 + ky;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int fi = 2 * f - 1 + kx;
                const float x = (ti >= 0 && ti < T_in && fi >= 0 && fi < n_mels) ? mel[(size_t) fi * ld + c0 + ti] : 0.0f;
                sum += wk[ky * 3 + kx] * x;
            }
        }
        const float v = sum + bc;
        out[((size_t) t * F1 + f) * C + c] = v > 0.0f ? v : 0.0f;
    }
}

void conv0(hipStream_t s, const float * mel, int ld, int c0, int T_in, int n_mels, const float * w, const float * b,
           int C, float * out, int T1, int F1) {
    if (C > 256) throw std::runtime_error("sf::conv0: C > 256");
    OWK_LAUNCH(k_sf_conv0, dim3(T1, (F1 + 7) / 8), dim3(256), 0, s, mel, ld, c0, T_in, n_mels, w, b, C, out,
                       F1);
}

// depthwise 3x3 s2 p1 (ggml_compute_forward_conv_2d_dw_whcn, ops.cpp:7035-7070) + bias
__global__ void k_sf_dwconv(const float * __restrict__ in, int Ti, int Fi, int C, const float * __restrict__ w,
                            const float * __restrict__ b, float * __restrict__ out, int To, int Fo) {
    const size_t idx = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t) To * Fo * C;
    if (idx >= total) return;
    const int c = (int) (idx % C);
    const int f = (int) ((idx / C) % Fo);
    const int t = (int) (idx / ((size_t) C * Fo));
    float sum = 0.0f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
        const int ti = 2 * t - 1 + ky;
        if (ti < 0 || ti >= Ti) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int fi = 2 * f - 1 + kx;
            if (fi < 0 || fi >= Fi) continue;
            sum += w[c * 9 + ky * 3 + kx] * in[((size_t) ti * Fi + fi) * C + c];
        }
    }
    out[idx] = sum + b[c];
}

void dwconv(hipStream_t s, const float * in, int Ti, int Fi, int C, const float * w, const float * b, float * out,
            int To, int Fo) {
    const size_t total = (size_t) To * Fo * C;
    if (!total) return;
    OWK_LAUNCH(k_sf_dwconv, dim3((unsigned) ((total + 255) / 256)), dim3(256), 0, s, in, Ti, Fi, C, w, b, out,
                       To, Fo);
}

// pointwise conv as an f32 GEMM: 64 positions x 64 channels per block, 4x4 per thread
template <int FLAT>
__global__ __launch_bounds__(256) void k_sf_pwconv(const float * __restrict__ in, int P, int C,
                                                   const float * __restrict__ w, const float * __restrict__ b, int Fo,
                                                   float * __restrict__ out32, _Float16 * __restrict__ out16, int ld16) {
    __shared__ float As[16][68], Ws[16][68];
    const int tid = threadIdx.x;
    const int p0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
    const int tp = tid >> 4, tn = tid & 15;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < C; k0 += 16) {
        for (int i = tid; i < 64 * 16; i += 256) {
            const int r = i >> 4, kk = i & 15;
            const int p = p0 + r, n = n0 + r;
            As[kk][r] = (p < P && k0 + kk < C) ? in[(size_t) p * C + k0 + kk] : 0.0f;
            Ws[kk][r] = (n < C && k0 + kk < C) ? w[(size_t) n * C + k0 + kk] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            const float4 a = *(const float4 *) &As[kk][tp * 4];
            const float4 ww = *(const float4 *) &Ws[kk][tn * 4];
            const float av[4] = {a.x, a.y, a.z, a.w}, wv[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += av[i] * wv[j];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = p0 + tp * 4 + i;
        if (p >= P) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tn * 4 + j;
            if (n >= C) continue;
            float v = acc[i][j] + b[n];
            v = v > 0.0f ? v : 0.0f;
            if (FLAT) {
                const int t = p / Fo, f = p - t * Fo;
                out16[(size_t) t * ld16 + n * Fo + f] = (_Float16) v;
            } else {
                out32[(size_t) p * C + n] = v;
            }
        }
    }
}

void pwconv(hipStream_t s, const float * in, int P, int C, const float * w, const float * b, int flatten, int Fo,
            float * out32, _Float16 * out16, int ld16) {
    if (P <= 0) return;
    const dim3 grid((P + 63) / 64, (C + 63) / 64);
    if (flatten)
        OWK_LAUNCH(k_sf_pwconv<1>, grid, dim3(256), 0, s, in, P, C, w, b, Fo, out32, out16, ld16);
    else
        OWK_LAUNCH(k_sf_pwconv<0>, grid, dim3(256), 0, s, in, P, C, w, b, Fo, out32, out16, ld16);
}

// ---------------------------------------------------------------------------------
// elementwise
// ---------------------------------------------------------------------------------
__global__ void k_sf_scale(const float * __restrict__ x, size_t n, float sc, float * __restrict__ out) {
    const size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = x[i] * sc;
}
void scale(hipStream_t s, const float * x, size_t n, float sc, float * out) {
    if (!n) return;
    OWK_LAUNCH(k_sf_scale, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, n, sc, out);
}
__global__ void k_sf_relu_f16(const float * __restrict__ x, size_t n, _Float16 * __restrict__ out) {
    const size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (_Float16) (x[i] > 0.0f ? x[i] : 0.0f);
}
void relu_f16(hipStream_t s, const float * x, size_t n, _Float16 * out) {
    if (!n) return;
    OWK_LAUNCH(k_sf_relu_f16, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, n, out);
}
__global__ void k_sf_to_f16(const float * __restrict__ x, size_t n, _Float16 * __restrict__ out) {
    const size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (_Float16) x[i];
}
void to_f16(hipStream_t s, const float * x, size_t n, _Float16 * out) {
    if (!n) return;
    OWK_LAUNCH(k_sf_to_f16, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, n, out);
}

// ---------------------------------------------------------------------------------
// attention (ref:1170-1235 relative-position MHSA, ref:1470-1503 transformer MHA)
//
// One block per (head, 8 query rows): 8 heads x T/8 blocks fill the chip at chunk-pass lengths
// (T ~ 400), where 16-row blocks left every CU a single block and no latency hiding. Keys stream
// through LDS in tiles of 64; each tile's global loads are issued into registers one tile ahead
// (they fly while the current tile is computed). The score rows [8][T] stay in LDS for the softmax
// and the P.V pass (whose V tiles are prefetched the same way, the first one under the softmax).
// The relative-position term uses the Transformer-XL shift in closed form: row i, key j reads
// P[T-1-i+j] (the pad/roll/view of ref:1203-1216), so the 64 keys of a tile need 71 consecutive
// P rows. Per-output arithmetic is independent of the tiling (same sums in the same order).
// ---------------------------------------------------------------------------------
constexpr int AQ = 8;    // query rows per block
constexpr int AKT = 64;  // keys per tile

template <int DH, bool REL>
__global__ __launch_bounds__(256) void k_sf_attn(const float * __restrict__ qkv, int ldq, int kcol, int vcol, int T,
                                                 int H, const float * __restrict__ ub, const float * __restrict__ vb,
                                                 const float * __restrict__ P, int ldP, float sc,
                                                 _Float16 * __restrict__ out, float * __restrict__ out32, int Tpad) {
    extern __shared__ float smem[];
    constexpr int LDK = DH + 4;
    constexpr int TPQ = 256 / AQ;                   // threads per query row
    constexpr int KPT = AKT * DH / 256;             // K / V tile floats per thread
    constexpr int PR = AQ - 1 + AKT;                // P rows per tile
    constexpr int PPT = (PR * DH + 255) / 256;      // P tile floats per thread
    float * S = smem;                       // [AQ][Tpad]
    float * Ks = S + AQ * Tpad;             // [AKT][LDK]
    float * Ps = Ks + AKT * LDK;            // [PR][LDK]
    float * Qv = Ps + PR * LDK;             // [AQ][DH] Q + pos_bias_v (REL; LDS keeps the VGPRs for prefetch)
    const int h = blockIdx.x, q0 = blockIdx.y * AQ, tid = threadIdx.x;
    const int ldp = H * DH;
    const int qi = tid / TPQ, kk = tid % TPQ;
    const int qrow = min(q0 + qi, T - 1);

    float kreg[KPT], preg[REL ? PPT : 1];
    auto load_kv = [&](int j0, int col) {
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            const int i = tid + 256 * u, r = i / DH, d = i - r * DH, j = j0 + r;
            kreg[u] = j < T ? qkv[(size_t) j * ldq + col + h * DH + d] : 0.0f;
        }
    };
    auto store_kv = [&]() {
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            const int i = tid + 256 * u, r = i / DH, d = i - r * DH;
            Ks[r * LDK + d] = kreg[u];
        }
    };
    auto load_p = [&](int j0) {
        const int pbase = T - 1 - (q0 + AQ - 1) + j0;
#pragma unroll
        for (int u = 0; u < PPT; ++u) {
            const int i = tid + 256 * u, r = i / DH, d = i - r * DH, p = pbase + r;
            preg[u] = (i < PR * DH && p >= 0 && p < 2 * T - 1) ? P[(size_t) p * ldP + h * DH + d] : 0.0f;
        }
    };
    auto store_p = [&]() {
#pragma unroll
        for (int u = 0; u < PPT; ++u) {
            const int i = tid + 256 * u, r = i / DH, d = i - r * DH;
            if (i < PR * DH) Ps[r * LDK + d] = preg[u];
        }
    };

    load_kv(0, kcol);
    if constexpr (REL) load_p(0);
    float qu[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) {
        const float q = qkv[(size_t) qrow * ldq + h * DH + d];
        qu[d] = REL ? q + ub[h * DH + d] : q;  // Q_u = Q + pos_bias_u (ggml_add, ref:1185)
    }
    if constexpr (REL)
        for (int i = tid; i < AQ * DH; i += 256) {
            const int r = i / DH, d = i - r * DH;
            Qv[i] = qkv[(size_t) min(q0 + r, T - 1) * ldq + h * DH + d] + vb[h * DH + d];
        }

    for (int j0 = 0; j0 < T; j0 += AKT) {
        __syncthreads();  // every thread done with the previous tile
        store_kv();
        if constexpr (REL) store_p();
        __syncthreads();
        if (j0 + AKT < T) {  // next tile in flight during this one
            load_kv(j0 + AKT, kcol);
            if constexpr (REL) load_p(j0 + AKT);
        }
#pragma unroll 1
        for (int rr = 0; rr < AKT / TPQ; ++rr) {  // (unrolled, the LDS reads of both keys were hoisted: 256+ VGPRs)
            const int kj = kk + TPQ * rr;
            const int j = j0 + kj;
            const float * kr = Ks + kj * LDK;
            float ac = 0.0f;
#pragma unroll
            for (int d = 0; d < DH; ++d) ac += qu[d] * kr[d];
            float s;
            if (REL) {
                const float * pr = Ps + ((AQ - 1 - qi) + kj) * LDK;
                const float * qv = Qv + qi * DH;
                float bd = 0.0f;
#pragma unroll 16
                for (int d = 0; d < DH; ++d) bd += qv[d] * pr[d];
                s = (ac + bd) * sc;  // ggml_add(ac, bd) then ggml_scale (ref:1222-1223)
            } else {
                s = ac * sc;
            }
            if (j < T) S[qi * Tpad + j] = s;
        }
    }
    load_kv(0, vcol);  // the first V tile flies under the softmax
    __syncthreads();

    // softmax per row (ggml_compute_forward_soft_max_f32: max, expf, double sum, * (float)(1/sum))
    const int lane = tid & 63, wave = tid >> 6;
    for (int r = wave * (AQ / 4); r < (wave + 1) * (AQ / 4); ++r) {
        float * row = S + r * Tpad;
        float mx = -INFINITY;
        for (int j = lane; j < T; j += 64) mx = fmaxf(mx, row[j]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        double sum = 0.0;
        for (int j = lane; j < T; j += 64) {
            const float e = expf(row[j] - mx);
            row[j] = e;
            sum += (double) e;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
        const float inv = (float) (1.0 / sum);
        for (int j = lane; j < T; j += 64) row[j] *= inv;
    }

    // out = P . V (ggml_mul_mat(attn, V), f32)
    constexpr int NOUT = (AQ * DH + 255) / 256;
    float acc[NOUT];
#pragma unroll
    for (int m = 0; m < NOUT; ++m) acc[m] = 0.0f;
    const float * Vs = Ks;
    for (int j0 = 0; j0 < T; j0 += AKT) {
        __syncthreads();  // softmax rows final / previous V tile consumed
        store_kv();
        __syncthreads();
        if (j0 + AKT < T) load_kv(j0 + AKT, vcol);
        const int nk = min(AKT, T - j0);
#pragma unroll
        for (int m = 0; m < NOUT; ++m) {
            const int o = tid + 256 * m;
            if (o < AQ * DH) {
                const int oq = o / DH, d = o - oq * DH;
                const float * srow = S + oq * Tpad + j0;
                float a = acc[m];
                for (int kj = 0; kj < nk; ++kj) a += srow[kj] * Vs[kj * LDK + d];
                acc[m] = a;
            }
        }
    }
#pragma unroll
    for (int m = 0; m < NOUT; ++m) {
        const int o = tid + 256 * m;
        if (o < AQ * DH) {
            const int oq = o / DH, d = o - oq * DH;
            if (q0 + oq < T) {
                if (out32) out32[(size_t) (q0 + oq) * ldp + h * DH + d] = acc[m];
                else out[(size_t) (q0 + oq) * ldp + h * DH + d] = (_Float16) acc[m];
            }
        }
    }
}

template <int DH, bool REL>
static void launch_attn(hipStream_t s, const float * qkv, int ldq, int kcol, int vcol, int T, int H, const float * u,
                        const float * v, const float * P, int ldP, float sc, _Float16 * out, float * out32) {
    const int Tpad = (T + AKT - 1) / AKT * AKT;
    const size_t lds = ((size_t) AQ * Tpad + (size_t) AKT * (DH + 4) +
                        (REL ? (size_t) (AQ - 1 + AKT) * (DH + 4) + (size_t) AQ * DH : 0)) * sizeof(float);
    if (lds > 160 * 1024) throw std::runtime_error("sf::attention: T too large for the LDS score tile");
    OWK_LAUNCH((k_sf_attn<DH, REL>), dim3(H, (T + AQ - 1) / AQ), dim3(256), lds, s, qkv, ldq, kcol, vcol, T, H,
                       u, v, P, ldP, sc, out, out32, Tpad);
}

void attention(hipStream_t s, int dh, bool rel, const float * qkv, int ldq, int kcol, int vcol, int T, int H,
               const float * u, const float * v, const float * P, float sc, _Float16 * out, float * out32, int ldP) {
    if (T <= 0) return;
    if (ldP <= 0) ldP = H * dh;
    if (dh == 64 && rel)
        launch_attn<64, true>(s, qkv, ldq, kcol, vcol, T, H, u, v, P, ldP, sc, out, out32);
    else if (dh == 24 && !rel)
        launch_attn<24, false>(s, qkv, ldq, kcol, vcol, T, H, u, v, P, ldP, sc, out, out32);
    else if (dh == 64 && !rel)
        launch_attn<64, false>(s, qkv, ldq, kcol, vcol, T, H, u, v, P, ldP, sc, out, out32);
    else
        throw std::runtime_error("sf::attention: unsupported head size");
}

// ---------------------------------------------------------------------------------
// conformer conv module middle (ref:1246-1266): GLU, depthwise conv k (ggml_ssm_conv),
// + bias, SiLU; f16 output feeds pointwise_conv2
// ---------------------------------------------------------------------------------
__global__ void k_sf_glu_dwconv(const float * __restrict__ x, int T, int C, const float * __restrict__ w, int K,
                                const float * __restrict__ b, _Float16 * __restrict__ out) {
    const size_t idx = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t) T * C) return;
    const int c = (int) (idx % C), t = (int) (idx / C);
    const int pad = (K - 1) / 2;
    float sum = 0.0f;
    for (int k = 0; k < K; ++k) {
        const int tt = t - pad + k;
        float g = 0.0f;
        if (tt >= 0 && tt < T) {
            const float a = x[(size_t) tt * 2 * C + c], gate = x[(size_t) tt * 2 * C + C + c];
            g = a * (1.0f / (1.0f + expf(-gate)));
        }
        sum += g * w[c * K + k];
    }
    const float y = sum + b[c];
    out[idx] = (_Float16) (y / (1.0f + expf(-y)));
}

void glu_dwconv(hipStream_t s, const float * x, int T, int C, const float * w, int k, const float * b, _Float16 * out) {
    const size_t n = (size_t) T * C;
    if (!n) return;
    OWK_LAUNCH(k_sf_glu_dwconv, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, T, C, w, k, b, out);
}

}  // namespace sf
}  // namespace owk
