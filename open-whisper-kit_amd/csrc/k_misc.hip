// Front-end (log-mel), normalisation, embedding and im2col kernels, gfx950.
#include "kernels.h"
#include "rln_row.h"

namespace owk {

// ----------------------------------------------------------------------------------
// wave-level reductions (64 lanes)
// ----------------------------------------------------------------------------------

// ----------------------------------------------------------------------------------
// LayerNorm -> f16 (ggml_compute_forward_norm_f32, ref ggml-cpu/ops.cpp:3578-3623,
// followed by the separate ggml_mul / ggml_add of whisper.cpp:2103-2108): mean from a
// double sum rounded to float, variance accumulated in double, scale = 1/sqrtf(var+eps),
// then ((x-mean)*scale)*w + b with one rounding per op (built with -ffp-contract=off).
// One wave per row; the f16 output feeds the next GEMM directly.
// ----------------------------------------------------------------------------------
constexpr int LN_V4 = 8;  // float4 per lane held in registers -> d <= 2048

// LayerNorm of one row held in registers (lane owns float4 groups lane + 64 j)
// o (optional, null: no f16 row), o32 (optional): the f16 / f32 output rows
// yout (optional): the f32 output row kept in registers (what o32 receives; zeros past the row)
__device__ __forceinline__ void ln_row_regs(const float4 (&xv)[LN_V4], int lane, int d, const float * __restrict__ w,
                                            const float * __restrict__ b, float eps, _Float16 * __restrict__ o,
                                            float * __restrict__ o32, int8_t * __restrict__ q8 = nullptr,
                                            float * __restrict__ q8d = nullptr, float4 (*yout)[LN_V4] = nullptr) {
    const int n4 = d >> 2;
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < LN_V4; ++j)
        s += ((double) xv[j].x + (double) xv[j].y) + ((double) xv[j].z + (double) xv[j].w);
    s = wave_sum_d(s);
    const float mean = (float) s / (float) d;
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < LN_V4; ++j) {
        if (lane + 64 * j < n4) {
            const float tx = xv[j].x - mean, ty = xv[j].y - mean, tz = xv[j].z - mean, tw = xv[j].w - mean;
            v += ((double) (tx * tx) + (double) (ty * ty)) + ((double) (tz * tz) + (double) (tw * tw));
        }
    }
    v = wave_sum_d(v);
    const float var = (float) (v / (double) d);
    const float scale = 1.0f / sqrtf(var + eps);
    const float4 * w4 = (const float4 *) w;
    const float4 * b4 = (const float4 *) b;
    if (yout)
#pragma unroll
        for (int j = 0; j < LN_V4; ++j) (*yout)[j] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < LN_V4; ++j) {
        const int i = lane + 64 * j;
        if (64 * j >= n4) break;  // wave-uniform: no lane of this group is in the row
        float4 y = float4{0.f, 0.f, 0.f, 0.f};
        if (i < n4) {
            const float4 ww = w4[i], bb = b4[i];
            y.x = (xv[j].x - mean) * scale * ww.x + bb.x;
            y.y = (xv[j].y - mean) * scale * ww.y + bb.y;
            y.z = (xv[j].z - mean) * scale * ww.z + bb.z;
            y.w = (xv[j].w - mean) * scale * ww.w + bb.w;
            half4 h;
            h[0] = (_Float16) y.x; h[1] = (_Float16) y.y; h[2] = (_Float16) y.z; h[3] = (_Float16) y.w;
            if (o) *(half4 *) (o + 4 * i) = h;
            if (o32) *(float4 *) (o32 + 4 * i) = y;
            if (yout) (*yout)[j] = y;
        }
        if (q8) {
            // Q8_0 of the f32 output (x86 quantize_row_q8_0, as k_quantize_q8): a 32-element
            // block is 8 consecutive float4 = 8 lanes; d % 32 == 0 keeps groups whole
            float m = fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w)));
            m = fmaxf(m, __shfl_xor(m, 1, 8));
            m = fmaxf(m, __shfl_xor(m, 2, 8));
            m = fmaxf(m, __shfl_xor(m, 4, 8));
            if (i < n4) {
                const float id = m != 0.0f ? 127.f / m : 0.0f;
                char4 qv;
                qv.x = (signed char) rintf(y.x * id);
                qv.y = (signed char) rintf(y.y * id);
                qv.z = (signed char) rintf(y.z * id);
                qv.w = (signed char) rintf(y.w * id);
                *(char4 *) (q8 + 4 * i) = qv;
                if ((lane & 7) == 0) q8d[i >> 3] = m / 127.f;  // raw f32 d (kernels.h QFmt)
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_layernorm_f16(const float * __restrict__ x, int rows, int d,
                                                       const float * __restrict__ w, const float * __restrict__ b,
                                                       float eps, _Float16 * __restrict__ out, int ldo,
                                                       const int * __restrict__ row_idx, float * __restrict__ out32,
                                                       int8_t * __restrict__ q8, float * __restrict__ q8d) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float4 * xr = (const float4 * ) (x + (size_t) (row_idx ? row_idx[row] : row) * d);
    const int n4 = d >> 2;
    // the whole row is loaded once, up front (one memory round trip per launch)
    float4 xv[LN_V4];
#pragma unroll
    for (int j = 0; j < LN_V4; ++j) {
        const int i = lane + 64 * j;
        xv[j] = i < n4 ? xr[i] : float4{0.f, 0.f, 0.f, 0.f};
    }
    ln_row_regs(xv, lane, d, w, b, eps, out + (size_t) row * ldo, out32 ? out32 + (size_t) row * d : nullptr,
                q8 ? q8 + (size_t) row * d : nullptr, q8 ? q8d + (size_t) row * (d / 32) : nullptr);
}

// Finishes an EPI_PARTIAL decode-row GEMM: sums its k splits in order (row-major partial
// rows [ks][M][N], k_gemm.hip), adds bias and the residual (out = resid + (acc + bias),
// whisper.cpp's ggml_add(mul_mat + b, inpL)), writes the new residual row, then LayerNorms it
// for the next matmul. One 256-thread block per row (a decode pass has <= 32 rows, so the
// row's partial loads are spread over 4 waves instead of one); the LayerNorm statistics are
// the same double sums as ln_row_regs (exact for a row of f32 values; the variance sum
// differs from the one-wave order only below double precision).
__global__ __launch_bounds__(256) void k_resid_layernorm(int M, int N, int KS, const float * __restrict__ part,
                                                         const float * __restrict__ bias, float * __restrict__ x,
                                                         const float * __restrict__ w, const float * __restrict__ b,
                                                         float eps, _Float16 * __restrict__ xn, int ldo,
                                                         int8_t * __restrict__ q8, float * __restrict__ q8d) {
    __shared__ double red[4];
    resid_ln_row<false>(blockIdx.x, M, N, KS, part, bias, x, w, b, eps, xn, ldo, q8, q8d, red);
}

void resid_layernorm(hipStream_t s, int M, int N, int ks, const float * part, const float * bias, float * x,
                     const float * lnw, const float * lnb, float eps, _Float16 * xn, int ldo, int8_t * q8, float * q8d) {
    if (M <= 0) return;
    if (M > 32 || N % 16 != 0 || N > 4 * 256 * RL_V4 || ks < 1 || ks > RL_KSMAX)
        throw std::runtime_error("resid_layernorm: unsupported shape");
    if (q8 && (N % 32 != 0 || !q8d)) throw std::runtime_error("resid_layernorm: Q8_0 output needs N % 32 == 0");
    // (one wave per row measured slower twice: round 2 with its split partials loaded one after another,
    // 159 -> 249 ms per step, profiles/archive/r02e_ab.txt; round 6 with every load issued first and no
    // barrier, 5.30 -> 5.39 us per launch alone, F16 RTF 1066 / 1076 -> 1056 / 1060, profiles/r06h_ab.txt)
    OWK_LAUNCH(k_resid_layernorm, dim3(M), dim3(256), 0, s, M, N, ks, part, bias, x, lnw, lnb, eps, xn, ldo,
                       q8, q8d);
}

void layernorm_f16(hipStream_t s, const float * x, int rows, int d, const float * w, const float * b, float eps,
                   _Float16 * out, int ldo, const int * row_idx, float * out32, int8_t * q8, float * q8d) {
    if (rows <= 0) return;
    if (d % 4 != 0 || d > 4 * 64 * LN_V4 || ldo % 4 != 0) throw std::runtime_error("layernorm_f16: unsupported width");
    if (q8 && (d % 32 != 0 || !q8d)) throw std::runtime_error("layernorm_f16: Q8_0 output needs d % 32 == 0");
    OWK_LAUNCH(k_layernorm_f16, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, d, w, b, eps, out, ldo,
                       row_idx, out32, q8, q8d);
}

// two LayerNorms in a row (the SortFormer conformer: a layer's final norm, then the next layer's first):
// y = LN1(x) -> out1 (f16, optional: null when nothing reads it) / out1_32 (f32, the new residual
// stream), then LN2(y) from the same f32 registers -> out2 (f16) / out2_32 -- exactly the two
// layernorm_f16 launches it replaces. out1 and out2 must not overlap (both __restrict__).
__global__ __launch_bounds__(256) void k_layernorm2_f16(const float * __restrict__ x, int rows, int d,
                                                        const float * __restrict__ w1, const float * __restrict__ b1,
                                                        _Float16 * __restrict__ out1, float * __restrict__ out1_32,
                                                        const float * __restrict__ w2, const float * __restrict__ b2,
                                                        _Float16 * __restrict__ out2, float * __restrict__ out2_32,
                                                        float eps) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float4 * xr = (const float4 *) (x + (size_t) row * d);
    const int n4 = d >> 2;
    float4 xv[LN_V4], yv[LN_V4];
#pragma unroll
    for (int j = 0; j < LN_V4; ++j) {
        const int i = lane + 64 * j;
        xv[j] = i < n4 ? xr[i] : float4{0.f, 0.f, 0.f, 0.f};
    }
    ln_row_regs(xv, lane, d, w1, b1, eps, out1 ? out1 + (size_t) row * d : nullptr, out1_32 + (size_t) row * d, nullptr,
                nullptr, &yv);
    ln_row_regs(yv, lane, d, w2, b2, eps, out2 + (size_t) row * d, out2_32 ? out2_32 + (size_t) row * d : nullptr);
}

void layernorm2_f16(hipStream_t s, const float * x, int rows, int d, const float * w1, const float * b1, _Float16 * out1,
                    float * out1_32, const float * w2, const float * b2, _Float16 * out2, float * out2_32, float eps) {
    if (rows <= 0) return;
    if (d % 4 != 0 || d > 4 * 64 * LN_V4 || !out1_32 || !out2) throw std::runtime_error("layernorm2_f16: unsupported");
    if (out1 && out1 < out2 + (size_t) rows * d && out2 < out1 + (size_t) rows * d)
        throw std::runtime_error("layernorm2_f16: out1 and out2 overlap");
    OWK_LAUNCH(k_layernorm2_f16, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, d, w1, b1, out1, out1_32, w2, b2, out2,
               out2_32, eps);
}

// token + position embedding (whisper.cpp:2515-2518: get_rows(d_te) + get_rows(d_pe))
__global__ void k_embed(const _Float16 * __restrict__ te, const float * __restrict__ pe, const int * __restrict__ tok,
                        const int * __restrict__ pos, int rows, int d, float * __restrict__ x) {
    const int r = blockIdx.x;
    if (r >= rows) return;
    const _Float16 * t = te + (size_t) tok[r] * d;
    const float * p = pe + (size_t) pos[r] * d;
    for (int i = threadIdx.x; i < d; i += blockDim.x) x[(size_t) r * d + i] = (float) t[i] + p[i];
}

void embed_tokens(hipStream_t s, const _Float16 * te, const float * pe, const int * tok, const int * pos, int rows,
                  int d, float * x) {
    if (rows <= 0) return;
    OWK_LAUNCH(k_embed, dim3(rows), dim3(256), 0, s, te, pe, tok, pos, rows, d, x);
}

// K-quant models: rows of the host-dequantized f32 embedding (ref get_rows -> dequantize_row_q*_K)
__global__ void k_embed_f32(const float * __restrict__ te, const float * __restrict__ pe, const int * __restrict__ tok,
                            const int * __restrict__ pos, int rows, int d, float * __restrict__ x) {
    const int r = blockIdx.x;
    if (r >= rows) return;
    const float * t = te + (size_t) tok[r] * d;
    const float * p = pe + (size_t) pos[r] * d;
    for (int i = threadIdx.x; i < d; i += blockDim.x) x[(size_t) r * d + i] = t[i] + p[i];
}

void embed_tokens_f32(hipStream_t s, const float * te, const float * pe, const int * tok, const int * pos, int rows,
                      int d, float * x) {
    if (rows <= 0) return;
    OWK_LAUNCH(k_embed_f32, dim3(rows), dim3(256), 0, s, te, pe, tok, pos, rows, d, x);
}

__global__ void k_embed_q5(const uint8_t * __restrict__ qs, const uint32_t * __restrict__ qh,
                           const _Float16 * __restrict__ dd, const float * __restrict__ pe,
                           const int * __restrict__ tok, const int * __restrict__ pos, int rows, int d,
                           float * __restrict__ x) {
    const int r = blockIdx.x;
    if (r >= rows) return;
    const size_t row = (size_t) tok[r];
    const int nb = d / 32;
    const float * p = pe + (size_t) pos[r] * d;
    for (int i = threadIdx.x; i < d; i += blockDim.x) {
        const int b = i >> 5, j = i & 31;
        const uint8_t byte = qs[row * (d / 2) + b * 16 + (j & 15)];
        const int lo = j < 16 ? (byte & 0x0F) : (byte >> 4);
        const int hi = (qh[row * nb + b] >> j) & 1;
        const float v = (float) ((lo | (hi << 4)) - 16) * (float) dd[row * nb + b];  // dequantize_row_q5_0
        x[(size_t) r * d + i] = v + p[i];
    }
}

__global__ void k_embed_q8(const int8_t * __restrict__ qs, const _Float16 * __restrict__ dd,
                           const float * __restrict__ pe, const int * __restrict__ tok, const int * __restrict__ pos,
                           int rows, int d, float * __restrict__ x) {
    const int r = blockIdx.x;
    if (r >= rows) return;
    const size_t row = (size_t) tok[r];
    const int nb = d / 32;
    const float * p = pe + (size_t) pos[r] * d;
    for (int i = threadIdx.x; i < d; i += blockDim.x) {
        const float v = (float) qs[row * d + i] * (float) dd[row * nb + (i >> 5)];  // dequantize_row_q8_0
        x[(size_t) r * d + i] = v + p[i];
    }
}

__global__ void k_embed_q4(const uint8_t * __restrict__ qs, const _Float16 * __restrict__ dd,
                           const float * __restrict__ pe, const int * __restrict__ tok, const int * __restrict__ pos,
                           int rows, int d, float * __restrict__ x) {
    const int r = blockIdx.x;
    if (r >= rows) return;
    const size_t row = (size_t) tok[r];
    const int nb = d / 32;
    const float * p = pe + (size_t) pos[r] * d;
    for (int i = threadIdx.x; i < d; i += blockDim.x) {
        const int b = i >> 5, j = i & 31;
        const uint8_t byte = qs[row * (d / 2) + b * 16 + (j & 15)];
        const int q = j < 16 ? (byte & 0x0F) : (byte >> 4);
        const float v = (float) (q - 8) * (float) dd[row * nb + b];  // dequantize_row_q4_0
        x[(size_t) r * d + i] = v + p[i];
    }
}

// Q4_1 / Q5_1: dequantize_row_q4_1 / _q5_1 (ref ggml/src/ggml-quants.c:327-420): y = q * d + m,
// contracted to one FMA by the reference's gcc build
__global__ void k_embed_q1(const uint8_t * __restrict__ qs, const uint32_t * __restrict__ qh,
                           const _Float16 * __restrict__ dd, const _Float16 * __restrict__ mm,
                           const float * __restrict__ pe, const int * __restrict__ tok, const int * __restrict__ pos,
                           int rows, int d, float * __restrict__ x) {
    const int r = blockIdx.x;
    if (r >= rows) return;
    const size_t row = (size_t) tok[r];
    const int nb = d / 32;
    const float * p = pe + (size_t) pos[r] * d;
    for (int i = threadIdx.x; i < d; i += blockDim.x) {
        const int b = i >> 5, j = i & 31;
        const uint8_t byte = qs[row * (d / 2) + b * 16 + (j & 15)];
        int q = j < 16 ? (byte & 0x0F) : (byte >> 4);
        if (qh) q |= ((qh[row * nb + b] >> j) & 1) << 4;
        const float v = fmaf((float) q, (float) dd[row * nb + b], (float) mm[row * nb + b]);
        x[(size_t) r * d + i] = v + p[i];
    }
}

void embed_tokens_q5(hipStream_t s, const Q5W & te, const float * pe, const int * tok, const int * pos, int rows, int d,
                     float * x) {
    if (rows <= 0) return;
    if (te.fmt == QF_Q4_1 || te.fmt == QF_Q5_1)
        OWK_LAUNCH(k_embed_q1, dim3(rows), dim3(256), 0, s, te.qs, te.fmt == QF_Q5_1 ? te.qh : nullptr, te.d,
                           te.m, pe, tok, pos, rows, d, x);
    else if (te.fmt == QF_Q4_0)
        OWK_LAUNCH(k_embed_q4, dim3(rows), dim3(256), 0, s, te.qs, te.d, pe, tok, pos, rows, d, x);
    else if (te.fmt == QF_Q8_0)
        OWK_LAUNCH(k_embed_q8, dim3(rows), dim3(256), 0, s, (const int8_t *) te.qs, te.d, pe, tok, pos, rows, d, x);
    else
        OWK_LAUNCH(k_embed_q5, dim3(rows), dim3(256), 0, s, te.qs, te.qh, te.d, pe, tok, pos, rows, d, x);
}

// ----------------------------------------------------------------------------------
// Log-mel spectrogram (ref whisper.cpp:3104-3260). Per frame: reflect-padded samples
// times the periodic Hann window (float product, as the reference), 201-bin DFT of
// the 400-sample frame evaluated in double (the reference's float radix-2/DFT FFT is
// a rounding of the exact value; so is this, at double precision), power, mel projection
// summed in double, log10(max(., 1e-10)).
// Frames past n_samples/160 hold only zero padding -> log10(1e-10) = -10 exactly.
// One block per (MEL_FPB frames, clip).
// ----------------------------------------------------------------------------------
constexpr int MEL_FPB = 4;  // frames per block
__global__ __launch_bounds__(256) void k_mel(const MelJob * __restrict__ jobs, const float * __restrict__ filters,
                                             const int * __restrict__ rng, int n_mel, const float * __restrict__ hann,
                                             const double * __restrict__ tw) {
    const MelJob job = jobs[blockIdx.y];
    const int n = job.n_samples;
    const int n_w = n + 200;  // samples after the 200-sample reflect pad
    const int n_compute = min(n_w / 160 + 1, job.n_len);
    float * mel = job.mel;
    __shared__ double frame[400];
    __shared__ double power[201];
    __shared__ double stw[800];  // cos / sin table in LDS (loaded once per MEL_FPB frames)
    __shared__ double ysub[800];  // the 16 x 25 sub-DFT outputs (re, im)
    if (blockIdx.x * MEL_FPB < n_compute)
        for (int j = threadIdx.x; j < 800; j += blockDim.x) stw[j] = tw[j];
    for (int fi = 0; fi < MEL_FPB; ++fi) {
        const int f = blockIdx.x * MEL_FPB + fi;
        if (f >= job.n_len) return;
        if (f >= n_compute) {
            for (int m = threadIdx.x; m < n_mel; m += blockDim.x) mel[(size_t) m * job.n_len + f] = -10.0f;
            continue;
        }
        __syncthreads();  // the previous frame's LDS reads are done
        const int off = f * 160;
        for (int j = threadIdx.x; j < 400; j += blockDim.x) {
            const int p = off + j;  // index into the padded signal
            float v = 0.0f;
            if (p < n_w) {
                v = p < 200 ? job.pcm[200 - p] : job.pcm[p - 200];
            }
            frame[j] = (double) (hann[j] * v);
        }
        __syncthreads();
        // the 400-point DFT as 16 x 25 (Cooley-Tukey, j = 16a + b): Y_b[r] = sum_a x[16a+b] W25^(ar) for
        // the 16 residues b, then X[k] = sum_b W400^(bk) Y_b[k mod 25] -- 33 K double FMAs per frame
        // instead of the direct sum's 160 K, the same exact-value target (twiddles from the 400 table:
        // W25^m = W400^(16m))
        for (int t = threadIdx.x; t < 400; t += blockDim.x) {
            const int b = t / 25, r = t - b * 25;
            double yr = 0.0, yi = 0.0;
            int idx = 0;  // 16 * (a * r mod 25)
            for (int a = 0; a < 25; ++a) {
                const double x = frame[16 * a + b];
                yr += x * stw[idx];
                yi -= x * stw[400 + idx];
                idx += 16 * r;
                if (idx >= 400) idx -= 400;
            }
            ysub[2 * t] = yr;
            ysub[2 * t + 1] = yi;
        }
        __syncthreads();
        for (int k = threadIdx.x; k < 201; k += blockDim.x) {
            const int r = k % 25;
            double re = 0.0, im = 0.0;
            int idx = 0;  // b * k mod 400
            for (int b = 0; b < 16; ++b) {
                const double c = stw[idx], sn = stw[400 + idx];
                const double yr = ysub[2 * (b * 25 + r)], yi = ysub[2 * (b * 25 + r) + 1];
                re += c * yr + sn * yi;
                im += c * yi - sn * yr;
                idx += k;
                if (idx >= 400) idx -= 400;
            }
            power[k] = re * re + im * im;
        }
        __syncthreads();
        for (int m = threadIdx.x; m < n_mel; m += blockDim.x) {
            const float * fr = filters + (size_t) m * 201;
            double sum = 0.0;
            for (int k = rng[2 * m], k1 = rng[2 * m + 1]; k < k1; ++k) sum += power[k] * (double) fr[k];
            mel[(size_t) m * job.n_len + f] = (float) log10(fmax(sum, 1e-10));
        }
    }
}

void mel_spectrogram(hipStream_t s, const MelJob * jobs_dev, int n_jobs, int max_frames, const float * filters,
                     const int * filter_rng, int n_mel, const double * twiddle, const float * hann) {
    if (n_jobs <= 0 || max_frames <= 0) return;
    OWK_LAUNCH(k_mel, dim3((max_frames + MEL_FPB - 1) / MEL_FPB, n_jobs), dim3(256), 0, s, jobs_dev, filters, filter_rng,
               n_mel, hann, twiddle);
}

// global max over the whole (padded) clip, clamp to max-8, (x+4)/4 (whisper.cpp:3228-3244)
__global__ __launch_bounds__(1024) void k_mel_norm(const MelJob * __restrict__ jobs, int n_mel) {
    const MelJob job = jobs[blockIdx.x];
    const size_t total = (size_t) n_mel * job.n_len;
    float m = -1e20f;
    for (size_t i = threadIdx.x; i < total; i += blockDim.x) m = fmaxf(m, job.mel[i]);
    __shared__ float red[1024];
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if ((int) threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    const double mmax = (double) red[0] - 8.0;
    for (size_t i = threadIdx.x; i < total; i += blockDim.x) {
        float v = job.mel[i];
        if ((double) v < mmax) v = (float) mmax;
        job.mel[i] = (float) (((double) v + 4.0) / 4.0);
    }
}

void mel_normalize(hipStream_t s, const MelJob * jobs_dev, int n_jobs, int n_mel) {
    if (n_jobs <= 0) return;
    OWK_LAUNCH(k_mel_norm, dim3(n_jobs), dim3(1024), 0, s, jobs_dev, n_mel);
}

// ----------------------------------------------------------------------------------
// im2col for the two conv1d layers (ggml_conv_1d_ph: im2col to F16 then mul_mat,
// ref ggml.c:4409-4437; whisper.cpp:2006-2014). Column index = c*3 + k, matching the
// weight's [out][in][k] memory order; K is zero-padded to the GEMM's 64 granule.
// ----------------------------------------------------------------------------------
__global__ void k_conv1_im2col(const MelWindow * __restrict__ wins, int n_mel, int n_ctx2, int kpad,
                               _Float16 * __restrict__ A) {
    const int clip = blockIdx.y;
    const MelWindow w = wins[clip];
    const size_t per_clip = (size_t) n_ctx2 * kpad;
    for (size_t e = (size_t) blockIdx.x * blockDim.x + threadIdx.x; e < per_clip; e += (size_t) gridDim.x * blockDim.x) {
        const int t = (int) (e / kpad), col = (int) (e % kpad);
        float v = 0.0f;
        if (col < 3 * n_mel) {
            const int c = col / 3, k = col - 3 * c;
            const int u = t + k - 1;  // position inside the window (padding 1)
            if (u >= 0 && u < n_ctx2) {
                const int src = w.offset + u;
                if (src < w.n_len) v = w.mel[(size_t) c * w.n_len + src];
            }
        }
        A[(size_t) clip * per_clip + e] = (_Float16) v;
    }
}

void conv1_im2col(hipStream_t s, const MelWindow * win_dev, int n_clips, int n_mel, int n_ctx2, int kpad, _Float16 * A) {
    OWK_LAUNCH(k_conv1_im2col, dim3(512, n_clips), dim3(256), 0, s, win_dev, n_mel, n_ctx2, kpad, A);
}

// conv2: stride 2, padding 1, input is the f16 conv1 output [clip][t_in][d]
__global__ void k_conv2_im2col(const _Float16 * __restrict__ x, int t_in, int d, _Float16 * __restrict__ A) {
    const int clip = blockIdx.y;
    const int t_out = t_in / 2;
    const int K = 3 * d;
    const size_t per_clip = (size_t) t_out * K;
    const _Float16 * xc = x + (size_t) clip * t_in * d;
    for (size_t e = (size_t) blockIdx.x * blockDim.x + threadIdx.x; e < per_clip; e += (size_t) gridDim.x * blockDim.x) {
        const int t = (int) (e / K), col = (int) (e % K);
        const int c = col / 3, k = col - 3 * c;
        const int u = 2 * t + k - 1;
        _Float16 v = (_Float16) 0.0f;
        if (u >= 0 && u < t_in) v = xc[(size_t) u * d + c];
        A[(size_t) clip * per_clip + e] = v;
    }
}

void conv2_im2col(hipStream_t s, const _Float16 * x, int n_clips, int t_in, int d, _Float16 * A) {
    OWK_LAUNCH(k_conv2_im2col, dim3(1024, n_clips), dim3(256), 0, s, x, t_in, d, A);
}

} // namespace owk
