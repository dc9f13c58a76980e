// Silero VAD (v6.2, 16 kHz) on gfx950: the reference's per-chunk ggml graph
// (ref/src/whisper.cpp:4519-4653), restructured for the GPU.
//
// The reference evaluates one 512-sample chunk per graph call: STFT conv, 4 conv1d
// layers, LSTM cell, 1x1 conv head. Only the LSTM carries state between chunks, so the
// work splits into
//   vad_encode_kernel  all chunks of all streams in parallel: reflect pad, STFT conv
//                      (F16 im2col), magnitude, 4 x (conv1d + bias + ReLU), and the LSTM
//                      input projection W_ih x + b_ih           (ref 4519-4565, 4574-4575)
//   vad_lstm_kernel    one workgroup per stream walks its chunks in order: W_hh h + b_hh,
//                      gates, cell/hidden update; W_hh lives in registers (row per thread)
//                                                              (ref 4567-4610)
//   vad_head_kernel    every chunk in parallel: ReLU, F16 1x1 conv, bias, sigmoid
//                                                              (ref 4640-4645)
// Numerics: every ggml_conv_1d rounds its input to F16 (im2col dst type F16) and dots it
// with F16 weights in f32; the LSTM matmuls are f32; sigmoid = 1/(1+exp(-x)).
#include "common.h"
#include "kernels.h"

namespace owk {

namespace {

constexpr int VAD_WIN = 512;   // n_window (model header)
constexpr int VAD_PAD = 64;    // reflect padding of the STFT input (ref 4522)
constexpr int VAD_XP = VAD_WIN + 2 * VAD_PAD;
constexpr int VAD_NB = 258;    // STFT basis rows (129 real + 129 imaginary)
constexpr int VAD_NF = 129;
constexpr int VAD_T0 = 4;      // STFT frames per chunk: (640 - 256) / 128 + 1
constexpr int VAD_H = 128;     // LSTM hidden size
constexpr int VAD_G = 4 * VAD_H;
constexpr int VAD_CH = 4;      // chunks per encode workgroup (weights read once per 4 chunks)
constexpr int VAD_THREADS = 256;

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float r16(float x) { return (float) (_Float16) x; }

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// Workgroup barrier that orders LDS only. __syncthreads() also drains the wave's global
// loads/stores (vmcnt) at every step; the LSTM recurrence shares nothing but LDS, so its
// prefetches and history stores stay in flight across the barrier.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// conv1d over VAD_CH chunks: in [ch][IC][Lin] (already F16-rounded), wT [(ic*K + k)][OC] f16,
// out [ch][OC][Lout] = relu(conv + bias); thread per output channel, im2col (ic, k) order.
template <int IC, int OC, int K, int LIN, int LOUT, int S, int P>
__device__ __forceinline__ void conv_relu(const float * in, const _Float16 * __restrict__ wT,
                                          const float * __restrict__ bias, float * out, bool round_out) {
    for (int oc = threadIdx.x; oc < OC; oc += VAD_THREADS) {
        float acc[VAD_CH][LOUT];
#pragma unroll
        for (int c = 0; c < VAD_CH; ++c)
#pragma unroll
            for (int t = 0; t < LOUT; ++t) acc[c][t] = 0.0f;
        for (int ic = 0; ic < IC; ++ic) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float w = (float) wT[(ic * K + k) * OC + oc];
#pragma unroll
                for (int t = 0; t < LOUT; ++t) {
                    const int pos = t * S + k - P;
                    if (pos < 0 || pos >= LIN) continue;
#pragma unroll
                    for (int c = 0; c < VAD_CH; ++c) acc[c][t] = __builtin_fmaf(w, in[(c * IC + ic) * LIN + pos], acc[c][t]);
                }
            }
        }
        const float b = bias[oc];
#pragma unroll
        for (int c = 0; c < VAD_CH; ++c)
#pragma unroll
            for (int t = 0; t < LOUT; ++t) {
                const float v = fmaxf(acc[c][t] + b, 0.0f);
                out[(c * OC + oc) * LOUT + t] = round_out ? r16(v) : v;
            }
    }
}

__global__ void __launch_bounds__(VAD_THREADS) vad_encode_kernel(
        const float * __restrict__ pcm, const int64_t * __restrict__ pcm_off, const int * __restrict__ pcm_len,
        const int * __restrict__ chunk_stream, const int * __restrict__ chunk_index, int n_chunks,
        const VadWeights w, float * __restrict__ ig) {
    __shared__ float xp[VAD_CH][VAD_XP];
    __shared__ float st[VAD_CH][VAD_NB][VAD_T0];
    __shared__ float mag[VAD_CH][VAD_NF][VAD_T0];
    __shared__ float c0[VAD_CH][128][4];
    __shared__ float c1[VAD_CH][64][2];
    __shared__ float c2[VAD_CH][64][1];
    __shared__ float c3[VAD_CH][128];
    const int tid = threadIdx.x;
    const int g0 = blockIdx.x * VAD_CH;

    // 1. window (zero past the stream's end, ref 5127-5144), reflect pad 64/64 (ops.cpp
    //    pad_reflect_1d), F16 rounding of the STFT im2col
    for (int i = tid; i < VAD_CH * VAD_XP; i += VAD_THREADS) {
        const int c = i / VAD_XP, j = i % VAD_XP;
        const int g = g0 + c;
        float v = 0.0f;
        if (g < n_chunks) {
            int src = j - VAD_PAD;
            if (src < 0) src = -src;
            if (src >= VAD_WIN) src = 2 * (VAD_WIN - 1) - src;
            const int s = chunk_stream[g];
            const int at = chunk_index[g] * VAD_WIN + src;
            if (at < pcm_len[s]) v = pcm[pcm_off[s] + at];
        }
        xp[c][j] = r16(v);
    }
    __syncthreads();

    // 2. STFT conv: 258 basis rows x 4 frames, kernel 256, stride 128 (ref 4524)
    for (int oc = tid; oc < VAD_NB; oc += VAD_THREADS) {
        float acc[VAD_CH][VAD_T0];
#pragma unroll
        for (int c = 0; c < VAD_CH; ++c)
#pragma unroll
            for (int t = 0; t < VAD_T0; ++t) acc[c][t] = 0.0f;
        for (int k = 0; k < 256; ++k) {
            const float b = (float) w.stft_T[k * VAD_NB + oc];
#pragma unroll
            for (int c = 0; c < VAD_CH; ++c)
#pragma unroll
                for (int t = 0; t < VAD_T0; ++t) acc[c][t] = __builtin_fmaf(b, xp[c][t * 128 + k], acc[c][t]);
        }
#pragma unroll
        for (int c = 0; c < VAD_CH; ++c)
#pragma unroll
            for (int t = 0; t < VAD_T0; ++t) st[c][oc][t] = acc[c][t];
    }
    __syncthreads();
    // magnitude sqrt(re^2 + im^2) (ref 4533-4537), rounded for the next im2col
    for (int i = tid; i < VAD_CH * VAD_NF * VAD_T0; i += VAD_THREADS) {
        const int c = i / (VAD_NF * VAD_T0), r = (i / VAD_T0) % VAD_NF, t = i % VAD_T0;
        const float re = st[c][r][t], im = st[c][VAD_NF + r][t];
        const float re2 = re * re, im2 = im * im;
        mag[c][r][t] = r16(__fsqrt_rn(re2 + im2));
    }
    __syncthreads();

    // 3. encoder (ref 4542-4565): k3 convs, strides 1/2/2/1, padding 1
    conv_relu<VAD_NF, 128, 3, 4, 4, 1, 1>(&mag[0][0][0], w.enc_T[0], w.enc_b[0], &c0[0][0][0], true);
    __syncthreads();
    conv_relu<128, 64, 3, 4, 2, 2, 1>(&c0[0][0][0], w.enc_T[1], w.enc_b[1], &c1[0][0][0], true);
    __syncthreads();
    conv_relu<64, 64, 3, 2, 1, 2, 1>(&c1[0][0][0], w.enc_T[2], w.enc_b[2], &c2[0][0][0], true);
    __syncthreads();
    conv_relu<64, 128, 3, 1, 1, 1, 1>(&c2[0][0][0], w.enc_T[3], w.enc_b[3], &c3[0][0], false);
    __syncthreads();

    // 4. LSTM input projection of cur[:, :, 0] (ref 4630, 4574-4575): f32 x f32
    for (int r = tid; r < VAD_G; r += VAD_THREADS) {
        float acc[VAD_CH];
#pragma unroll
        for (int c = 0; c < VAD_CH; ++c) acc[c] = 0.0f;
        for (int j = 0; j < VAD_H; ++j) {
            const float wv = w.ih_T[j * VAD_G + r];
#pragma unroll
            for (int c = 0; c < VAD_CH; ++c) acc[c] = __builtin_fmaf(wv, c3[c][j], acc[c]);
        }
        const float b = w.b_ih[r];
#pragma unroll
        for (int c = 0; c < VAD_CH; ++c)
            if (g0 + c < n_chunks) ig[(size_t) (g0 + c) * VAD_G + r] = acc[c] + b;
    }
}

// One workgroup per stream; thread r owns gate row r. hs/gs in LDS, two barriers per chunk.
__global__ void __launch_bounds__(VAD_G) vad_lstm_kernel(
        const float * __restrict__ ig, const int * __restrict__ stream_first, const int * __restrict__ stream_n,
        const float * __restrict__ w_hh, const float * __restrict__ b_hh, float * __restrict__ state,
        float * __restrict__ hist) {
    __shared__ float hs[VAD_H];
    __shared__ float gs[VAD_G];
    const int s = blockIdx.x;
    const int r = threadIdx.x;
    const int first = stream_first[s], n = stream_n[s];
    float * hst = state + (size_t) s * 2 * VAD_H;  // [h][c] of this stream

    float wr[VAD_H];
#pragma unroll
    for (int j = 0; j < VAD_H; j += 4) {
        const float4 v = *(const float4 *) (w_hh + (size_t) r * VAD_H + j);
        wr[j] = v.x; wr[j + 1] = v.y; wr[j + 2] = v.z; wr[j + 3] = v.w;
    }
    const float bh = b_hh[r];
    float c = 0.0f;
    if (r < VAD_H) {
        hs[r] = hst[r];
        c = hst[VAD_H + r];
    }
    __syncthreads();
    // ig rows prefetched one block of VAD_PF steps ahead: the only global-memory wait of
    // the recurrence is at block boundaries
    constexpr int VAD_PF = 8;
    float buf[VAD_PF];
#pragma unroll
    for (int k = 0; k < VAD_PF; ++k) buf[k] = k < n ? ig[(size_t) (first + k) * VAD_G + r] : 0.0f;
    for (int tb = 0; tb < n; tb += VAD_PF) {
        float nxt[VAD_PF];
#pragma unroll
        for (int k = 0; k < VAD_PF; ++k) {
            const int tt = tb + VAD_PF + k;
            nxt[k] = tt < n ? ig[(size_t) (first + tt) * VAD_G + r] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < VAD_PF; ++k) {
            const int t = tb + k;
            if (t >= n) break;
            // packed FMAs (v_pk_fma_f32): two of the four partial sums per instruction
            f32x2 a01 = {0.0f, 0.0f}, a23 = {0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < VAD_H; j += 4) {
                const float4 h4 = *(const float4 *) &hs[j];
                a01 = __builtin_elementwise_fma(f32x2{wr[j], wr[j + 1]}, f32x2{h4.x, h4.y}, a01);
                a23 = __builtin_elementwise_fma(f32x2{wr[j + 2], wr[j + 3]}, f32x2{h4.z, h4.w}, a23);
            }
            const float hid = ((a01.x + a01.y) + (a23.x + a23.y)) + bh;
            const float pre = buf[k] + hid;  // inp_gate + hid_gate (ref 4582)
            gs[r] = (r >= 2 * VAD_H && r < 3 * VAD_H) ? tanhf(pre) : sigm(pre);
            lds_barrier();
            if (r < VAD_H) {
                const float fc = gs[VAD_H + r] * c;
                const float ig_ = gs[r] * gs[2 * VAD_H + r];
                c = fc + ig_;
                const float h = gs[3 * VAD_H + r] * tanhf(c);
                hs[r] = h;
                hist[(size_t) (first + t) * VAD_H + r] = h;
            }
            lds_barrier();
        }
#pragma unroll
        for (int k = 0; k < VAD_PF; ++k) buf[k] = nxt[k];
    }
    if (r < VAD_H) {
        hst[r] = hs[r];
        hst[VAD_H + r] = c;
    }
}

// one wave per chunk: sigmoid(f16(w_f) . f16(relu(h)) + b_f)
__global__ void __launch_bounds__(256) vad_head_kernel(const float * __restrict__ hist, int n_chunks,
                                                       const _Float16 * __restrict__ wf, const float * __restrict__ bf,
                                                       float * __restrict__ probs) {
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (g >= n_chunks) return;
    const float * h = hist + (size_t) g * VAD_H;
    float v = (float) wf[lane] * r16(fmaxf(h[lane], 0.0f));
    v = __builtin_fmaf((float) wf[lane + 64], r16(fmaxf(h[lane + 64], 0.0f)), v);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) probs[g] = sigm(v + bf[0]);
}

} // namespace

void launch_vad(const VadWeights & w, const float * pcm, const int64_t * pcm_off, const int * pcm_len,
                const int * chunk_stream, const int * chunk_index, int n_chunks, const int * stream_first,
                const int * stream_n, int n_streams, float * ig, float * hist, float * state, float * probs,
                hipStream_t stream) {
    if (n_chunks <= 0) return;
    vad_encode_kernel<<<(n_chunks + VAD_CH - 1) / VAD_CH, VAD_THREADS, 0, stream>>>(
        pcm, pcm_off, pcm_len, chunk_stream, chunk_index, n_chunks, w, ig);
    vad_lstm_kernel<<<n_streams, VAD_G, 0, stream>>>(ig, stream_first, stream_n, w.w_hh, w.b_hh, state, hist);
    vad_head_kernel<<<(n_chunks + 3) / 4, 256, 0, stream>>>(hist, n_chunks, w.wf, w.bf, probs);
    OWK_HIP_CHECK(hipGetLastError());
}

} // namespace owk
