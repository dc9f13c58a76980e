// Attention kernels, gfx950.
//
// Encoder: flash attention on MFMA (f16 operands, f32 online softmax) reproducing the
// reference's tiled CPU path (ggml-cpu/ops.cpp:8275-8546, taken for the encoder since
// n_q >= 32 and n_kv = 1536 is a multiple of 16): F32 accumulators, and the 36 all-zero
// padded keys of kv_pad (GGML_PAD(1500,256) rows never written, whisper.cpp:2055,
// 2142-2159) folded in analytically at the end (score 0, value 0).
//
// Decoder: one wave per (query row, head) emulating the reference's per-key visit
// order. In decode steps and short prefills the reference takes the "one_chunk" path
// (ops.cpp:8140-8233) whose V accumulator is F16 and is rounded after every key;
// that rounding is reproduced exactly (scores via f32 dot of f16 Q/K, expf, fma,
// f32->f16 RNE per key). Long prefills (n_q >= 32) use the tiled F32 path.
#include "kernels.h"

#include <algorithm>

namespace owk {

typedef __attribute__((address_space(3))) void * lds_ptr_t;

// soft_max probability -> f16 after its f32 rounding (ggml_soft_max writes f32, mul_mat converts
// that to f16): the empty asm keeps hipcc from folding the multiply into v_fma_mixlo_f16, one
// rounding of the exact product, which differs on f16 ties (as f16_rn in k_gemm.hip)
__device__ __forceinline__ _Float16 p_f16(float p) {
    asm volatile("" : "+v"(p));
    return (_Float16) p;
}

// ----------------------------------------------------------------------------------
// Encoder flash attention.
// Block = 4 waves = 64 queries of one (clip, head); KV tiles of 64 keys staged in LDS:
//   K tile  [64 keys][64 dims] (row-major, from the [clip*T+t][d] K buffer)
//   Vt tile [64 dims][64 keys] (from the transposed V written by the QKV epilogue)
// S^T = K . Q^T is computed so each lane owns 16 scores of ONE query (lane&15): the
// softmax needs only 2 cross-lane shuffles and P^T feeds the P.V MFMA as the B operand
// straight from registers (key order inside a k-step permuted consistently on both
// operands).
// ----------------------------------------------------------------------------------
constexpr int FA_KT = 64;                     // keys per tile
constexpr int FA_TILE_BYTES = FA_KT * 64 * 2; // 8 KB (K tile or Vt tile)

// XCD-aware block order of the encoder attention (1-D grid): the 8 XCDs, each with a private L2, take
// blocks round-robin by linear id, so a (clip, head)'s query tiles laid out consecutively landed on 8
// XCDs and each XCD fetched that pair's K / V tiles again (FETCH_SIZE 5.8x the Q/K/V bytes). Here the
// s-th block of XCD x (linear id 8 s + x) takes (clip, head) pair x + 8 (s / nt), query tile s % nt: all
// tiles of a pair on one XCD. The grid is padded to whole groups of 8 pairs; padding blocks exit.
__device__ __forceinline__ bool enc_attn_block(int nt, int H, int n_clips, int & qt, int & h, int & clip) {
    const int L = blockIdx.x, x = L & 7, sl = L >> 3;
    const int p = x + 8 * (sl / nt);
    if (p >= H * n_clips) return false;
    qt = sl % nt;
    h = p % H;
    clip = p / H;
    return true;
}
inline dim3 enc_attn_grid(int nt, int H, int n_clips) { return dim3(8 * nt * ((H * n_clips + 7) / 8)); }

__global__ __launch_bounds__(256, 2) void k_attn_encoder(const _Float16 * __restrict__ q, const _Float16 * __restrict__ k,
                                                         const _Float16 * __restrict__ vt, int T, int Tpad, int H,
                                                         float scale, int n_zero_pad, _Float16 * __restrict__ out,
                                                         float * __restrict__ out32, int n_clips) {
    __shared__ __attribute__((aligned(1024))) char smem[4 * FA_TILE_BYTES];  // 2 stages x (K, Vt)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int qt, h, clip;
    if (!enc_attn_block((T + 63) / 64, H, n_clips, qt, h, clip)) return;
    const int d = H * 64;
    const int g = lane >> 4, l16 = lane & 15;

    // Q fragments (B operand of S^T = K.Q^T): q = l16, dims 32*s + 8*g .. +8
    const int qi = qt * 64 + wave * 16 + l16;
    const int qc = min(qi, T - 1);
    const _Float16 * qrow = q + ((size_t) clip * T + qc) * d + h * 64;
    const half8 qf0 = *(const half8 *) (qrow + 8 * g);
    const half8 qf1 = *(const half8 *) (qrow + 32 + 8 * g);

    const _Float16 * kbase = k + (size_t) clip * T * d + h * 64;
    const _Float16 * vbase = vt + ((size_t) clip * H + h) * 64 * Tpad;

    auto stage = [&](int buf, int kt) {
        char * sK = smem + buf * 2 * FA_TILE_BYTES;
        char * sV = sK + FA_TILE_BYTES;
        // 8 KB each = 8 groups of 8 rows x 128 B; 2 groups per wave per tensor
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int grp = wave * 2 + i;
            const int row = grp * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((row >> 1) & 7);
            const int key = min(kt * FA_KT + row, T - 1);
            __builtin_amdgcn_global_load_lds((const void *) (kbase + (size_t) key * d + c * 8),
                                             (lds_ptr_t) (sK + grp * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *) (vbase + (size_t) row * Tpad + kt * FA_KT + c * 8),
                                             (lds_ptr_t) (sV + grp * 1024), 16, 0, 0);
        }
    };

    floatx4 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    // the online softmax runs in base 2: scores scaled by scale * log2(e), exponentials by the
    // native v_exp_f32 (2 instructions where the accurate expf took ~10: this loop is VALU-bound
    // beside its 16 MFMAs per tile). Mathematically the same softmax; the roundings move by ~1e-6
    // relative against the reference's f32 tiled path (parity bars: tests/test_gpu_parity.py)
    const float scale2 = scale * 1.44269504088896341f;
    float m = -INFINITY;  // running max (base-2 units) of this lane's query (uniform over its 4 lanes)
    float lsum = 0.0f;    // partial row sum over this lane's keys

    const int ntiles = (T + FA_KT - 1) / FA_KT;
    stage(0, 0);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < ntiles) stage(cur ^ 1, kt + 1);
        const char * sK = smem + cur * 2 * FA_TILE_BYTES;
        const char * sV = sK + FA_TILE_BYTES;

        // S^T tiles: keys 16*t + 4*g + e, query l16
        floatx4 sc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int row = t * 16 + l16;
            const half8 a0 = *(const half8 *) (sK + row * 128 + (((0 + g) ^ ((row >> 1) & 7)) << 4));
            const half8 a1 = *(const half8 *) (sK + row * 128 + (((4 + g) ^ ((row >> 1) & 7)) << 4));
            floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
            z = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, qf0, z, 0, 0, 0);
            z = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, qf1, z, 0, 0, 0);
            sc[t] = z;
        }
        float tmax = -INFINITY;
        if ((kt + 1) * FA_KT <= T) {  // a full tile (every one but the last): no key mask
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = sc[t][e] * scale2;
                    sc[t][e] = v;
                    tmax = fmaxf(tmax, v);
                }
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int key = kt * FA_KT + t * 16 + 4 * g + e;
                    float v = sc[t][e] * scale2;
                    if (key >= T) v = -INFINITY;
                    sc[t][e] = v;
                    tmax = fmaxf(tmax, v);
                }
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mnew = fmaxf(m, tmax);
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);  // m = -inf on the first tile -> 0
        const bool moved = __builtin_amdgcn_ballot_w64(mnew != m) != 0;  // wave-uniform
        m = mnew;
        float ps = 0.0f;
        half8 pb[2];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float p = __builtin_amdgcn_exp2f(sc[t][e] - mnew);
                ps += p;
                pb[t >> 1][(t & 1) * 4 + e] = (_Float16) p;
            }
        lsum = lsum * alpha + ps;
        // the accumulator rescale only when some query's max moved (alpha = 1 everywhere otherwise: o * 1
        // is o, bit for bit)
        if (moved)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] *= alpha;

        // O^T[dim][q] += V^T[dim][key] . P^T[key][q]; k-step ks covers keys 32*ks..+32 with
        // element j<4 -> key 32ks + 4g + j, j>=4 -> key 32ks + 16 + 4g + (j-4)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const int row = dt * 16 + l16;  // dim
            const char * vr = sV + row * 128;
            const int sw = (row >> 1) & 7;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int b0 = ks * 64 + 8 * g;        // byte offset of key 32ks + 4g
                const int b1 = ks * 64 + 32 + 8 * g;   // byte offset of key 32ks + 16 + 4g
                const half4 lo = *(const half4 *) (vr + ((((b0 >> 4) ^ sw) << 4) | (b0 & 15)));
                const half4 hi = *(const half4 *) (vr + ((((b1 >> 4) ^ sw) << 4) | (b1 & 15)));
                half8 a;
                a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
                a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, pb[ks], o[dt], 0, 0, 0);
            }
        }
        __syncthreads();
    }

    // total row sum over the 4 lanes of each query, then the zero-padded keys
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    if (n_zero_pad > 0) {
        const float mnew = fmaxf(m, 0.0f);
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        lsum = lsum * alpha + (float) n_zero_pad * __builtin_amdgcn_exp2f(0.0f - mnew);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] *= alpha;
    }
    if (qi < T) {
        const float inv = lsum == 0.0f ? 0.0f : 1.0f / lsum;
        const size_t ro = ((size_t) clip * T + qi) * d + h * 64;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            if (out32) {  // f32 output (Q5_0 models quantize it to Q8_0 themselves)
                float4 r;
                r.x = o[dt][0] * inv; r.y = o[dt][1] * inv; r.z = o[dt][2] * inv; r.w = o[dt][3] * inv;
                *(float4 *) (out32 + ro + dt * 16 + 4 * g) = r;
                continue;
            }
            half4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) r[e] = (_Float16) (o[dt][e] * inv);
            *(half4 *) (out + ro + dt * 16 + 4 * g) = r;
        }
    }
}

// ----------------------------------------------------------------------------------
// Encoder attention WITHOUT flash attention (context flash_attn = false; the mode the
// reference needs for DTW timestamps, whisper.cpp:2163-2189): KQ = K.Q over exactly T keys
// (no zero padding), soft_max_ext(KQ * scale) with the exact row max first and a
// double-accumulated sum (ggml_compute_forward_soft_max_f32, ops.cpp:5160-5272), then the
// probabilities are ROUNDED TO F16 (mul_mat(V, KQ_soft_max) converts its f32 operand) and
// multiplied with V. Same block/lane mapping as k_attn_encoder; three sweeps over the keys
// (max, sum, output).
// ----------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void k_attn_encoder_sm(const _Float16 * __restrict__ q,
                                                            const _Float16 * __restrict__ k,
                                                            const _Float16 * __restrict__ vt, int T, int Tpad, int H,
                                                            float scale, _Float16 * __restrict__ out,
                                                            float * __restrict__ out32, int n_clips) {
    __shared__ __attribute__((aligned(1024))) char smem[4 * FA_TILE_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int qt, h, clip;
    if (!enc_attn_block((T + 63) / 64, H, n_clips, qt, h, clip)) return;
    const int d = H * 64;
    const int g = lane >> 4, l16 = lane & 15;
    const int qi = qt * 64 + wave * 16 + l16;
    const int qc = min(qi, T - 1);
    const _Float16 * qrow = q + ((size_t) clip * T + qc) * d + h * 64;
    const half8 qf0 = *(const half8 *) (qrow + 8 * g);
    const half8 qf1 = *(const half8 *) (qrow + 32 + 8 * g);
    const _Float16 * kbase = k + (size_t) clip * T * d + h * 64;
    const _Float16 * vbase = vt + ((size_t) clip * H + h) * 64 * Tpad;

    auto stage = [&](int buf, int kt, bool with_v) {
        char * sK = smem + buf * 2 * FA_TILE_BYTES;
        char * sV = sK + FA_TILE_BYTES;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int grp = wave * 2 + i;
            const int row = grp * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((row >> 1) & 7);
            const int key = min(kt * FA_KT + row, T - 1);
            __builtin_amdgcn_global_load_lds((const void *) (kbase + (size_t) key * d + c * 8),
                                             (lds_ptr_t) (sK + grp * 1024), 16, 0, 0);
            if (with_v)
                __builtin_amdgcn_global_load_lds((const void *) (vbase + (size_t) row * Tpad + kt * FA_KT + c * 8),
                                                 (lds_ptr_t) (sV + grp * 1024), 16, 0, 0);
        }
    };
    // scores of one K tile: sc[t][e] = s(key 16t + 4g + e, query l16) * scale, -inf past T
    auto scores = [&](const char * sK, int kt, floatx4 (&sc)[4]) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int row = t * 16 + l16;
            const half8 a0 = *(const half8 *) (sK + row * 128 + (((0 + g) ^ ((row >> 1) & 7)) << 4));
            const half8 a1 = *(const half8 *) (sK + row * 128 + (((4 + g) ^ ((row >> 1) & 7)) << 4));
            floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
            z = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, qf0, z, 0, 0, 0);
            z = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, qf1, z, 0, 0, 0);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int key = kt * FA_KT + t * 16 + 4 * g + e;
                z[e] = key < T ? z[e] * scale : -INFINITY;
            }
            sc[t] = z;
        }
    };
    const int ntiles = (T + FA_KT - 1) / FA_KT;

    // sweep 1: exact row max
    float m = -INFINITY;
    stage(0, 0, false);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < ntiles) stage(cur ^ 1, kt + 1, false);
        floatx4 sc[4];
        scores(smem + cur * 2 * FA_TILE_BYTES, kt, sc);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) m = fmaxf(m, sc[t][e]);
        __syncthreads();
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));

    // sweep 2: sum of exp(s - max), accumulated in double
    double l = 0.0;
    stage(0, 0, false);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < ntiles) stage(cur ^ 1, kt + 1, false);
        floatx4 sc[4];
        scores(smem + cur * 2 * FA_TILE_BYTES, kt, sc);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) l += (double) expf(sc[t][e] - m);
        __syncthreads();
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = (float) (1.0 / l);

    // sweep 3: P = f16(exp(s - max) * inv), O = P . V
    floatx4 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    stage(0, 0, true);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < ntiles) stage(cur ^ 1, kt + 1, true);
        const char * sK = smem + cur * 2 * FA_TILE_BYTES;
        const char * sV = sK + FA_TILE_BYTES;
        floatx4 sc[4];
        scores(sK, kt, sc);
        half8 pb[2];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) pb[t >> 1][(t & 1) * 4 + e] = p_f16(expf(sc[t][e] - m) * inv);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const int row = dt * 16 + l16;
            const char * vr = sV + row * 128;
            const int sw = (row >> 1) & 7;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int b0 = ks * 64 + 8 * g;
                const int b1 = ks * 64 + 32 + 8 * g;
                const half4 lo = *(const half4 *) (vr + ((((b0 >> 4) ^ sw) << 4) | (b0 & 15)));
                const half4 hi = *(const half4 *) (vr + ((((b1 >> 4) ^ sw) << 4) | (b1 & 15)));
                half8 a;
                a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
                a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, pb[ks], o[dt], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    if (qi < T) {
        const size_t ro = ((size_t) clip * T + qi) * d + h * 64;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            if (out32) {
                *(float4 *) (out32 + ro + dt * 16 + 4 * g) = make_float4(o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
                continue;
            }
            half4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) r[e] = (_Float16) o[dt][e];
            *(half4 *) (out + ro + dt * 16 + 4 * g) = r;
        }
    }
}

void attn_encoder_softmax(hipStream_t s, const _Float16 * q, const _Float16 * k, const _Float16 * vt, int n_clips, int T,
                          int Tpad, int H, float scale, _Float16 * out, float * out32) {
    if (Tpad < ((T + FA_KT - 1) / FA_KT) * FA_KT) throw std::runtime_error("attn_encoder_softmax: Tpad too small");
    OWK_LAUNCH(k_attn_encoder_sm, enc_attn_grid((T + 63) / 64, H, n_clips), dim3(256), 0, s, q, k, vt, T, Tpad, H,
               scale, out, out32, n_clips);
}

void attn_encoder(hipStream_t s, const _Float16 * q, const _Float16 * k, const _Float16 * vt, int n_clips, int T,
                  int Tpad, int H, float scale, int n_zero_pad, _Float16 * out, float * out32) {
    if (Tpad < ((T + FA_KT - 1) / FA_KT) * FA_KT) throw std::runtime_error("attn_encoder: Tpad too small");
    OWK_LAUNCH(k_attn_encoder, enc_attn_grid((T + 63) / 64, H, n_clips), dim3(256), 0, s, q, k, vt, T, Tpad, H,
               scale, n_zero_pad, out, out32, n_clips);
}

// ----------------------------------------------------------------------------------
// Decode-step attention, reference-order emulation of the one_chunk path
// (ops.cpp:8140-8233), one wave per (query row, head):
//   for each key in visit order:
//     if s > M { M = s; ms = exp(Mold-M); acc = f16(acc*ms); vs = 1 } else { vs = exp(s-M) }
//     acc = f16(fma(v, vs, acc));  S = S*ms + vs
// Only the acc/S recurrences are sequential. Per chunk of 64 keys:
//   1. K and V tiles stream HBM -> LDS with global_load_lds, AS_NBUF chunks in flight
//      (the HBM-bound part: K + V of the row's clip, 2 x 128 B per key and head);
//   2. lane = key: s = (q . k) * scale; an inclusive max-scan over the wave gives each
//      key's running max before it (Mex), hence its (ms, vs) pair in parallel;
//   3. lane = head dim: the exact per-key recurrence, with ms/vs broadcast by readlane
//      and the rescale branch taken only on the (wave-uniform) new-maximum keys.
// ----------------------------------------------------------------------------------
constexpr int AS_KC = 64;       // keys per chunk
constexpr int AS_NBUF = 3;      // chunks in flight
constexpr int AS_TILE = AS_KC * 128;
constexpr int AS_RLB = 16;      // keys per readlane batch in the recurrence

// inclusive max-scan over the 64 lanes (DPP: row_shr 1/2/4/8, then row_bcast 15/31)
#define OWK_DPP_MAX(v, ctrl, rmask, bmask)                                                                       \
    fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, -INFINITY),           \
                                                                   __builtin_bit_cast(int, v), ctrl, rmask, bmask, \
                                                                   false)))
__device__ __forceinline__ float wave_incl_max(float v) {
    v = OWK_DPP_MAX(v, 0x111, 0xf, 0xf);  // row_shr:1
    v = OWK_DPP_MAX(v, 0x112, 0xf, 0xf);  // row_shr:2
    v = OWK_DPP_MAX(v, 0x114, 0xf, 0xf);  // row_shr:4
    v = OWK_DPP_MAX(v, 0x118, 0xf, 0xf);  // row_shr:8
    v = OWK_DPP_MAX(v, 0x142, 0xa, 0xf);  // row_bcast:15 -> rows 1, 3
    v = OWK_DPP_MAX(v, 0x143, 0xc, 0xf);  // row_bcast:31 -> rows 2, 3
    return v;
}
// lane i <- lane i-1 of v; lane 0 <- fill (DPP wave_shr:1)
__device__ __forceinline__ float wave_shr1(float v, float fill) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, fill), __builtin_bit_cast(int, v),
                                                                 0x138, 0xf, 0xf, false));
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int AS_MAX_LIST = 2048;  // listed keys (self-attention cells) per row

// CROSS: the head-major cross K/V (non-temporal loads; also names the instantiation so cross
// and self attention are apart in profiles).
// NW = 2 (cross attention): a loader wave and a math wave per (row, head). Under the full decode step's
// HBM load a wave's LDS-DMA issue stalls while the memory pipeline is backed up, and with one wave those
// stalls stopped its math too (SQ_WAIT_INST_ANY 27 % of the wave's cycles at 32 rows x 20 heads x 1500
// keys, profiles/r05n_attn_cross_ab.txt); the loader wave takes the stalls, the math wave runs on.
// Hand-off per chunk by two workgroup barriers: B1 (loader: chunk c landed, vmcnt) and B2 (math wave:
// chunk c is in its registers, so the loader may refill that buffer with chunk c + AS_NBUF).
template <bool LIST, bool CROSS, int NW = 1>
__global__ __launch_bounds__(64 * NW) void k_attn_step(const _Float16 * __restrict__ q, int ldq,
                                                  const _Float16 * __restrict__ kb, const _Float16 * __restrict__ vb,
                                                  int ld_kv, int hs, const AttnRow * __restrict__ rows,
                                                  const int * __restrict__ key_idx, float scale,
                                                  _Float16 * __restrict__ out, int ldo, float * __restrict__ out32,
                                                  int8_t * __restrict__ q8, float * __restrict__ q8d) {
    // NOTE: any ordinary LDS store in this kernel (s_list below) makes the compiler drain
    // every in-flight global_load_lds (s_waitcnt vmcnt(0)) before the ring reads of each
    // chunk; the host therefore launches LIST = true only for passes with a listed row
    __shared__ __attribute__((aligned(1024))) char smem[AS_NBUF * 2 * AS_TILE];
    __shared__ int s_list[LIST ? AS_MAX_LIST : 1];
    static_assert(NW == 1 || (NW == 2 && !LIST), "the two-wave form streams contiguous keys only");
    const int lane = threadIdx.x & 63;
    const bool loader = NW == 2 && threadIdx.x < 64;  // wave 0 of a two-wave block
    const AttnRow job = rows[blockIdx.y];
    if (job.mode != 0) return;  // tiled (F32) rows: k_attn_decoder
    const int h = blockIdx.x;
    const int n = job.n_keys;
    // the output (f32 or f16) and, for a Q5_0 consumer, its Q8_0 rounding (two 32-lane blocks;
    // x86 quantize_row_q8_0 as k_quantize_q8)
    auto emit = [&](float y) {
        const size_t o = (size_t) job.q_row * ldo + h * 64 + lane;
        if (out32) out32[o] = y;
        else out[o] = (_Float16) y;
        if (q8) {
            float m = fabsf(y);
#pragma unroll
            for (int sh = 16; sh > 0; sh >>= 1) m = fmaxf(m, __shfl_xor(m, sh, 32));
            const float id = m != 0.0f ? 127.f / m : 0.0f;
            q8[o] = (int8_t) rintf(y * id);
            if ((lane & 31) == 0) q8d[o >> 5] = m / 127.f;  // raw f32 d (kernels.h QFmt)
        }
    };
    if (n <= 0) {
        if (!loader) emit(0.0f);
        return;
    }
    // a listed row whose cells are not one contiguous run (the host passes contiguous runs
    // as key_list = -1 with kv_base at the first cell)
    const bool listed = LIST && job.key_list >= 0;
    if (listed) {
        // cell indices to LDS up front: the stage loop then issues no global loads whose
        // results it must wait for (a vmcnt wait would also drain the in-flight K/V tiles)
        const int * list = key_idx + job.key_list;
        for (int i = lane; i < n; i += 64) s_list[i] = list[i];
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
    }
    const _Float16 * kh = kb + job.kv_base + (size_t) h * hs;
    const _Float16 * vh = vb + job.kv_base + (size_t) h * hs;

    // q of this (row, head): uniform -> scalar registers
    const half8 * qp = (const half8 *) (q + (size_t) job.q_row * ldq + h * 64);
    half8 qv[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) qv[c] = qp[c];

    const int nchunks = (n + AS_KC - 1) / AS_KC;
    // LDS images of a chunk, 8 keys x 128 B per KB: K rows with their 16-B segments XOR-swizzled
    // (segment s of key row kk at s ^ (kk & 7): conflict-free lane-per-key ds_read_b128 rows), V rows
    // plain. The load of row kk = 8i + (lane >> 3) by lane: the XOR term depends on the lane only.
    const int kseg = (lane & 7) ^ (lane >> 3);
    const int vseg = lane & 7;
    // contiguous keys (no cell list): buffer loads off one per-lane offset and a scalar chunk offset (no
    // per-load 64-bit address math); the resource's range ends at the last key's row, so the rows past n of
    // a partial last chunk read as nothing from memory (they are never used)
    const int row_b = ld_kv * 2;
    const uint32_t range = (uint32_t) (((size_t) (n - 1) * ld_kv + 64) * 2);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void *) kh, (short) 0, range, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void *) vh, (short) 0, range, 0x00020000);
    const int ko = (lane >> 3) * row_b + kseg * 16, vo = (lane >> 3) * row_b + vseg * 16;
    // stage chunk c into buffer b: 8 + 8 loads of 1 KB (8 keys x 128 B each)
    auto stage = [&](int b, int c) {
        char * sK = smem + b * 2 * AS_TILE;
        char * sV = sK + AS_TILE;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            // cross K/V are read once per decode step (larger than the MALL): non-temporal
            if (listed) {
                const int kk = i * 8 + (lane >> 3);
                const int cell = s_list[min(c * AS_KC + kk, n - 1)];
                __builtin_amdgcn_global_load_lds((const void *) (kh + (size_t) cell * ld_kv + kseg * 8),
                                                 (lds_ptr_t) (sK + i * 1024), 16, 0, CROSS ? 2 : 0);
                __builtin_amdgcn_global_load_lds((const void *) (vh + (size_t) cell * ld_kv + vseg * 8),
                                                 (lds_ptr_t) (sV + i * 1024), 16, 0, CROSS ? 2 : 0);
            } else {
                const int so = (c * AS_KC + i * 8) * row_b;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_ptr_t) (sK + i * 1024), 16, ko, so, 0, CROSS ? 2 : 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_ptr_t) (sV + i * 1024), 16, vo, so, 0, CROSS ? 2 : 0);
            }
        }
    };

    // chunk c has landed once at most the chunks staged after it are outstanding
    auto wait_chunk = [&](int c) {
        const int ahead = min(AS_NBUF - 1, nchunks - 1 - c);
        static_assert(AS_NBUF == 3, "vmcnt ladder below assumes 3 buffers");
        if (ahead == 2) wait_vmcnt<32>();
        else if (ahead == 1) wait_vmcnt<16>();
        else wait_vmcnt<0>();
    };
    if (NW == 1 || loader) {
#pragma unroll
        for (int c = 0; c < AS_NBUF; ++c)
            if (c < nchunks) stage(c, c);
    }
    if (loader) {
        for (int c = 0; c < nchunks; ++c) {
            wait_chunk(c);
            __builtin_amdgcn_s_barrier();  // B1
            __builtin_amdgcn_s_barrier();  // B2
            if (c + AS_NBUF < nchunks) stage(c % AS_NBUF, c + AS_NBUF);
        }
        return;
    }

    float M = -INFINITY, S = 0.0f;
    _Float16 acc = (_Float16) 0.0f;  // the reference's F16 VKQ accumulator (VKQ16)
    for (int c = 0; c < nchunks; ++c) {
        if (NW == 1) wait_chunk(c);
        else __builtin_amdgcn_s_barrier();  // B1
        const char * sK = smem + (c % AS_NBUF) * 2 * AS_TILE;
        const char * sV = sK + AS_TILE;
        const int base = c * AS_KC;
        const int nk = min(AS_KC, n - base);

        // the chunk's K row (lane = key) and V column (lane = head dim) go to registers first and the
        // buffer is refilled (chunk c + AS_NBUF) before any math: AS_NBUF chunks stay in flight across
        // the scores and the sequential part (rows nk.. of a partial chunk are read but not used)
        half8 krow[8];
        {
            const char * kr = sK + lane * 128;
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) krow[cc] = *(const half8 *) (kr + ((cc ^ (lane & 7)) << 4));
        }
        const _Float16 * vcol = (const _Float16 *) sV + lane;
        const bool full = nk == AS_KC;
        _Float16 vv[AS_KC];
#pragma unroll
        for (int kk = 0; kk < AS_KC; ++kk) vv[kk] = vcol[kk * 64];
        if (NW == 2) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // K and V reads of this buffer done
            __builtin_amdgcn_s_barrier();                       // B2
        } else if (c + AS_NBUF < nchunks) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // K and V reads of this buffer done
            stage(c % AS_NBUF, c + AS_NBUF);
        }

        // 2. scores, lane = key: f32 dot2 of f16 pairs, 8 independent partial sums
        float s;
        {
            float part[8];
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) {
                const half8 kv = krow[cc];
                float a = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    const half2v k2 = {kv[e], kv[e + 1]}, q2 = {qv[cc][e], qv[cc][e + 1]};
                    a = __builtin_amdgcn_fdot2(k2, q2, a, false);
                }
                part[cc] = a;
            }
            const float a = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
            s = lane < nk ? a * scale : -INFINITY;
        }
        // running max before each key: DPP inclusive max-scan, then a one-lane wave shift
        const float pm = wave_incl_max(s);
        const float mex = fmaxf(wave_shr1(pm, M), M);
        const bool nm = lane < nk && s > mex;
        const float e = expf(nm ? mex - s : s - mex);
        const float ms = nm ? e : 1.0f;
        const float vs = nm ? 1.0f : e;
        M = fmaxf(M, __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pm), 63)));

        // 3. recurrence, lane = head dim
        if (full && __builtin_amdgcn_ballot_w64(nm) == 0) {
            // no new maximum in the chunk (the common case once the first keys are seen):
            // every ms is 1, so acc*ms and S*ms are exact and each key costs one mixed FMA on
            // acc and one add on S (vs broadcast by readlane, 16 keys' worth into scalar registers
            // at a time so the readlane -> VALU hazard wait is paid once per batch, not per key)
#pragma unroll
            for (int kb = 0; kb < AS_KC; kb += AS_RLB) {
                float vsb[AS_RLB];
#pragma unroll
                for (int j = 0; j < AS_RLB; ++j)
                    vsb[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vs), kb + j));
#pragma unroll
                for (int j = 0; j < AS_RLB; ++j) {
                    acc = (_Float16) fmaf((float) vv[kb + j], vsb[j], (float) acc);
                    S = S + vsb[j];
                }
            }
        } else if (full) {
            // acc*ms with ms == 1 is exact, so the rescale is applied unconditionally (branch-free)
            // and each key costs two dependent mixed-precision FMAs (f32 math, f16 result)
#pragma unroll
            for (int kb = 0; kb < AS_KC; kb += AS_RLB / 2) {
                float msb[AS_RLB / 2], vsb[AS_RLB / 2];
#pragma unroll
                for (int j = 0; j < AS_RLB / 2; ++j) {
                    msb[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ms), kb + j));
                    vsb[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vs), kb + j));
                }
#pragma unroll
                for (int j = 0; j < AS_RLB / 2; ++j) {
                    acc = (_Float16) ((float) acc * msb[j]);
                    acc = (_Float16) fmaf((float) vv[kb + j], vsb[j], (float) acc);
                    S = fmaf(S, msb[j], vsb[j]);
                }
            }
        } else {  // the last, partial chunk (nothing staged after it); keys nk.. are skipped
#pragma unroll
            for (int kb = 0; kb < AS_KC; kb += AS_RLB / 2) {
                if (kb >= nk) break;
                float msb[AS_RLB / 2], vsb[AS_RLB / 2];
#pragma unroll
                for (int j = 0; j < AS_RLB / 2; ++j) {
                    msb[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ms), kb + j));
                    vsb[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vs), kb + j));
                }
#pragma unroll
                for (int j = 0; j < AS_RLB / 2; ++j) {
                    if (kb + j < nk) {
                        acc = (_Float16) ((float) acc * msb[j]);
                        acc = (_Float16) fmaf((float) vv[kb + j], vsb[j], (float) acc);
                        S = fmaf(S, msb[j], vsb[j]);
                    }
                }
            }
        }
    }
    for (int j = 0; j < job.n_zero_pad; ++j) {  // all-zero keys: s = 0, v = 0 (acc + 0*vs == acc)
        if (0.0f > M) {
            const float ms = expf(M - 0.0f);
            M = 0.0f;
            acc = (_Float16) ((float) acc * ms);
            S = fmaf(S, ms, 1.0f);
        } else {
            S = fmaf(S, 1.0f, expf(0.0f - M));
        }
    }
    const float S_inv = S == 0.0f ? 0.0f : 1.0f / S;
    emit((float) acc * S_inv);
}

// ----------------------------------------------------------------------------------
// Decoder attention for rows on the tiled path (prefills of >= 32 tokens: F32
// accumulator over tiles of 16 keys, ops.cpp:8417-8510). Block = 4 waves = 4 heads.
// ----------------------------------------------------------------------------------
constexpr int DA_MAX_KEYS = 2048;

__global__ __launch_bounds__(256) void k_attn_decoder(const _Float16 * __restrict__ q, int ldq,
                                                      const _Float16 * __restrict__ kb, const _Float16 * __restrict__ vb,
                                                      int ld_kv, int hs, const AttnRow * __restrict__ rows,
                                                      const int * __restrict__ key_idx, int H, float scale,
                                                      _Float16 * __restrict__ out, int ldo, float * __restrict__ out32) {
    __shared__ float sc[4][DA_MAX_KEYS];
    __shared__ _Float16 qs[4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const AttnRow job = rows[blockIdx.y];
    if (job.mode != 1) return;  // one_chunk rows: k_attn_step; soft_max rows: k_attn_softmax
    const int h = blockIdx.x * 4 + wave;
    if (h >= H) return;
    const int n = job.n_keys;
    const int * list = job.key_list >= 0 ? key_idx + job.key_list : nullptr;
    const _Float16 * kh = kb + job.kv_base + (size_t) h * hs;
    const _Float16 * vh = vb + job.kv_base + (size_t) h * hs;

    qs[wave][lane] = q[(size_t) job.q_row * ldq + h * 64 + lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    // phase 1: scores
    for (int i = lane; i < n; i += 64) {
        const int cell = list ? list[i] : i;
        const half8 * kr = (const half8 *) (kh + (size_t) cell * ld_kv);
        float acc = 0.0f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const half8 kv = kr[c];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc = fmaf((float) kv[e], (float) qs[wave][c * 8 + e], acc);
        }
        sc[wave][i] = acc * scale;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

    float result;
    if (job.mode == 0) {
        float M = -INFINITY, S = 0.0f, acc = 0.0f;  // acc always holds an f16-representable value
        int i = 0;
        // prefetch V for the first key
        for (; i < n; ++i) {
            const int cell = list ? list[i] : i;
            const float v = (float) vh[(size_t) cell * ld_kv + lane];
            const float s = sc[wave][i];
            float ms = 1.0f, vs = 1.0f;
            if (s > M) {
                const float Mold = M;
                M = s;
                ms = expf(Mold - M);
                acc = (float) (_Float16) (acc * ms);
            } else {
                vs = expf(s - M);
            }
            acc = (float) (_Float16) fmaf(v, vs, acc);
            S = fmaf(S, ms, vs);
        }
        for (int j = 0; j < job.n_zero_pad; ++j) {  // all-zero keys: s = 0, v = 0
            float ms = 1.0f, vs = 1.0f;
            if (0.0f > M) {
                const float Mold = M;
                M = 0.0f;
                ms = expf(Mold - M);
                acc = (float) (_Float16) (acc * ms);
            } else {
                vs = expf(0.0f - M);
            }
            S = fmaf(S, ms, vs);
        }
        const float S_inv = S == 0.0f ? 0.0f : 1.0f / S;
        result = acc * S_inv;
    } else {
        float M = -INFINITY, S = 0.0f, acc = 0.0f;
        const int total = n + job.n_zero_pad;
        for (int t0 = 0; t0 < total; t0 += 16) {
            const int t1 = min(t0 + 16, total);
            float tmax = -INFINITY;
            for (int i = t0; i < t1; ++i) tmax = fmaxf(tmax, i < n ? sc[wave][i] : 0.0f);
            if (tmax == -INFINITY) continue;
            const float Mnew = fmaxf(M, tmax);
            if (Mnew > M) {
                const float ms = expf(M - Mnew);
                acc *= ms;
                S *= ms;
            }
            M = Mnew;
            float ts = 0.0f;
            for (int i = t0; i < t1; ++i) {
                const float s = i < n ? sc[wave][i] : 0.0f;
                const float p = expf(s - Mnew);
                ts += p;
                if (i < n) {
                    const int cell = list ? list[i] : i;
                    acc = fmaf((float) vh[(size_t) cell * ld_kv + lane], p, acc);
                }
            }
            S += ts;
        }
        const float S_inv = S == 0.0f ? 0.0f : 1.0f / S;
        result = acc * S_inv;
    }
    if (out32) out32[(size_t) job.q_row * ldo + h * 64 + lane] = result;
    else out[(size_t) job.q_row * ldo + h * 64 + lane] = (_Float16) result;
}

// ----------------------------------------------------------------------------------
// Decoder attention WITHOUT flash attention (flash_attn = false contexts; rows with
// mode 2): KQ over the listed keys (self: visible cells; cross: exactly n_audio_ctx),
// soft_max with the exact max and a double sum, probabilities rounded to F16 for the
// P.V product (whisper.cpp:2616-2628 self, 2697-2738 cross). Optionally the f32
// probabilities of alignment heads are captured for DTW timestamps (whisper.cpp:2720-2736):
// cap[a][key][cap_row] for alignment head a = amap[h] >= 0.
// Block = 4 waves per (row, head).
// ----------------------------------------------------------------------------------
constexpr int SM_MAX_KEYS = 2048;

// NT threads per block: 256, or 1024 when the pass has few (row, head) blocks (one row per step:
// 20 blocks on 256 CUs) so each block keeps 4x the loads in flight. Every sum is taken in an order
// that does not depend on NT (a row's output must not depend on how many rows share its pass):
// the double softmax sum over 256 fixed key residues (mod 256) by the first 256 threads, and P.V
// over SM_PV_GROUPS fixed key residues (mod 128), each summed in key order, then the groups in
// group order.
constexpr int SM_PV_GROUPS = 128;
template <int NT>
__global__ __launch_bounds__(NT) void k_attn_softmax(const _Float16 * __restrict__ q, int ldq,
                                                      const _Float16 * __restrict__ kb, const _Float16 * __restrict__ vb,
                                                      int ld_kv, int hs, const AttnRow * __restrict__ rows,
                                                      const int * __restrict__ key_idx, float scale,
                                                      _Float16 * __restrict__ out, int ldo,
                                                      const int * __restrict__ amap, float * __restrict__ cap,
                                                      int cap_rows, float * __restrict__ out32) {
    constexpr int NW = NT / 64;
    constexpr int TG = NT / 8;                    // thread groups of 8 (one 128-byte V row each)
    constexpr int GPT = SM_PV_GROUPS / TG;        // key residues per thread group: 4 (NT 256) or 1 (NT 1024)
    constexpr int U = 8 / GPT;                    // keys of each residue per iteration (8 loads in flight)
    static_assert(GPT * TG == SM_PV_GROUPS && U * GPT == 8, "P.V group layout");
    __shared__ float sp[SM_MAX_KEYS > SM_PV_GROUPS * 64 ? SM_MAX_KEYS : SM_PV_GROUPS * 64];
    __shared__ _Float16 p16[SM_MAX_KEYS];
    __shared__ float redf[NW];
    __shared__ double redd[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const AttnRow job = rows[blockIdx.y];
    if (job.mode != 2) return;
    const int h = blockIdx.x;
    const int n = job.n_keys;
    const int * list = job.key_list >= 0 ? key_idx + job.key_list : nullptr;
    const _Float16 * kh = kb + job.kv_base + (size_t) h * hs;
    const _Float16 * vh = vb + job.kv_base + (size_t) h * hs;
    const _Float16 * qr = q + (size_t) job.q_row * ldq + h * 64;
    // P . V thread groups (below): tg (8 threads, head dims 8 seg .. +8) owns the key residues
    // g = tg + TG j (mod SM_PV_GROUPS). The V rows of the first P . V iteration do not depend on the
    // scores: their loads go out now, with the K rows, so the row pays one HBM round trip, not two
    const int tg = tid >> 3, seg = tid & 7;
    half8 vv0[GPT][U];
    half8 k0[8];
    {
        // every cell index first (one round trip when the row has a cell list), then this thread's
        // first K row and every V row: a list load between them made hipcc wait for all earlier
        // loads before each one, and a K load issued behind the V rows waited for them
        int kcell = max(0, min(tid, n - 1));
        int cell[GPT][U];
#pragma unroll
        for (int j = 0; j < GPT; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) cell[j][u] = max(0, min(tg + TG * j + SM_PV_GROUPS * u, n - 1));
        if (list) {
            kcell = list[kcell];
#pragma unroll
            for (int j = 0; j < GPT; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) cell[j][u] = list[cell[j][u]];
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) k0[c] = ((const half8 *) (kh + (size_t) kcell * ld_kv))[c];
#pragma unroll
        for (int j = 0; j < GPT; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) vv0[j][u] = *(const half8 *) (vh + (size_t) cell[j][u] * ld_kv + seg * 8);
    }

    // scores (lane = key; the first key's K row is already loaded, later iterations unrolled so
    // several keys' loads are in flight)
    float mx = -INFINITY;
    if (tid < n) {
        float part[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const half8 qv = ((const half8 *) qr)[c];
            float a = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) a = fmaf((float) k0[c][e], (float) qv[e], a);
            part[c] = a;
        }
        const float s = (((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]))) * scale;
        sp[tid] = s;
        mx = s;
    }
#pragma unroll 3
    for (int i = tid + NT; i < n; i += NT) {
        const int cell = list ? list[i] : i;
        const half8 * kr = (const half8 *) (kh + (size_t) cell * ld_kv);
        float part[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const half8 kv = kr[c];
            const half8 qv = ((const half8 *) qr)[c];
            float a = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) a = fmaf((float) kv[e], (float) qv[e], a);
            part[c] = a;
        }
        const float s = (((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]))) * scale;
        sp[i] = s;
        mx = fmaxf(mx, s);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    mx = redf[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) mx = fmaxf(mx, redf[w]);
    // exp (every thread), then the double-accumulated sum by threads 0..255 over keys = tid mod 256
    for (int i = tid; i < n; i += NT) sp[i] = expf(sp[i] - mx);
    __syncthreads();
    if (tid < 256) {
        double sum = 0.0;
        for (int i = tid; i < n; i += 256) sum += (double) sp[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
        if (lane == 0) redd[wave] = sum;
    }
    __syncthreads();
    const double sum = (redd[0] + redd[1]) + (redd[2] + redd[3]);
    const float inv = (float) (1.0 / sum);
    const int a = amap ? amap[h] : -1;
    for (int i = tid; i < n; i += NT) {
        const float p = sp[i] * inv;
        p16[i] = p_f16(p);
        if (a >= 0) cap[((size_t) a * n + i) * cap_rows + job.q_row] = p;
    }
    __syncthreads();
    // P . V: thread group tg (8 threads, head dims 8 seg .. +8: one 16-byte load per key) owns the
    // key residues g = tg + TG j (mod SM_PV_GROUPS), each accumulated in key order
    float acc[GPT][8];
#pragma unroll
    for (int j = 0; j < GPT; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[j][e] = 0.0f;
    for (int i0 = 0; i0 < n; i0 += SM_PV_GROUPS * U) {
        half8 vv[GPT][U];
        float pp[GPT][U];
        if (i0 == 0) {
#pragma unroll
            for (int j = 0; j < GPT; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) vv[j][u] = vv0[j][u];
        } else {  // cell indices first, then the V rows (as the first iteration's prefetch)
            int cell[GPT][U];
#pragma unroll
            for (int j = 0; j < GPT; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) cell[j][u] = min(i0 + tg + TG * j + SM_PV_GROUPS * u, n - 1);
            if (list) {
#pragma unroll
                for (int j = 0; j < GPT; ++j)
#pragma unroll
                    for (int u = 0; u < U; ++u) cell[j][u] = list[cell[j][u]];
            }
#pragma unroll
            for (int j = 0; j < GPT; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) vv[j][u] = *(const half8 *) (vh + (size_t) cell[j][u] * ld_kv + seg * 8);
        }
#pragma unroll
        for (int j = 0; j < GPT; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int ii = i0 + tg + TG * j + SM_PV_GROUPS * u;
                pp[j][u] = ii < n ? (float) p16[min(ii, n - 1)] : 0.0f;
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < GPT; ++j)
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[j][e] = fmaf(pp[j][u], (float) vv[j][u][e], acc[j][e]);
    }
    float * red = sp;  // the scores are consumed: reuse as [SM_PV_GROUPS][64] partials
    __syncthreads();
#pragma unroll
    for (int j = 0; j < GPT; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[(tg + TG * j) * 64 + seg * 8 + e] = acc[j][e];
    __syncthreads();
    if (wave == 0) {
        float r = 0.0f;
        for (int g = 0; g < SM_PV_GROUPS; ++g) r += red[g * 64 + lane];
        if (out32) out32[(size_t) job.q_row * ldo + h * 64 + lane] = r;
        else out[(size_t) job.q_row * ldo + h * 64 + lane] = (_Float16) r;
    }
}

// The same soft_max attention with every (row, head) spread over several blocks, bit-identical to
// k_attn_softmax (probabilities, DTW captures and outputs):
//   (A) k_sm_split_scores: a block per 128 consecutive keys computes their scores and the chunk maximum;
//   (B) k_sm_split_pv: SMS_GB blocks per (row, head), block b owning the P.V key residues (mod 128)
//       g = 16 b .. 16 b + 15 -- k_attn_softmax's P.V groups. Every block recomputes the row's exact max
//       and double sum from the stored scores with k_attn_softmax's per-thread residues (mod 256) and
//       wave trees, forms the probabilities of its keys, and runs each group's fma chain over its keys
//       in key order; the (row, head)'s last-arriving block adds the 128 group partials in group order
//       (an arrival ticket per (row, head) in the workspace, zero between launches: the workspace is
//       zeroed when allocated and the last arriver resets its ticket).
// One (row, head) in one block reads 384 KB of K / V through one CU (configs[4]'s one-row steps: 20
// blocks on 256 CUs, ~25 us per cross pass); spread over 12 + 8 blocks per head it streams at the chip's
// rate. Workspace per (row, head): scores [SM_MAX_KEYS] f32, chunk maxima [SMS_MAXC], group partials
// [128][64], ticket (attn_softmax_ws_floats).
constexpr int SMS_CK = 128;
constexpr int SMS_MAXC = SM_MAX_KEYS / SMS_CK;
constexpr int SMS_GB = 8;                              // P.V blocks per (row, head)
constexpr int SMS_GPB = SM_PV_GROUPS / SMS_GB;         // residue groups per P.V block (16)
constexpr int SMS_UMAX = SM_MAX_KEYS / SM_PV_GROUPS;   // keys per residue group (16)
constexpr int SMS_PART = SM_MAX_KEYS + SMS_MAXC;       // group partials [SM_PV_GROUPS][64]
constexpr int SMS_TICKET = SMS_PART + SM_PV_GROUPS * 64;  // the (row, head)'s arrival ticket (int)
constexpr int SMS_PER_RH = SMS_TICKET + 16;
static_assert(SMS_GPB * 8 == 128 && SMS_GPB * SMS_UMAX == 256, "P.V block thread layout");
static_assert(SMS_MAXC <= 64, "one chunk maximum per lane");

__global__ __launch_bounds__(SMS_CK) void k_sm_split_scores(const _Float16 * __restrict__ q, int ldq,
                                                            const _Float16 * __restrict__ kb, int ld_kv, int hs,
                                                            const AttnRow * __restrict__ rows,
                                                            const int * __restrict__ key_idx, float scale, int H,
                                                            float * __restrict__ ws) {
    __shared__ float redf[SMS_CK / 64];
    const AttnRow job = rows[blockIdx.y];
    if (job.mode != 2) return;
    const int h = blockIdx.x % H, c = blockIdx.x / H;
    const int n = job.n_keys;
    if (c * SMS_CK >= n) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float * w = ws + ((size_t) blockIdx.y * H + h) * SMS_PER_RH;
    const int * list = job.key_list >= 0 ? key_idx + job.key_list : nullptr;
    const _Float16 * kh = kb + job.kv_base + (size_t) h * hs;
    const _Float16 * qr = q + (size_t) job.q_row * ldq + h * 64;
    const int i = c * SMS_CK + tid;
    float s = -INFINITY;
    if (i < n) {
        const int cell = list ? list[i] : i;
        const half8 * kr = (const half8 *) (kh + (size_t) cell * ld_kv);
        float part[8];
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
            const half8 kv = kr[cc];
            const half8 qv = ((const half8 *) qr)[cc];
            float a = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) a = fmaf((float) kv[e], (float) qv[e], a);
            part[cc] = a;
        }
        s = (((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]))) * scale;
        w[i] = s;
    }
    float mx = s;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    if (tid == 0) w[SM_MAX_KEYS + c] = fmaxf(redf[0], redf[1]);
}

__global__ __launch_bounds__(256) void k_sm_split_pv(const _Float16 * __restrict__ vb, int ld_kv, int hs,
                                                     const AttnRow * __restrict__ rows, const int * __restrict__ key_idx,
                                                     int H, const int * __restrict__ amap, float * __restrict__ cap,
                                                     int cap_rows, float * ws, _Float16 * __restrict__ out, int ldo,
                                                     float * __restrict__ out32) {
    __shared__ _Float16 p16[SMS_GPB][SMS_UMAX];
    __shared__ double redd[4];
    __shared__ int s_last;
    const AttnRow job = rows[blockIdx.y];
    if (job.mode != 2) return;
    const int h = blockIdx.x % H, b = blockIdx.x / H;
    const int n = job.n_keys;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float * w = ws + ((size_t) blockIdx.y * H + h) * SMS_PER_RH;
    const int nc = (n + SMS_CK - 1) / SMS_CK;  // score chunks = keys per residue group, rounded up
    const int * list = job.key_list >= 0 ? key_idx + job.key_list : nullptr;
    const _Float16 * vh = vb + job.kv_base + (size_t) h * hs;
    // P.V thread (tid < 128): residue group g of this block, head dims 8 seg .. +8, keys g + 128 u. Its V
    // rows go out first (they do not depend on the softmax): the HBM round trip overlaps the sum below
    const int gl = (tid >> 3) & (SMS_GPB - 1), seg = tid & 7, g = b * SMS_GPB + gl;
    // cell indices first, then every V row with no branch between the loads: a list load or a guard
    // between them made hipcc wait for every earlier load before each one (12 serial round trips at
    // 1500 keys). Rows past the last chunk repeat the last key and threads 128.. repeat 0..127's rows
    // (cache hits, never used).
    half8 vv[SMS_UMAX];
    {
        int cell[SMS_UMAX];
#pragma unroll
        for (int u = 0; u < SMS_UMAX; ++u) cell[u] = max(0, min(g + SM_PV_GROUPS * u, n - 1));
        if (list) {
#pragma unroll
            for (int u = 0; u < SMS_UMAX; ++u) cell[u] = list[cell[u]];
        }
#pragma unroll
        for (int u = 0; u < SMS_UMAX; ++u) vv[u] = *(const half8 *) (vh + (size_t) cell[u] * ld_kv + seg * 8);
    }
    // this thread's stored scores, all loads in flight at once: the sum's keys tid + 256 j and the key
    // whose probability it forms below
    constexpr int SJ = SM_MAX_KEYS / 256;
    float sv[SJ];
#pragma unroll
    for (int j = 0; j < SJ; ++j) sv[j] = tid + 256 * j < n ? w[tid + 256 * j] : 0.0f;
    const int ip = b * SMS_GPB + (tid & (SMS_GPB - 1)) + SM_PV_GROUPS * (tid >> 4);
    const float wp = ip < n ? w[ip] : 0.0f;
    // the row maximum over the chunk maxima: one load per lane, then the (exact, order-free) max tree
    float mx = lane < nc ? w[SM_MAX_KEYS + lane] : -INFINITY;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    // k_attn_softmax's sum: thread t < 256 over keys t + 256 j in j order, each exp as its (float) sp,
    // then the trees
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < SJ; ++j)
        if (tid + 256 * j < n) sum += (double) expf(sv[j] - mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) redd[wave] = sum;
    __syncthreads();
    const float inv = (float) (1.0 / ((redd[0] + redd[1]) + (redd[2] + redd[3])));
    {  // the probabilities of this block's keys: thread (group tid & 15, key tid >> 4 of the group)
        const int a = amap ? amap[h] : -1;
        const int i = ip;
        float p = 0.0f;
        if (i < n) {
            p = expf(wp - mx) * inv;
            if (a >= 0) cap[((size_t) a * n + i) * cap_rows + job.q_row] = p;
        }
        p16[tid & (SMS_GPB - 1)][tid >> 4] = p_f16(p);
    }
    __syncthreads();
    float * part = w + SMS_PART;
    if (tid < 128) {
        // k_attn_softmax's chain for group g: fma over its keys in key order (keys past n: p = 0, exact)
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
#pragma unroll
        for (int u = 0; u < SMS_UMAX; ++u) {
            if (u < nc) {
                const float pp = g + SM_PV_GROUPS * u < n ? (float) p16[gl][u] : 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] = fmaf(pp, (float) vv[u][e], acc[e]);
            }
        }
        // hand-off inside the launch (cdna_hip_programming.md Guideline 16, R1): partials stored
        // write-through (agent-scope atomic stores: sc1, past the XCD's non-coherent L2) and drained
        // (vmcnt(0): every store acknowledged at the coherence point) before the barrier that precedes
        // the arrival ticket; the last arriver reads them with agent-scope atomic loads. Only the
        // hand-off's own locations are involved, all accessed as agent-scope atomics, so no cache-wide
        // release / acquire is needed: the formal fences (buffer_wbl2 of the whole L2 before the ticket,
        // buffer_inv after it) measured +3.9 us per launch at one row x 448 keys and +2 us at 1500
        // (13.78 / 14.34 us against 9.88 / 12.3, profiles/r06h_ab.txt), 20-30 % of configs[4]'s step
#pragma unroll
        for (int e = 0; e < 8; ++e)
            __hip_atomic_store(part + g * 64 + seg * 8 + e, acc[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    int * ticket = (int *) (w + SMS_TICKET);
    if (tid == 0) s_last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == SMS_GB - 1;
    __syncthreads();
    if (!s_last || tid >= 64) return;
    // the last arriver: the 128 group partials in group order (agent-scope, L1-bypassing loads), as
    // k_attn_softmax's wave 0 adds them; then the ticket is reset for the next launch
    // two batches of 64 loads in flight (the vmcnt limit), then the adds: two memory round trips (all
    // four waves loading once and adding through LDS measured 0.5 us slower, profiles/r06v_smpv_reduce_ab.txt)
    float r = 0.0f;
#pragma unroll
    for (int g0 = 0; g0 < SM_PV_GROUPS; g0 += 64) {
        float v[64];
#pragma unroll
        for (int j = 0; j < 64; ++j) v[j] = __hip_atomic_load(part + (g0 + j) * 64 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int j = 0; j < 64; ++j) r += v[j];
    }
    if (out32) out32[(size_t) job.q_row * ldo + h * 64 + tid] = r;
    else out[(size_t) job.q_row * ldo + h * 64 + tid] = (_Float16) r;
    if (tid == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

size_t attn_softmax_ws_floats(int n_rows, int H) { return (size_t) n_rows * H * SMS_PER_RH; }
int attn_softmax_force_nt = 0;

void attn_decoder_softmax(hipStream_t s, const _Float16 * q, int ldq, const _Float16 * kbase, const _Float16 * vbase,
                          int ld_kv, int hs, const AttnRow * rows_dev, int n_rows, const int * key_idx, int H, float scale,
                          int max_keys, _Float16 * out, int ldo, const int * amap, float * cap, int cap_rows,
                          float * out32, float * ws, size_t ws_floats) {
    if (n_rows <= 0) return;
    if (max_keys > SM_MAX_KEYS) throw std::runtime_error("attn_decoder_softmax: too many keys");
    // key-split form (bit-identical to the single-block kernel below) for passes of few (row, head)
    // blocks, where one block per head leaves the chip idle: 12.3 vs 17.3 us at 1 row x 1500 keys;
    // at 32 rows its per-block recomputation of the row's softmax costs more (102 vs 45 us;
    // tests/test_gpu_kernels.py::test_softmax_attention_split_bit_identical)
    if (ws && n_rows * H <= 128) {
        if (ws_floats < attn_softmax_ws_floats(n_rows, H)) throw std::runtime_error("attn_decoder_softmax: workspace");
        const int nc = (max_keys + SMS_CK - 1) / SMS_CK;
        OWK_LAUNCH(k_sm_split_scores, dim3(H * nc, n_rows), dim3(SMS_CK), 0, s, q, ldq, kbase, ld_kv, hs, rows_dev,
                   key_idx, scale, H, ws);
        OWK_LAUNCH(k_sm_split_pv, dim3(H * SMS_GB, n_rows), dim3(256), 0, s, vbase, ld_kv, hs, rows_dev, key_idx, H,
                   amap, cap, cap_rows, ws, out, ldo, out32);
        return;
    }
    // outputs do not depend on the width (k_attn_softmax): 1024 threads when the pass has few (row, head)
    // blocks AND long rows, 256 otherwise -- measured (test_softmax_attention_split_bit_identical, r05q): one
    // row of <= 200 keys (configs[4]'s self attention) 5.0-5.5 us at 256 threads vs 5.9-6.4 at 1024; 32 rows
    // x 1500 keys 42 vs 60 us; 5 rows x 384 keys 7.7 vs 7.4 us (attn_softmax_force_nt: the test hook's A/B)
    // 512 threads for few (row, head) blocks of 257-512 keys (configs[4]'s self attention once the prompt carry
    // passes 256 keys): one row x 320-448 keys 6.3-6.8 us against 7.2-7.7 at 256 and 6.9-7.3 at 1024 threads
    // (profiles/r05p_sm_width_sweep.txt)
    const int f = attn_softmax_force_nt;
    if (f == 256 || (f == 0 && (n_rows * H > 128 || max_keys <= 256)))
        OWK_LAUNCH(k_attn_softmax<256>, dim3(H, n_rows), dim3(256), 0, s, q, ldq, kbase, vbase, ld_kv, hs, rows_dev,
                           key_idx, scale, out, ldo, amap, cap, cap_rows, out32);
    else if (f == 512 || (f == 0 && max_keys <= 512))
        OWK_LAUNCH(k_attn_softmax<512>, dim3(H, n_rows), dim3(512), 0, s, q, ldq, kbase, vbase, ld_kv, hs, rows_dev,
                           key_idx, scale, out, ldo, amap, cap, cap_rows, out32);
    else
        OWK_LAUNCH(k_attn_softmax<1024>, dim3(H, n_rows), dim3(1024), 0, s, q, ldq, kbase, vbase, ld_kv, hs, rows_dev,
                           key_idx, scale, out, ldo, amap, cap, cap_rows, out32);
}

int attn_max_listed_keys() { return AS_MAX_LIST; }
int attn_max_tiled_keys() { return DA_MAX_KEYS; }

void attn_cross_kernel(hipStream_t s, int which, const _Float16 * q, int ldq, const _Float16 * kbase,
                       const _Float16 * vbase, int hs, const AttnRow * rows_dev, int n_rows, int H, float scale,
                       _Float16 * out, int ldo) {
    if (n_rows <= 0) return;
    if (which == 1)
        OWK_LAUNCH((k_attn_step<false, true>), dim3(H, n_rows), dim3(64), 0, s, q, ldq, kbase, vbase, 64, hs, rows_dev,
                           nullptr, scale, out, ldo, nullptr, nullptr, nullptr);
    else if (which == 2)
        OWK_LAUNCH((k_attn_step<false, true, 2>), dim3(H, n_rows), dim3(128), 0, s, q, ldq, kbase, vbase, 64, hs,
                           rows_dev, nullptr, scale, out, ldo, nullptr, nullptr, nullptr);
    else
        throw std::runtime_error("attn_cross_kernel: which is 1 (one wave) or 2 (loader + math waves)");
}

void attn_decoder(hipStream_t s, const _Float16 * q, int ldq, const _Float16 * kbase, const _Float16 * vbase, int ld_kv,
                  int hs, const AttnRow * rows_dev, int n_rows, const int * key_idx, int H, float scale, int max_keys,
                  _Float16 * out, int ldo, bool any_one_chunk, bool any_tiled, float * out32, bool oc_listed,
                  int8_t * q8, float * q8d) {
    if (n_rows <= 0) return;
    if (any_one_chunk) {
        if (key_idx && oc_listed) {
            if (max_keys > AS_MAX_LIST) throw std::runtime_error("attn_decoder: too many listed keys");
            OWK_LAUNCH((k_attn_step<true, false>), dim3(H, n_rows), dim3(64), 0, s, q, ldq, kbase, vbase, ld_kv, hs,
                               rows_dev, key_idx, scale, out, ldo, out32, q8, q8d);
        } else {
            // cross attention (no cell lists): the once-per-step K/V stream, one wave per (row, head)
            // (the loader + math wave form: RTF 1073 / 1070 vs 1064 with one wave, attn_cross 47.8 vs 48.5 us in
            // the F16 bench step, bit-identical; profiles/r05n_attn_cross_ab.txt)
            if (!key_idx)
                OWK_LAUNCH((k_attn_step<false, true, 2>), dim3(H, n_rows), dim3(128), 0, s, q, ldq, kbase, vbase, ld_kv,
                                   hs, rows_dev, key_idx, scale, out, ldo, out32, q8, q8d);
            else  // self attention on contiguous cell runs: the same two-wave form (attn_self 78.8 -> 77.0 ms per
                  // F16 step in an interleaved A/B, bit-identical; profiles/r06r_self2_ab.txt)
                OWK_LAUNCH((k_attn_step<false, false, 2>), dim3(H, n_rows), dim3(128), 0, s, q, ldq, kbase, vbase, ld_kv,
                                   hs, rows_dev, key_idx, scale, out, ldo, out32, q8, q8d);
        }
    }
    if (any_tiled) {
        if (max_keys > DA_MAX_KEYS) throw std::runtime_error("attn_decoder: too many keys");
        OWK_LAUNCH(k_attn_decoder, dim3((H + 3) / 4, n_rows), dim3(256), 0, s, q, ldq, kbase, vbase, ld_kv,
                           hs, rows_dev, key_idx, H, scale, out, ldo, out32);
    }
}

} // namespace owk
