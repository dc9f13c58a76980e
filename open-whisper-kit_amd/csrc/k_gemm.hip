// MFMA f16 GEMMs with fused Whisper epilogues, gfx950.
//
// Numerics follow the reference ggml CPU mul_mat for F16 weights
// (ggml-cpu.c:1227 ggml_compute_forward_mul_mat, vec_dot_type F16): the activation
// operand is an f16 tensor (rounded once, RNE, by the producer kernel), products are
// exact in f32, accumulation is f32 (MFMA v_mfma_f32_16x16x32_f16). Only the order of
// the f32 additions differs from the reference SIMD dot product.
#include "kernels.h"

#include <algorithm>

namespace owk {

__device__ __forceinline__ float gelu_lookup(const uint16_t * tab, float x) {
    // ggml_vec_gelu_f32 with GGML_GELU_FP16 (ggml-cpu/vec.h:995-1009)
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    const _Float16 h = (_Float16) x;
    const uint16_t r = tab[__builtin_bit_cast(uint16_t, h)];
    return (float) __builtin_bit_cast(_Float16, r);
}

template <int MODE>
__device__ __forceinline__ void epi_store(const EpiParams & p, int r, int c, float acc) {
    if constexpr (MODE == EPI_F16) {
        float v = acc;
        if (p.bias) v += p.bias[c];
        v *= p.scale;
        p.out16[(size_t) r * p.ldo + c] = (_Float16) v;
    } else if constexpr (MODE == EPI_GELU_F16) {
        const float v = acc + p.bias[c];
        p.out16[(size_t) r * p.ldo + c] = (_Float16) gelu_lookup(p.gelu_tab, v);
    } else if constexpr (MODE == EPI_RESID_F32) {
        const float v = acc + p.bias[c];
        const size_t o = (size_t) r * p.ldo + c;
        p.out32[o] = p.resid[o] + v;
    } else if constexpr (MODE == EPI_CONV2) {
        const float v = gelu_lookup(p.gelu_tab, acc + p.bias[c]);
        const int t = r % p.T;
        p.out32[(size_t) r * p.ldo + c] = p.pos[(size_t) t * p.ldo + c] + v;
    } else if constexpr (MODE == EPI_QKV_ENC) {
        const int d = p.d;
        if (c < d) {
            p.out16[(size_t) r * d + c] = (_Float16) (acc + p.bias[c]);
        } else if (c < 2 * d) {
            p.out16b[(size_t) r * d + (c - d)] = (_Float16) acc;
        } else {
            const int cc = c - 2 * d;
            const int clip = r / p.T, t = r % p.T;
            const int h = cc >> 6, dim = cc & 63;
            const int H = d >> 6;
            p.out16c[(((size_t) clip * H + h) * 64 + dim) * p.Tpad + t] = (_Float16) (acc + p.bias2[cc]);
        }
    } else if constexpr (MODE == EPI_KV_CROSS) {
        const int d = p.d;
        const int clip = r / p.T, t = r - clip * p.T;
        const size_t row = (size_t) (p.slot_map ? p.slot_map[clip] : clip) * p.T + t;
        if (c < d) {
            p.out16b[row * d + c] = (_Float16) (acc * p.scale);
        } else {
            p.out16c[row * d + (c - d)] = (_Float16) (acc + p.bias2[c - d]);
        }
    } else if constexpr (MODE == EPI_QKV_DEC) {
        const int d = p.d;
        if (c < d) {
            p.out16[(size_t) r * p.ldo + c] = (_Float16) ((acc + p.bias[c]) * p.scale);
        } else if (c < 2 * d) {
            p.out16b[p.row_off[r] + (c - d)] = (_Float16) (acc * p.scale);
        } else {
            p.out16c[p.row_off[r] + (c - 2 * d)] = (_Float16) (acc + p.bias2[c - 2 * d]);
        }
    } else if constexpr (MODE == EPI_F32) {
        p.out32[(size_t) r * p.ldo + c] = acc;
    } else if constexpr (MODE == EPI_BIAS_F32) {
        const float v = p.bias ? acc + p.bias[c] : acc;
        const size_t o = (size_t) r * p.ldo + c;
        p.out32[o] = v;
        if (p.out16) p.out16[o] = (_Float16) v;
    } else if constexpr (MODE == EPI_SILU_F16) {
        // ggml_silu_f32 (ggml-cpu/vec.h): x / (1 + exp(-x))
        const float v = acc + p.bias[c];
        p.out16[(size_t) r * p.ldo + c] = (_Float16) (v / (1.0f + expf(-v)));
    } else if constexpr (MODE == EPI_HALF_RESID) {
        // ggml_add(x, b) -> ggml_scale(0.5) -> ggml_add(residual, .) (sortformer.cpp:1163-1167)
        const float v = (acc + p.bias[c]) * 0.5f;
        const size_t o = (size_t) r * p.ldo + c;
        p.out32[o] = p.resid[o] + v;
    } else if constexpr (MODE == EPI_RELU_F16) {
        const float v = acc + p.bias[c];
        p.out16[(size_t) r * p.ldo + c] = (_Float16) (v > 0.0f ? v : 0.0f);
    } else if constexpr (MODE == EPI_SIGMOID_F32) {
        const float v = acc + p.bias[c];
        p.out32[(size_t) r * p.ldo + c] = 1.0f / (1.0f + expf(-v));
    }
}
template <> __device__ __forceinline__ void epi_store<EPI_PARTIAL>(const EpiParams &, int, int, float) {}

typedef __attribute__((address_space(3))) void * lds_ptr_t;

// ---------------------------------------------------------------------------------
// 128x128x64 block tile, 4 waves (2x2) of 64x64, mfma_f32_16x16x32_f16.
// global -> LDS with global_load_lds (16 B/lane, lane-linear LDS image); the bank
// swizzle is applied on the global source address: physical 16-B chunk
// pc = c ^ ((row >> 1) & 7) makes every ds_read_b128 lane group conflict-free.
// ---------------------------------------------------------------------------------
constexpr int GB_M = 128, GB_N = 128, GB_K = 64;
constexpr int GB_STAGE = (GB_M + GB_N) * GB_K * 2;  // bytes per pipeline stage

template <int MODE>
__global__ __launch_bounds__(256, 2) void k_gemm_big(int M, int N, int K, const _Float16 * __restrict__ A, int lda,
                                                       const _Float16 * __restrict__ W, int ldw, EpiParams ep) {
    __shared__ __attribute__((aligned(1024))) char smem[2 * GB_STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // XCD-aware tile order: blocks b and b+8 land on the same XCD (round-robin
    // dispatch); give each XCD a contiguous run of tiles so neighbours share L2.
    const int nbn = (N + GB_N - 1) / GB_N;
    const int nb = gridDim.x;
    int bid = blockIdx.x;
    {
        const int xcd = bid & 7, q = nb >> 3, rr = nb & 7;
        const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
        bid = base + (bid >> 3);
    }
    const int bm = bid / nbn, bn = bid - bm * nbn;
    const int m0 = bm * GB_M, n0 = bn * GB_N;

    auto stage = [&](int buf, int k0) {
        char * sA = smem + buf * GB_STAGE;
        char * sB = sA + GB_M * GB_K * 2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int grp = wave * 4 + i;
            const int row = grp * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((row >> 1) & 7);
            const int ga = min(m0 + row, M - 1);
            const int gb = min(n0 + row, N - 1);
            __builtin_amdgcn_global_load_lds((const void *) (A + (size_t) ga * lda + k0 + c * 8),
                                             (lds_ptr_t) (sA + grp * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *) (W + (size_t) gb * ldw + k0 + c * 8),
                                             (lds_ptr_t) (sB + grp * 1024), 16, 0, 0);
        }
    };

    const int wm = wave >> 1, wn = wave & 1;
    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / GB_K;
    stage(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * GB_K);
        const char * sA = smem + cur * GB_STAGE;
        const char * sB = sA + GB_M * GB_K * 2;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            half8 a[4], b[4];
            const int c = ks * 4 + (lane >> 4);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int ra = wm * 64 + t * 16 + (lane & 15);
                const int rb = wn * 64 + t * 16 + (lane & 15);
                a[t] = *(const half8 *) (sA + ra * 128 + ((c ^ ((ra >> 1) & 7)) << 4));
                b[t] = *(const half8 *) (sB + rb * 128 + ((c ^ ((rb >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }

#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + e;
                if (r < M && c < N) epi_store<MODE>(ep, r, c, acc[i][j][e]);
            }
        }
}

// ---------------------------------------------------------------------------------
// Skinny GEMM for decode steps (M <= 64 rows): 8 waves per block share one 16-column
// slab of W, each wave streams 1/8 of K straight from HBM into registers (no LDS
// round trip: every W byte is used by exactly one wave), partial sums are reduced
// through LDS in a fixed wave order (deterministic) and the epilogue is fused.
// ---------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(512) void k_gemm_skinny(int M, int N, int K, const _Float16 * __restrict__ A, int lda,
                                                    const _Float16 * __restrict__ W, int ldw, EpiParams ep) {
    __shared__ floatx4 red[8][4][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = blockIdx.x * 16;
    const int MT = (M + 15) >> 4;
    const int nsteps = K >> 5;
    const int ks0 = (wave * nsteps) >> 3, ks1 = ((wave + 1) * nsteps) >> 3;

    floatx4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int n = min(n0 + (lane & 15), N - 1);
    const _Float16 * wp = W + (size_t) n * ldw + 8 * (lane >> 4);
    const _Float16 * ap[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ap[i] = A + (size_t) min(i * 16 + (lane & 15), M - 1) * lda + 8 * (lane >> 4);

    int ks = ks0;
    for (; ks + 1 < ks1; ks += 2) {
        const half8 b0 = *(const half8 *) (wp + ks * 32);
        const half8 b1 = *(const half8 *) (wp + ks * 32 + 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i < MT) {
                const half8 a0 = *(const half8 *) (ap[i] + ks * 32);
                const half8 a1 = *(const half8 *) (ap[i] + ks * 32 + 32);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, acc[i], 0, 0, 0);
            }
        }
    }
    if (ks < ks1) {
        const half8 b0 = *(const half8 *) (wp + ks * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i < MT) {
                const half8 a0 = *(const half8 *) (ap[i] + ks * 32);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, acc[i], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][i][lane] = acc[i];
    __syncthreads();
    if (tid < 256) {
        const int i = tid >> 6, ln = tid & 63;
        if (i < MT) {
            floatx4 s = red[0][i][ln];
#pragma unroll
            for (int w = 1; w < 8; ++w) s += red[w][i][ln];
            const int c = n0 + (ln & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = i * 16 + 4 * (ln >> 4) + e;
                if (r < M && c < N) epi_store<MODE>(ep, r, c, s[e]);
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// Decode-row GEMM (M <= 32 rows, the per-step decoder matmuls): weight streaming.
//
// Weights are read from a TILED copy made once at load time (tile_weights): the
// 16 x 32 (n x k) block an MFMA step consumes is stored as 1 KB in exactly the lane
// order of the B operand, so a wave's J k-steps are one contiguous J KB stream.
// One 16-column tile per block; wave w takes J consecutive k-steps and issues ALL its
// weight and activation loads before the first MFMA, so a launch has the whole weight
// matrix in flight -- the decode GEMM is a single HBM round trip. K beyond
// waves*J*32 is split over gridDim.y blocks; their partial tiles go to a workspace and
// a second small launch adds them in fixed k order (deterministic; no device-scope
// fence, which is costly across the 8 XCDs).
// ---------------------------------------------------------------------------------
constexpr int GR_MAXW = 16;  // waves per block

__global__ void k_tile_weights(const _Float16 * __restrict__ W, int N, int K, _Float16 * __restrict__ out) {
    const int nsteps = K >> 5;
    const size_t total = (size_t) ((N + 15) >> 4) * nsteps * 64;
    for (size_t p = (size_t) blockIdx.x * blockDim.x + threadIdx.x; p < total; p += (size_t) gridDim.x * blockDim.x) {
        const int l = (int) (p & 63);
        const size_t ts = p >> 6;
        const int st = (int) (ts % nsteps);
        const int t = (int) (ts / nsteps);
        const int n = t * 16 + (l & 15), k = st * 32 + 8 * (l >> 4);
        half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (n < N) v = *(const half8 *) (W + (size_t) n * K + k);
        *(half8 *) (out + p * 8) = v;
    }
}

void tile_weights(hipStream_t s, const _Float16 * W, int N, int K, _Float16 * out) {
    if (K % 32) throw std::runtime_error("tile_weights: K % 32");
    hipLaunchKernelGGL(k_tile_weights, dim3(2048), dim3(256), 0, s, W, N, K, out);
}

size_t tiled_weight_elems(int N, int K) { return (size_t) ((N + 15) / 16) * 16 * K; }

template <int MODE, int MT, int J>
__global__ __launch_bounds__(GR_MAXW * 64) void k_gemm_rows(int M, int N, int K, const _Float16 * __restrict__ A,
                                                            int lda, const _Float16 * __restrict__ Wt, EpiParams ep,
                                                            float * __restrict__ part) {
    __shared__ floatx4 red[GR_MAXW][MT][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int tile = blockIdx.x, n0 = tile * 16;
    const int nsteps = K >> 5;
    const int ks0 = (blockIdx.y * nw + wave) * J;
    const int nj = max(0, min(J, nsteps - ks0));

    // branch-free: every load is issued (k-step clamped into the matrix); operands past
    // this wave's k range are zeros so the extra MFMAs add exact zeros
    const half8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    const _Float16 * wp = Wt + ((size_t) tile * nsteps) * 512 + lane * 8;
    half8 b[J], a[MT][J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const half8 t = *(const half8 *) (wp + (size_t) min(ks0 + j, nsteps - 1) * 512);
        b[j] = j < nj ? t : z8;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const _Float16 * ap = A + (size_t) min(i * 16 + (lane & 15), M - 1) * lda + 8 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const half8 t = *(const half8 *) (ap + min(ks0 + j, nsteps - 1) * 32);
            a[i][j] = j < nj ? t : z8;
        }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every load issued ahead of the first wait
    floatx4 acc[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][j], b[j], acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < MT; ++i) red[wave][i][lane] = acc[i];
    __syncthreads();

    if (MODE != EPI_PARTIAL && gridDim.y > 1) {  // split-K partial tiles for k_gemm_rows_reduce
        if (tid < MT * 64) {
            const int i = tid >> 6, ln = tid & 63;
            floatx4 sum = red[0][i][ln];
            for (int w = 1; w < nw; ++w) sum += red[w][i][ln];
            ((floatx4 *) part)[(((size_t) blockIdx.y * gridDim.x + tile) * MT + i) * 64 + ln] = sum;
        }
        return;
    }
    // epilogue spread over every thread: one output (row r, column c) each, adjacent
    // threads on adjacent columns; the wave partials are summed in fixed wave order
    for (int o = tid; o < MT * 256; o += blockDim.x) {
        const int r = o >> 4, cc = o & 15;
        const int i = r >> 4, rr = r & 15;
        const int ln = 16 * (rr >> 2) + cc, e = rr & 3;
        const float * rp = (const float *) &red[0][i][ln] + e;
        float sum = rp[0];
        for (int w = 1; w < nw; ++w) sum += rp[w * MT * 64 * 4];
        const int c = n0 + cc;
        if (r < M && c < N) {
            if constexpr (MODE == EPI_PARTIAL)
                part[((size_t) blockIdx.y * M + r) * N + c] = sum;  // row-major [ks][M][N] for resid_layernorm
            else
                epi_store<MODE>(ep, r, c, sum);
        }
    }
}

template <int MODE, int MT>
__global__ __launch_bounds__(MT * 64) void k_gemm_rows_reduce(int M, int N, int KS, const float * __restrict__ part,
                                                              EpiParams ep) {
    const int tid = threadIdx.x, i = tid >> 6, ln = tid & 63;
    const int n0 = blockIdx.x * 16;
    floatx4 sum = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < KS; ++ks) sum += ((const floatx4 *) part)[(((size_t) ks * gridDim.x + blockIdx.x) * MT + i) * 64 + ln];
    const int c = n0 + (ln & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int r = i * 16 + 4 * (ln >> 4) + e;
        if (r < M && c < N) epi_store<MODE>(ep, r, c, sum[e]);
    }
}

// launch geometry of the decode-row GEMM: J k-steps per wave, nw waves, KS k-splits
struct RowsPlan {
    int J, nw, KS;
};
static int env_int(const char * name, int dflt) {
    const char * v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}
// partial (EPI_PARTIAL) launches split K for free (resid_layernorm adds the splits), so
// they take shorter k ranges per wave and twice the blocks; full-epilogue launches avoid
// a second (reduce) launch unless K is very long (tools/gemm_sweep.py measurements)
static RowsPlan rows_plan(int K, bool partial) {
    const int nsteps = K / 32;
    RowsPlan p;
    if (partial) p.J = nsteps <= 64 ? 2 : 4;
    else p.J = nsteps <= 32 ? 2 : nsteps <= 64 ? 4 : 8;
    static const int j_over = env_int("OWK_GR_J", 0), ks_over = env_int("OWK_GR_KS", 0);  // tuning sweeps
    if (j_over == 2 || j_over == 4 || j_over == 8) p.J = j_over;
    p.KS = (nsteps + GR_MAXW * p.J - 1) / (GR_MAXW * p.J);
    if (ks_over > p.KS && ks_over <= nsteps / p.J) p.KS = ks_over;
    const int per = (nsteps + p.KS - 1) / p.KS;
    p.nw = (per + p.J - 1) / p.J;
    return p;
}

template <template <int> class L, typename... Args> static void dispatch_mode(int mode, Args &&... args) {
    switch (mode) {
        case EPI_F16: L<EPI_F16>::run(args...); break;
        case EPI_GELU_F16: L<EPI_GELU_F16>::run(args...); break;
        case EPI_RESID_F32: L<EPI_RESID_F32>::run(args...); break;
        case EPI_CONV2: L<EPI_CONV2>::run(args...); break;
        case EPI_QKV_ENC: L<EPI_QKV_ENC>::run(args...); break;
        case EPI_KV_CROSS: L<EPI_KV_CROSS>::run(args...); break;
        case EPI_QKV_DEC: L<EPI_QKV_DEC>::run(args...); break;
        case EPI_F32: L<EPI_F32>::run(args...); break;
        case EPI_BIAS_F32: L<EPI_BIAS_F32>::run(args...); break;
        case EPI_SILU_F16: L<EPI_SILU_F16>::run(args...); break;
        case EPI_HALF_RESID: L<EPI_HALF_RESID>::run(args...); break;
        case EPI_RELU_F16: L<EPI_RELU_F16>::run(args...); break;
        case EPI_SIGMOID_F32: L<EPI_SIGMOID_F32>::run(args...); break;
        default: throw std::runtime_error("gemm: bad epilogue mode");
    }
}

template <int MODE> struct LaunchBig {
    static void run(hipStream_t s, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
                    const EpiParams & ep) {
        const int nbm = (M + GB_M - 1) / GB_M, nbn = (N + GB_N - 1) / GB_N;
        hipLaunchKernelGGL(k_gemm_big<MODE>, dim3(nbm * nbn), dim3(256), 0, s, M, N, K, A, lda, W, ldw, ep);
    }
};
template <int MODE> struct LaunchSkinny {
    static void run(hipStream_t s, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
                    const EpiParams & ep) {
        hipLaunchKernelGGL(k_gemm_skinny<MODE>, dim3((N + 15) / 16), dim3(512), 0, s, M, N, K, A, lda, W, ldw, ep);
    }
};

template <int MODE> struct LaunchRows {
    template <int MT, int J>
    static void go(hipStream_t s, dim3 grid, int nw, int M, int N, int K, const _Float16 * A, int lda,
                   const _Float16 * Wt, const EpiParams & ep, float * part) {
        hipLaunchKernelGGL((k_gemm_rows<MODE, MT, J>), grid, dim3(nw * 64), 0, s, M, N, K, A, lda, Wt, ep, part);
        if (grid.y > 1 && MODE != EPI_PARTIAL)
            hipLaunchKernelGGL((k_gemm_rows_reduce<MODE, MT>), dim3(grid.x), dim3(MT * 64), 0, s, M, N, (int) grid.y,
                               part, ep);
    }
    static void run(hipStream_t s, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * Wt,
                    const EpiParams & ep, const GemmWs * ws) {
        const RowsPlan pl = rows_plan(K, MODE == EPI_PARTIAL);
        const int tiles = (N + 15) / 16;
        float * part = nullptr;
        if (pl.KS > 1 || MODE == EPI_PARTIAL) {
            const size_t need = (size_t) pl.KS * tiles * 2 * 64 * 4;  // floats (MT <= 2)
            if (!ws || ws->partial_floats < need) throw std::runtime_error("gemm_rows: split-K workspace too small");
            part = ws->partial;
        }
        const dim3 grid(tiles, pl.KS);
        const bool one = M <= 16;
        switch (pl.J) {
            case 2: one ? go<1, 2>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part) : go<2, 2>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part); break;
            case 4: one ? go<1, 4>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part) : go<2, 4>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part); break;
            default: one ? go<1, 8>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part) : go<2, 8>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part); break;
        }
    }
};

static void check_shape(int M, int N, int K, int lda, int ldw, int kmul) {
    if (M <= 0 || N <= 0 || K <= 0 || K % kmul != 0 || lda < K || ldw < K || (lda % 8) || (ldw % 8))
        throw std::runtime_error("gemm: unsupported shape M=" + std::to_string(M) + " N=" + std::to_string(N) +
                                 " K=" + std::to_string(K));
}

void gemm_f16(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
              const EpiParams & ep) {
    check_shape(M, N, K, lda, ldw, GB_K);
    dispatch_mode<LaunchBig>(mode, s, M, N, K, A, lda, W, ldw, ep);
}

void gemm_f16_skinny(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W,
                     int ldw, const EpiParams & ep) {
    check_shape(M, N, K, lda, ldw, 32);
    if (M > 64) throw std::runtime_error("gemm_skinny: M > 64");
    dispatch_mode<LaunchSkinny>(mode, s, M, N, K, A, lda, W, ldw, ep);
}

size_t gemm_ws_floats(int N, int K) {
    const RowsPlan p = rows_plan(K, false);
    return p.KS > 1 ? (size_t) p.KS * ((N + 15) / 16) * 2 * 64 * 4 : 0;
}
size_t gemm_partial_floats(int N, int K) { return (size_t) rows_plan(K, true).KS * ((N + 15) / 16) * 2 * 64 * 4; }
int gemm_partial_splits(int K) { return rows_plan(K, true).KS; }

void gemm(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
          const EpiParams & ep, const GemmWs * ws, const _Float16 * Wt) {
    if (mode == EPI_PARTIAL) {
        if (!(M <= 32 && K % 32 == 0 && Wt && N % 16 == 0)) throw std::runtime_error("gemm: EPI_PARTIAL needs the decode-row path");
        check_shape(M, N, K, lda, ldw, 32);
        LaunchRows<EPI_PARTIAL>::run(s, M, N, K, A, lda, Wt, ep, ws);
        return;
    }
    if (M <= 32 && K % 32 == 0 && Wt) {
        check_shape(M, N, K, lda, ldw, 32);
        dispatch_mode<LaunchRows>(mode, s, M, N, K, A, lda, Wt, ep, ws);
    } else if (M <= 64 && K % 32 == 0) {
        gemm_f16_skinny(s, mode, M, N, K, A, lda, W, ldw, ep);
    } else {
        gemm_f16(s, mode, M, N, K, A, lda, W, ldw, ep);
    }
}

} // namespace owk
