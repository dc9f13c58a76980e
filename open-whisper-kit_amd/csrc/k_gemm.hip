// MFMA f16 GEMMs with fused Whisper epilogues, gfx950.
//
// Numerics follow the reference ggml CPU mul_mat for F16 weights
// (ggml-cpu.c:1227 ggml_compute_forward_mul_mat, vec_dot_type F16): the activation
// operand is an f16 tensor (rounded once, RNE, by the producer kernel), products are
// exact in f32, accumulation is f32 (MFMA v_mfma_f32_16x16x32_f16). Only the order of
// the f32 additions differs from the reference SIMD dot product.
#include "kernels.h"
#include "gemm_epi.h"

#include <algorithm>
#include <cstring>

namespace owk {

// the GEMM epilogues and the decode-row reduction order live in gemm_epi.h

// Eight consecutive outputs (row r, columns c .. c+7; c % 8 == 0) of one lane: the same values as
// eight epi_store calls, written with 16-byte vector accesses where the mode's layout allows (the
// per-element 2/4-byte stores of a large tile's epilogue were store-issue bound: MLP0 with GELU
// 1161 us against 861 us with an f32 epilogue, tools/gemm_big_check.py). vec: the row's 8 columns
// are inside N and every operand row start is 16-byte aligned (checked per launch).
__device__ __forceinline__ half8 to_half8(const float (&v)[8]) {
    half8 h;
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = f16_rn(v[e]);
    return h;
}
__device__ __forceinline__ void load8(const float * p, float (&v)[8]) {
    const float4 a = ((const float4 *) p)[0], b = ((const float4 *) p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(float * p, const float (&v)[8]) {
    ((float4 *) p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    ((float4 *) p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

template <int MODE>
__device__ __forceinline__ void epi_row8(const EpiParams & p, int r, int c, const float (&acc)[8], bool vec) {
    constexpr bool VEC = MODE == EPI_F16 || MODE == EPI_GELU_F16 || MODE == EPI_RESID_F32 || MODE == EPI_CONV2 ||
                         MODE == EPI_QKV_ENC || MODE == EPI_KV_CROSS || MODE == EPI_F32 || MODE == EPI_BIAS_F32 ||
                         MODE == EPI_SILU_F16 || MODE == EPI_HALF_RESID || MODE == EPI_RELU_F16 ||
                         MODE == EPI_SIGMOID_F32;
    if (!VEC || !vec) {
#pragma unroll
        for (int e = 0; e < 8; ++e) epi_store<MODE>(p, r, c + e, acc[e]);
        return;
    }
    float v[8], bb[8];
    const size_t o = (size_t) r * p.ldo + c;
    if constexpr (MODE == EPI_F16) {
        if (p.bias) load8(p.bias + c, bb);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ((p.bias ? acc[e] + bb[e] : acc[e])) * p.scale;
        *(half8 *) (p.out16 + o) = to_half8(v);
    } else if constexpr (MODE == EPI_GELU_F16) {
        load8(p.bias + c, bb);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_lookup(p.gelu_tab, acc[e] + bb[e]);
        *(half8 *) (p.out16 + o) = to_half8(v);
    } else if constexpr (MODE == EPI_RESID_F32 || MODE == EPI_HALF_RESID) {
        float rs[8];
        load8(p.bias + c, bb);
        load8(p.resid + o, rs);
#pragma unroll
        for (int e = 0; e < 8; ++e)
            v[e] = MODE == EPI_RESID_F32 ? rs[e] + (acc[e] + bb[e]) : rs[e] + (acc[e] + bb[e]) * 0.5f;
        store8(p.out32 + o, v);
    } else if constexpr (MODE == EPI_CONV2) {
        float ps[8];
        load8(p.bias + c, bb);
        load8(p.pos + (size_t) (r % p.T) * p.ldo + c, ps);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ps[e] + gelu_lookup(p.gelu_tab, acc[e] + bb[e]);
        store8(p.out32 + o, v);
    } else if constexpr (MODE == EPI_QKV_ENC) {
        // Q (+bias) and K columns only: V tiles keep the transposed per-element path
        const int d = p.d;
        if (c < d) {
            load8(p.bias + c, bb);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = acc[e] + bb[e];
            *(half8 *) (p.out16 + (size_t) r * d + c) = to_half8(v);
        } else if (c < 2 * d) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = acc[e];
            *(half8 *) (p.out16b + (size_t) r * d + (c - d)) = to_half8(v);
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) epi_store<MODE>(p, r, c + e, acc[e]);
        }
    } else if constexpr (MODE == EPI_KV_CROSS) {
        // 32-bit offsets (the host checks slots x T x d < 2^32) and the clip by a float reciprocal with an
        // exact integer fix-up instead of 64-bit products and an integer division: 574 -> 563-567 us per
        // launch at 32 clips x 1500 rows; the plain F16 epilogue of the same shape runs 346-358 us, so the
        // rest is the head-major stores (profiles/r05o_gemm_enc_modes.txt)
        const int d = p.d, T = p.T;
        int clip = (int) ((float) r * __builtin_amdgcn_rcpf((float) T));
        clip -= clip * T > r;
        clip += (clip + 1) * T <= r;
        const uint32_t t = (uint32_t) (r - clip * T);
        const uint32_t slot = (uint32_t) (p.slot_map ? p.slot_map[clip] : clip);
        const uint32_t base = slot * (uint32_t) T * (uint32_t) d + t * 64u;
        if (c < d) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = acc[e] * p.scale;
            *(half8 *) (p.out16b + (base + (uint32_t) (c >> 6) * (uint32_t) T * 64u + (uint32_t) (c & 63))) = to_half8(v);
        } else {
            const int cv = c - d;
            load8(p.bias2 + cv, bb);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = acc[e] + bb[e];
            *(half8 *) (p.out16c + (base + (uint32_t) (cv >> 6) * (uint32_t) T * 64u + (uint32_t) (cv & 63))) = to_half8(v);
        }
    } else if constexpr (MODE == EPI_F32) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = acc[e];
        store8(p.out32 + o, v);
    } else if constexpr (MODE == EPI_BIAS_F32) {
        if (p.bias) load8(p.bias + c, bb);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = p.bias ? acc[e] + bb[e] : acc[e];
        store8(p.out32 + o, v);
        if (p.out16) *(half8 *) (p.out16 + o) = to_half8(v);
    } else if constexpr (MODE == EPI_SILU_F16 || MODE == EPI_RELU_F16) {
        load8(p.bias + c, bb);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float x = acc[e] + bb[e];
            v[e] = MODE == EPI_SILU_F16 ? x / (1.0f + expf(-x)) : (x > 0.0f ? x : 0.0f);
        }
        if (p.out16) *(half8 *) (p.out16 + o) = to_half8(v);
        if (p.out32) store8(p.out32 + o, v);
    } else if constexpr (MODE == EPI_SIGMOID_F32) {
        load8(p.bias + c, bb);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 1.0f / (1.0f + expf(-(acc[e] + bb[e])));
        store8(p.out32 + o, v);
    }
}

// the vector epilogue's alignment requirements for this launch (16-byte rows of every operand)
static bool epi_vec_ok(int mode, const EpiParams & p, int N) {
    auto al = [](const void * q) { return ((uintptr_t) q & 15) == 0; };
    if (N % 8 || !al(p.bias) || !al(p.bias2) || !al(p.resid) || !al(p.out32) || !al(p.out16) || !al(p.out16b) ||
        !al(p.out16c) || !al(p.pos))
        return false;
    switch (mode) {
        case EPI_QKV_ENC: case EPI_KV_CROSS: return p.d % 8 == 0;
        case EPI_QKV_DEC: case EPI_PARTIAL: return false;
        default: return p.ldo % 8 == 0;
    }
}

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
            const int r0 = m0 + wm * 64 + i * 16 + 4 * (lane >> 4);
            if constexpr (MODE == EPI_QKV_ENC) {
                // V columns go to the transposed [clip][head][dim][Tpad] image: a lane's 4 rows
                // are 4 consecutive t of one clip (T % 4 == 0, r0 % 4 == 0): one 8-byte store
                const int d = ep.d;
                if (c >= 2 * d && c < N && r0 + 3 < M && ep.T % 4 == 0) {
                    const int cc = c - 2 * d;
                    const int clip = r0 / ep.T, t = r0 - clip * ep.T;
                    const float bv = ep.bias2[cc];
                    half4 hv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) hv[e] = (_Float16) (acc[i][j][e] + bv);
                    *(half4 *) (ep.out16c + (((size_t) clip * (d >> 6) + (cc >> 6)) * 64 + (cc & 63)) * ep.Tpad + t) = hv;
                    continue;
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = r0 + e;
                if (r < M && c < N) epi_store<MODE>(ep, r, c, acc[i][j][e]);
            }
        }
}

// ---------------------------------------------------------------------------------
// 64x64 block tile for mid-size GEMMs whose 128x128 grid leaves most CUs idle (SortFormer
// chunk passes: M = a few hundred rows, N = 192..2048; small Whisper models at one clip).
// Those launches are latency-bound: k_gemm_big keeps one 64-deep K stage in flight, so every
// stage pays a full load round trip (M 400 x N 512 x K 512: 16 blocks, 19 us). Here K advances
// in 32-deep steps through an 8-slot LDS ring (slot = 64 x 32 f16 of A + of W = 8 KB, 64 KB in
// all, two blocks per CU) with 7 steps in flight: top of step j: s_waitcnt vmcnt (this wave's
// step-j DMA landed, later steps stay in flight) -> s_barrier (every wave's step-j DMA landed,
// every wave done with step j-1) -> issue step j+7 into step j-1's slot -> 4 MFMAs per wave.
// 4 waves (2 x 2) of 32 x 32. Same MFMA sequence per output as k_gemm_big (32-deep K steps in
// ascending order): bit-identical results. LDS image: 64-B rows, 16-B chunk c of
// row r at c ^ ((r >> 2) & 3), swizzle applied on the global source address).
// ---------------------------------------------------------------------------------
constexpr int GM_K = 32, GM_SLOTS = 8;

// TM = 64: 4 waves (2 x 2) of 32 x 32; TM = 32 (twice the blocks of a narrow grid, for launches
// whose 64x64 grid still leaves CUs idle): 2 waves of 16 x 32. TM * 4 threads: thread t stages row
// t >> 2 of A and of W.
template <int MODE, int TM>
__global__ __launch_bounds__(TM * 4) void k_gemm_mid(int M, int N, int K, const _Float16 * __restrict__ A, int lda,
                                                    const _Float16 * __restrict__ W, int ldw, EpiParams ep) {
    constexpr int AHEAD = GM_SLOTS - 1;  // steps in flight beyond the one being computed
    constexpr int OP = TM * GM_K * 2;    // one operand of one K-step
    constexpr int WR = TM / 32;          // 16-row MFMA tiles per wave
    __shared__ __attribute__((aligned(1024))) char smem[GM_SLOTS * 2 * OP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = TM == 64 ? wave >> 1 : wave, wn = TM == 64 ? wave & 1 : 0;

    const int nbn = (N + TM - 1) / TM;
    const int nb = gridDim.x;
    int bid = blockIdx.x;
    {  // XCD-aware order (k_gemm_big): a contiguous run of tiles per XCD
        const int xcd = bid & 7, q = nb >> 3, rr = nb & 7;
        const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
        bid = base + (bid >> 3);
    }
    const int bm = bid / nbn, bn = bid - bm * nbn;
    const int m0 = bm * TM, n0 = bn * TM;

    // staging: thread t carries row t >> 2, 16-B chunk t & 3 of A and of W; wave w's 64 lanes
    // write rows 16w .. 16w+15 lane-linearly (1 KB)
    const int srow = tid >> 2;
    const int sch = ((lane & 3) ^ ((srow >> 2) & 3)) * 8;
    const _Float16 * ga = A + (size_t) min(m0 + srow, M - 1) * lda + sch;
    const _Float16 * gw = W + (size_t) min(n0 + srow, N - 1) * ldw + sch;
    auto stage = [&](int slot, int k0) {
        char * sA = smem + slot * 2 * OP + wave * 1024;
        __builtin_amdgcn_global_load_lds((const void *) (ga + k0), (lds_ptr_t) sA, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (gw + k0), (lds_ptr_t) (sA + OP), 16, 0, 0);
    };

    const int g = lane >> 4, l16 = lane & 15;
    int offA[WR], offB[2];
#pragma unroll
    for (int i = 0; i < WR; ++i) {
        const int ra = wm * 16 * WR + i * 16 + l16;
        offA[i] = ra * 64 + ((g ^ ((ra >> 2) & 3)) << 4);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int rb = wn * 32 + j * 16 + l16;
        offB[j] = OP + rb * 64 + ((g ^ ((rb >> 2) & 3)) << 4);
    }
    floatx4 acc[WR][2];
#pragma unroll
    for (int i = 0; i < WR; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / GM_K;
#pragma unroll
    for (int i = 0; i < AHEAD; ++i)
        if (i < nk) stage(i, i * GM_K);
    int slot = 0;
    for (int j = 0; j < nk; ++j) {
        // 2 loads per step per thread: steps j+1 .. j+later (issued) may stay in flight
        const int later = min(AHEAD - 1, nk - 1 - j);
        switch (later) {
            case 6: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
            case 5: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
            case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
            case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
            case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
            case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
            default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        }
        __builtin_amdgcn_s_barrier();
        if (j + AHEAD < nk) stage(slot == 0 ? GM_SLOTS - 1 : slot - 1, (j + AHEAD) * GM_K);  // step j-1's slot
        const char * sA = smem + slot * 2 * OP;
        half8 a[WR], b[2];
#pragma unroll
        for (int i = 0; i < WR; ++i) a[i] = *(const half8 *) (sA + offA[i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) b[i] = *(const half8 *) (sA + offB[i]);
#pragma unroll
        for (int i = 0; i < WR; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
                acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[jj], acc[i][jj], 0, 0, 0);
        slot = slot + 1 == GM_SLOTS ? 0 : slot + 1;
    }

#pragma unroll
    for (int i = 0; i < WR; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int c = n0 + wn * 32 + jj * 16 + l16;
            const int r0 = m0 + wm * 16 * WR + i * 16 + 4 * g;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (r0 + e < M && c < N) epi_store<MODE>(ep, r0 + e, c, acc[i][jj][e]);
        }
}

// ---------------------------------------------------------------------------------
// 256x256 block tiles for the large encoder / cross-KV GEMMs (M = clips x 1500 rows): k_gemm_8p below
// (and the quantized k_gemm_q16 with 128-row tiles). Round 2's 4/5-slot ring version (32-deep K-steps,
// two in flight across each barrier) was superseded by the 8-phase schedule (profiles/
// r03s6_gemm_8phase_vs_ring.txt: 8-17 % faster on every encoder shape) and removed in round 4.
// LDS images use 16-B chunks XOR-swizzled by row so the ds_read_b128 of 16 consecutive rows hit 16
// distinct bank groups.
// ---------------------------------------------------------------------------------
constexpr int G2_M = 256, G2_N = 256, G2_K = 32;

// Tile of the (XCD-remapped, so per-XCD contiguous) index t: groups of TO_GM row panels swept column
// by column, so the ~32 tiles an XCD runs at once cover 8 row panels x 4 column panels -- A and W
// panels both re-used from that XCD's L2 (row-major order ran 1.6 row panels x all 20 column
// panels of MLP0 at once: every W panel re-fetched per row panel, 2 GB of FETCH_SIZE per launch,
// profiles/archive/r02n_pmc_fetch_summary.txt)
constexpr int TO_GM = 8;
__device__ __forceinline__ void tile_order(int t, int ntiles, int nbn, int & bm, int & bn) {
    static const bool grouped = true;
    if (!grouped) {
        bm = t / nbn;
        bn = t - bm * nbn;
        return;
    }
    const int nbm = ntiles / nbn;
    const int per = TO_GM * nbn;
    const int grp = t / per, first = grp * TO_GM;
    const int gm = min(TO_GM, nbm - first);  // the last group may hold fewer row panels
    const int r = t - grp * per;
    bm = first + r % gm;
    bn = r / gm;
}

// ---------------------------------------------------------------------------------
// 256x256 block tile with the CDNA guide's 8-phase schedule (round 3; cdna_hip_programming.md §5
// "The 256^2 8-phase template"): K-tiles of 64, two LDS buffers of 64 KB (even / odd tiles), each
// cut into four 16 KB parts of 128 rows x 64 k:
//   A0 = A rows wr*128 + [0, 64) of both wave rows,   A1 = rows wr*128 + [64, 128),
//   W0 = W rows wc*64 + [0, 32) of all wave columns,  W1 = rows wc*64 + [32, 64).
// A wave (wr, wc) owns a 128 x 64 output block = four 64 x 32 quadrants; a K-tile is 4 phases, one
// quadrant each (16 MFMAs over K = 64), reading the fragments it needs first:
//   phase 1: A0 + W0 -> (A0, W0)   phase 2: W1 -> (A0, W1)   phase 3: A1 -> (A1, W1)   phase 4: -
//   (A1, W0)
// and staging one part of a later tile (2 global_load_lds of 16 B per thread): phases 1 / 2 stage W1 /
// A1 of tile t+1, phases 3 / 4 stage A0 / W0 of tile t+2 -- each at least two phases after that part's
// last read. Phase 4 ends with s_waitcnt vmcnt(4): the 4 loads of tile t+2 stay in flight, tile t+1 has
// landed (read from the next phase on, behind two barriers). Per phase: ds_reads + staging, s_barrier,
// lgkmcnt(0), 16 MFMAs under s_setprio(1), s_barrier; the two wave rows run one barrier apart (wave row 1
// takes an extra s_barrier first, wave row 0 one at the end), so one row's MFMAs overlap the other's LDS
// reads. 16-B chunk c of part row r is stored at chunk c ^ sw8(r): conflict-free ds_read_b128 for 16
// consecutive rows (A) and for the permuted W rows of the C^T tiles. Output and epilogues as
// round 2's ring kernel (SWAP: C^T tiles, 16-byte vector epilogues).
// ---------------------------------------------------------------------------------
constexpr int G8_K = 64;
constexpr int G8_PART = 128 * G8_K * 2;  // 16 KB
constexpr int G8_BUF = 4 * G8_PART;      // 64 KB

__device__ __forceinline__ int sw8(int r) {
    return ((r >> 1) & 1) | ((((r >> 2) ^ (r >> 3)) & 1) << 1) | ((((r >> 3) ^ (r >> 4)) & 1) << 2);
}

template <int MODE, bool SWAP>
__global__ __launch_bounds__(512, 1) void k_gemm_8p(int M, int N, int K, const _Float16 * __restrict__ A, int lda,
                                                    const _Float16 * __restrict__ W, int ldw, EpiParams ep) {
    __shared__ __attribute__((aligned(1024))) char smem[2 * G8_BUF];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int nbn = (N + G2_N - 1) / G2_N;
    const int nb = gridDim.x;
    int bid = blockIdx.x;
    {  // XCD-aware order, then the grouped tile order (tile_order)
        const int xcd = bid & 7, q = nb >> 3, rr = nb & 7;
        const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
        bid = base + (bid >> 3);
    }
    int bm, bn;
    tile_order(bid, nb, nbn, bm, bn);
    const int m0 = bm * G2_M, n0 = bn * G2_N;

    // staging: wave w fills part rows 16w .. 16w+15 of a part (2 x 1 KB pieces of 8 rows x 128 B);
    // lane l: row 16w + 8i + (l >> 3), physical chunk l & 7 <- logical chunk (l & 7) ^ sw8(row)
    const _Float16 * src[4][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int pr = wave * 16 + i * 8 + (lane >> 3);
        const int ch = ((lane & 7) ^ sw8(pr)) * 8;
        const int ra0 = (pr >> 6) * 128 + (pr & 63), ra1 = ra0 + 64;      // A0 / A1 part rows -> tile rows
        const int rw0 = (pr >> 5) * 64 + (pr & 31), rw1 = rw0 + 32;       // W0 / W1
        src[0][i] = A + (size_t) min(m0 + ra0, M - 1) * lda + ch;
        src[1][i] = A + (size_t) min(m0 + ra1, M - 1) * lda + ch;
        src[2][i] = W + (size_t) min(n0 + rw0, N - 1) * ldw + ch;
        src[3][i] = W + (size_t) min(n0 + rw1, N - 1) * ldw + ch;
    }
    const int nt = K / G8_K;
    // part p (0 A0, 1 A1, 2 W0, 3 W1) of tile t into buffer t & 1
    auto stage = [&](int p, int t) {
        char * dst = smem + (t & 1) * G8_BUF + p * G8_PART + wave * 2048;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const _Float16 * sp = p == 0 ? src[0][i] : p == 1 ? src[1][i] : p == 2 ? src[2][i] : src[3][i];
            __builtin_amdgcn_global_load_lds((const void *) (sp + (size_t) t * G8_K), (lds_ptr_t) (dst + i * 1024), 16, 0, 0);
        }
    };

    // fragment byte offsets inside a part: A frag i (of the wave's quadrant row) / W frag j, K half h
    const int g = lane >> 4, l16 = lane & 15;
    int offA[4], offW[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int pr = wr * 64 + i * 16 + l16;
        offA[i] = pr * 128 + ((g ^ sw8(pr)) << 4);  // logical chunk g (+ 4 for the second K half)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // swap: W frag j row p = wc*64 + (j>>1)*32 + (p>>2)*8 + (j&1)*4 + (p&3) (the C^T tiles' row permutation)
        const int pr = SWAP ? wc * 32 + (l16 >> 2) * 8 + (j & 1) * 4 + (l16 & 3) : wc * 32 + (j & 1) * 16 + l16;
        offW[j] = pr * 128 + ((g ^ sw8(pr)) << 4);
    }
    auto rdA = [&](const char * part, int i, int h) {  // chunk (h*4 + g) ^ sw8 = (g ^ sw8) ^ (h*4)
        return *(const half8 *) (part + (offA[i] ^ (h << 6)));
    };
    auto rdW = [&](const char * part, int j, int h) { return *(const half8 *) (part + (offW[j] ^ (h << 6))); };

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // prologue: tile 0 whole, tile 1's A0 / W0; tile 0 landed everywhere
    stage(0, 0);
    stage(2, 0);
    stage(3, 0);
    stage(1, 0);
    if (nt > 1) {
        stage(0, 1);
        stage(2, 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // the wave rows one barrier apart
    __builtin_amdgcn_sched_barrier(0);

    half8 fa[4][2], fw[4][2];
    auto mma = [&](int i0, int j0) {  // quadrant rows i0..i0+3 (fa), columns j0, j0+1 (fw)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (SWAP)
                        acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j0 + j][h], fa[i][h], acc[i0 + i][j0 + j], 0, 0, 0);
                    else
                        acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][h], fw[j0 + j][h], acc[i0 + i][j0 + j], 0, 0, 0);
                }
        __builtin_amdgcn_s_setprio(0);
    };
#define G8_SYNC_MMA(I0, J0)                                          \
    __builtin_amdgcn_sched_barrier(0);                               \
    __builtin_amdgcn_s_barrier();                                    \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");               \
    __builtin_amdgcn_sched_barrier(0);                               \
    mma(I0, J0);                                                     \
    __builtin_amdgcn_sched_barrier(0);                               \
    __builtin_amdgcn_s_barrier();                                    \
    __builtin_amdgcn_sched_barrier(0);

    for (int t = 0; t < nt; ++t) {
        const char * buf = smem + (t & 1) * G8_BUF;
        // phase 1: A0 + W0 fragments; stage W1 of tile t+1
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) fa[i][h] = rdA(buf, i, h);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) fw[j][h] = rdW(buf + 2 * G8_PART, j, h);
        if (t + 1 < nt) stage(3, t + 1);
        G8_SYNC_MMA(0, 0)
        // phase 2: W1 fragments; stage A1 of tile t+1
#pragma unroll
        for (int j = 2; j < 4; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) fw[j][h] = rdW(buf + 3 * G8_PART, j, h);
        if (t + 1 < nt) stage(1, t + 1);
        G8_SYNC_MMA(0, 2)
        // phase 3: A1 fragments; stage A0 of tile t+2
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) fa[i][h] = rdA(buf + G8_PART, i, h);
        if (t + 2 < nt) stage(0, t + 2);
        G8_SYNC_MMA(4, 2)
        // phase 4: no reads; stage W0 of tile t+2, then tile t+1 landed (t+2's 4 loads in flight)
        if (t + 2 < nt) {
            stage(2, t + 2);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        G8_SYNC_MMA(4, 0)
    }
#undef G8_SYNC_MMA
    if (wr == 0) __builtin_amdgcn_s_barrier();  // every wave ends on the same barrier count

    // GELU epilogues: the 64 K-entry f16 table (128 KB) is staged in the operand LDS once the main loop's
    // reads are done, so the tile's 65 536 lookups are LDS reads, not scattered 2-byte global loads
    EpiParams epl = ep;
    if constexpr (MODE == EPI_GELU_F16 || MODE == EPI_CONV2) {
        static_assert(2 * G8_BUF >= 65536 * 2, "GELU table in the operand LDS");
        __syncthreads();
        uint4 * lt = (uint4 *) smem;
        const uint4 * gt = (const uint4 *) ep.gelu_tab;
#pragma unroll 4
        for (int k = tid; k < 65536 * 2 / 16; k += 512) lt[k] = gt[k];
        __syncthreads();
        epl.gelu_tab = (const uint16_t *) smem;
    }
    if (SWAP) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = m0 + wr * 128 + i * 16 + l16;
            if (r >= M) continue;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = n0 + wc * 64 + h * 32 + g * 8;
                const float v[8] = {acc[i][2 * h][0], acc[i][2 * h][1], acc[i][2 * h][2], acc[i][2 * h][3],
                                    acc[i][2 * h + 1][0], acc[i][2 * h + 1][1], acc[i][2 * h + 1][2], acc[i][2 * h + 1][3]};
                if (c + 8 <= N) {
                    epi_row8<MODE>(epl, r, c, v, ep.vec != 0);
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        if (c + e < N) epi_store<MODE>(epl, r, c + e, v[e]);
                }
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int cl = n0 + wc * 64 + j * 16 + l16;
            const int c = cl + ep.c_off;
            const int r0 = m0 + wr * 128 + i * 16 + 4 * g;
            if constexpr (MODE == EPI_QKV_ENC) {
                const int d = ep.d;
                if (c >= 2 * d && cl < N && r0 + 3 < M && ep.T % 4 == 0) {
                    const int cc = c - 2 * d;
                    const int clip = r0 / ep.T, t = r0 - clip * ep.T;
                    const float bv = ep.bias2[cc];
                    half4 hv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) hv[e] = (_Float16) (acc[i][j][e] + bv);
                    *(half4 *) (ep.out16c + (((size_t) clip * (d >> 6) + (cc >> 6)) * 64 + (cc & 63)) * ep.Tpad + t) = hv;
                    continue;
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = r0 + e;
                if (r < M && cl < N) epi_store<MODE>(epl, r, c, acc[i][j][e]);
            }
        }
}

// ---------------------------------------------------------------------------------
// Quantized large-tile GEMM (gemm_q16: encoder / cross-K/V matrices of Q5_0 / Q8_0 / Q4_0 models).
// A = the Q8_0 integers of the activation rows and W = the weight integers, both as exact f16
// values; each 32-wide K-step is one quantization block: its MFMA dot is an exact integer
// (|sum| <= 32 * 127 * 16 < 2^24) that enters the f32 accumulator as
// acc = fma(dot, d_w * d_a, acc) -- ggml_vec_dot_q5_0_q8_0's per-block term (the f32 product of the
// two f16 scales, fused multiply-add). Block 128 x 256, 8 waves of 64 x 64 (acc 64 registers: the
// per-block scaling needs the room a 256-row tile does not leave), a ring of 32-deep K-steps (4 slots,
// two K-steps in flight across each barrier, counted vmcnt) carrying 128 A rows, 256 W rows and the
// step's 128 + 256 scales (da / dw block-major; da rows permuted so a lane's 4 rows are one float4).
// Output: C^T tiles (lane = 16 consecutive columns of one row), epi_row8 vector epilogues.
// ---------------------------------------------------------------------------------
constexpr int GQ16_M = 128;
constexpr int GQ16_A = GQ16_M * G2_K * 2;        // 8 KB
constexpr int GQ16_W = G2_N * G2_K * 2;          // 16 KB
constexpr int GQ16_SLOT = GQ16_A + GQ16_W + 2048;  // + da 512 B, dw 1 KB, 512 B scratch
constexpr int GQ16_SLOTS = 4;

template <int MODE>
__global__ __launch_bounds__(512, 2) void k_gemm_q16(int M, int N, int K, const _Float16 * __restrict__ A,
                                                     const _Float16 * __restrict__ W, EpiParams ep) {
    constexpr int AHEAD = GQ16_SLOTS - 2;
    __shared__ __attribute__((aligned(1024))) char smem[GQ16_SLOTS * GQ16_SLOT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int nbn = (N + G2_N - 1) / G2_N;
    const int nbt = gridDim.x;
    int bid = blockIdx.x;
    {  // XCD-aware order
        const int xcd = bid & 7, q = nbt >> 3, rr = nbt & 7;
        const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
        bid = base + (bid >> 3);
    }
    int bm, bn;
    tile_order(bid, nbt, nbn, bm, bn);
    const int m0 = bm * GQ16_M, n0 = bn * G2_N;

    auto wsw = [](int r) { return ((r >> 2) ^ (r >> 3)) & 3; };
    // staging: wave w: A rows 16w .. 16w+15 (one 1 KB piece), W rows 32w .. 32w+31 (two), one 256-B
    // scale piece (waves 0-1: d_a, 2-5: d_w, 6-7: a repeat of d_w pieces into scratch, so that every
    // wave issues 4 loads per step)
    const int arow = wave * 16 + (lane >> 2);
    const _Float16 * ga = A + (size_t) min(m0 + arow, M - 1) * K + ((lane & 3) ^ ((arow >> 2) & 3)) * 8;
    const _Float16 * gw[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = wave * 32 + i * 16 + (lane >> 2);
        gw[i] = W + (size_t) min(n0 + row, N - 1) * K + ((lane & 3) ^ wsw(row)) * 8;
    }
    const int sp = wave < 2 ? wave : wave < 6 ? wave - 2 : wave - 6;
    const float * gs = wave < 2 ? ep.qs_da + m0 + sp * 64 + lane * 4 : ep.qs_dw + n0 + sp * 64 + lane * 4;
    const size_t gs_step = wave < 2 ? (size_t) ep.qs_mpad : (size_t) ep.qs_npad;
    const int ls = wave < 2 ? GQ16_A + GQ16_W + sp * 256 : wave < 6 ? GQ16_A + GQ16_W + 512 + sp * 256
                                                                     : GQ16_A + GQ16_W + 1536 + sp * 256;
    auto stage = [&](int slot, int kstep) {
        char * base = smem + slot * GQ16_SLOT;
        const int k0 = kstep * G2_K;
        __builtin_amdgcn_global_load_lds((const void *) (ga + k0), (lds_ptr_t) (base + wave * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void *) (gw[i] + k0), (lds_ptr_t) (base + GQ16_A + wave * 2048 + i * 1024),
                                             16, 0, 0);
        if (lane < 16)
            __builtin_amdgcn_global_load_lds((const void *) (gs + (size_t) kstep * gs_step), (lds_ptr_t) (base + ls), 16, 0, 0);
    };

    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[i][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int g = lane >> 4, l16 = lane & 15;
    int offA[4], offB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = wr * 64 + i * 16 + l16;
        offA[i] = r * 64 + ((g ^ ((r >> 2) & 3)) << 4);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int r = wc * 64 + (t >> 1) * 32 + (l16 >> 2) * 8 + (t & 1) * 4 + (l16 & 3);
        offB[t] = GQ16_A + r * 64 + ((g ^ wsw(r)) << 4);
    }
    const int nk = K / G2_K;
    auto wait_step = [&](int next) {
        const int later = min(AHEAD - 1, nk - 1 - next);
        if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
#pragma unroll
    for (int i = 0; i < AHEAD; ++i)
        if (i < nk) stage(i, i);
    wait_step(0);
    __builtin_amdgcn_s_barrier();
    if (AHEAD < nk) stage(AHEAD, AHEAD);
    half8 b[4], a[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) b[t] = *(const half8 *) (smem + offB[t]);
    a[0] = *(const half8 *) (smem + offA[0]);
    a[1] = *(const half8 *) (smem + offA[1]);
    typedef float f2 __attribute__((ext_vector_type(2)));
    int slot = 0;
    for (int j = 0; j < nk; ++j) {
        const char * sA = smem + slot * GQ16_SLOT;
        const int nslot = slot + 1 == GQ16_SLOTS ? 0 : slot + 1;
        // this step's scales: d_a of the lane's 4 rows, d_w of its 16 columns
        const float * sc = (const float *) (sA + GQ16_A + GQ16_W);
        const float4 da4 = *(const float4 *) (sc + wr * 64 + l16 * 4);
        const float sda[4] = {da4.x, da4.y, da4.z, da4.w};
        f2 sdw[4][2];  // [t][pair]: columns (t >> 1) * 32 + g * 8 + (t & 1) * 4 + 2 * pair + {0, 1}
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float4 w0 = *(const float4 *) (sc + 128 + wc * 64 + h * 32 + g * 8);
            const float4 w1 = *(const float4 *) (sc + 128 + wc * 64 + h * 32 + g * 8 + 4);
            sdw[2 * h][0] = f2{w0.x, w0.y}; sdw[2 * h][1] = f2{w0.z, w0.w};
            sdw[2 * h + 1][0] = f2{w1.x, w1.y}; sdw[2 * h + 1][1] = f2{w1.z, w1.w};
        }
        half8 bn[4], an[2];
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
            if (gg == 0) {
                an[0] = *(const half8 *) (sA + offA[2]);
                an[1] = *(const half8 *) (sA + offA[3]);
            } else if (j + 1 < nk) {
                wait_step(j + 1);
                __builtin_amdgcn_s_barrier();
                if (j + 1 + AHEAD < nk) stage(slot == 0 ? GQ16_SLOTS - 1 : slot - 1, j + 1 + AHEAD);
                const char * nA = smem + nslot * GQ16_SLOT;
#pragma unroll
                for (int t = 0; t < 4; ++t) bn[t] = *(const half8 *) (nA + offB[t]);
                an[0] = *(const half8 *) (nA + offA[0]);
                an[1] = *(const half8 *) (nA + offA[1]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                floatx4 dot[4];
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    dot[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[t], a[i], floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                const float dav = sda[2 * gg + i];
                const f2 da2 = f2{dav, dav};
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int pr = 0; pr < 2; ++pr) {
                        const f2 dd = sdw[t][pr] * da2;  // d_w * d_a, f32
                        const f2 dt = f2{dot[t][2 * pr], dot[t][2 * pr + 1]};
                        f2 ac = f2{acc[2 * gg + i][t][2 * pr], acc[2 * gg + i][t][2 * pr + 1]};
                        ac = __builtin_elementwise_fma(dt, dd, ac);
                        acc[2 * gg + i][t][2 * pr] = ac.x;
                        acc[2 * gg + i][t][2 * pr + 1] = ac.y;
                    }
            }
            __builtin_amdgcn_sched_barrier(0);
            a[0] = an[0];
            a[1] = an[1];
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) b[t] = bn[t];
        slot = nslot;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = m0 + wr * 64 + i * 16 + l16;
        if (r >= M) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = n0 + wc * 64 + h * 32 + g * 8;
            const float v[8] = {acc[i][2 * h][0], acc[i][2 * h][1], acc[i][2 * h][2], acc[i][2 * h][3],
                                acc[i][2 * h + 1][0], acc[i][2 * h + 1][1], acc[i][2 * h + 1][2], acc[i][2 * h + 1][3]};
            if (c + 8 <= N) {
                epi_row8<MODE>(ep, r, c, v, ep.vec != 0);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (c + e < N) epi_store<MODE>(ep, r, c + e, v[e]);
            }
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
    OWK_LAUNCH(k_tile_weights, dim3(2048), dim3(256), 0, s, W, N, K, out);
}

size_t tiled_weight_elems(int N, int K) { return (size_t) ((N + 15) / 16) * 16 * K; }

template <int MODE, int MT, int J, bool NTW = false>  // NTW: non-temporal weight loads
__global__ __launch_bounds__(GR_MAXW * 64) void k_gemm_rows(int M, int N, int K, const _Float16 * __restrict__ A,
                                                            int lda, const _Float16 * __restrict__ Wt, EpiParams ep,
                                                            float * __restrict__ part) {
    __shared__ floatx4 red[GR_MAXW][MT][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int tile = blockIdx.x, n0 = tile * 16;
    const int nsteps = K >> 5;
    const int ks0 = (blockIdx.y * nw + wave) * J;
    const int nj = max(0, min(J, nsteps - ks0));
    const half8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};

    // branch-free: every load is issued (k-step clamped into the matrix); operands past
    // this wave's k range are zeros so the extra MFMAs add exact zeros
    const _Float16 * wp = Wt + ((size_t) tile * nsteps) * 512 + lane * 8;
    half8 b[J], a[MT][J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const half8 * src = (const half8 *) (wp + (size_t) min(ks0 + j, nsteps - 1) * 512);
        const half8 t = NTW ? __builtin_nontemporal_load(src) : *src;
        b[j] = j < nj ? t : z8;
    }
    __builtin_amdgcn_sched_barrier(0);  // the weight loads stay ahead of everything below

#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const _Float16 * ap = A + (size_t) min(i * 16 + (lane & 15), M - 1) * lda + 8 * (lane >> 4);
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const half8 t = *(const half8 *) (ap + min(ks0 + j, nsteps - 1) * 32);
                a[i][j] = j < nj ? t : z8;
            }
        }

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
        const float sum = wave_order_sum<GR_MAXW>((const float *) &red[0][i][ln] + e, MT * 64 * 4, nw);
        const int c = n0 + cc;
        if (r < M && c < N) {
            if constexpr (MODE == EPI_PARTIAL)
                part[((size_t) blockIdx.y * M + r) * N + c] = sum;  // row-major [ks][M][N] for resid_layernorm
            else
                epi_store<MODE>(ep, r, c, sum);
        }
    }
}

// k_gemm_rows with NT column tiles per block (KS = 1, full epilogues): every wave loads its activation
// fragments once and runs them against NT weight tiles, so the activation rows are read from L2 once per
// NT tiles instead of once per tile (the logits GEMM: 3242 tiles x 10 waves x 8 KB = 265 MB of L2
// reads for 133 MB of weights). Per output the same MFMA chain and the same fixed wave order as
// k_gemm_rows: bit-identical.
template <int MODE, int MT, int J, int NT>
__global__ __launch_bounds__(GR_MAXW * 64) void k_gemm_rows_nt(int M, int N, int K, const _Float16 * __restrict__ A,
                                                               int lda, const _Float16 * __restrict__ Wt, EpiParams ep,
                                                               float * __restrict__ part) {
    __shared__ floatx4 red[GR_MAXW][NT][MT][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int ntiles = (N + 15) >> 4, t0 = blockIdx.x * NT;
    const int nsteps = K >> 5;
    const int ks0 = (blockIdx.y * nw + wave) * J;  // EPI_PARTIAL: k split blockIdx.y
    const int nj = max(0, min(J, nsteps - ks0));
    const half8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    half8 b[NT][J], a[MT][J];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const _Float16 * wp = Wt + ((size_t) min(t0 + t, ntiles - 1) * nsteps) * 512 + lane * 8;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const half8 v = __builtin_nontemporal_load((const half8 *) (wp + (size_t) min(ks0 + j, nsteps - 1) * 512));
            b[t][j] = j < nj ? v : z8;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const _Float16 * ap = A + (size_t) min(i * 16 + (lane & 15), M - 1) * lda + 8 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const half8 v = *(const half8 *) (ap + min(ks0 + j, nsteps - 1) * 32);
            a[i][j] = j < nj ? v : z8;
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        floatx4 acc[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int i = 0; i < MT; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][j], b[t][j], acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MT; ++i) red[wave][t][i][lane] = acc[i];
    }
    __syncthreads();
    for (int o = tid; o < NT * MT * 256; o += blockDim.x) {
        const int t = o / (MT * 256), q = o - t * (MT * 256);
        const int r = q >> 4, cc = q & 15;
        const int i = r >> 4, rr = r & 15;
        const int ln = 16 * (rr >> 2) + cc, e = rr & 3;
        const float sum = wave_order_sum<GR_MAXW>((const float *) &red[0][t][i][ln] + e, NT * MT * 64 * 4, nw);
        const int c = (t0 + t) * 16 + cc;
        if (r < M && c < N) {
            if constexpr (MODE == EPI_PARTIAL)
                part[((size_t) blockIdx.y * M + r) * N + c] = sum;  // row-major [ks][M][N] for resid_layernorm
            else
                epi_store<MODE>(ep, r, c, sum);
        }
    }
}

// k_gemm_rows_nt with the decoder's LayerNorm in the prologue (F16 weights, M <= 32 rows, K = the
// LayerNorm width, one k split): A = f16(LayerNorm(x)) of the residual stream x [M][K] f32 -- what a
// separate resid_layernorm launch wrote as f16 rows before (ggml_norm + mul + add, ref whisper.cpp:
// 2528-2536, 2638-2646, 2750-2758). The waves of a block cover all K / 32 k-steps between them: each
// loads its k range of x for every row (the f32 values its MFMA A fragments are made of), the row
// statistics are combined over the waves in LDS in fixed wave order (mean = the f32 of the double sum
// / N; variance = the double sum of the f32-rounded centred squares / N, scale = 1 / sqrtf(var + eps),
// as resid_layernorm / ggml_norm, ops.cpp:3578-3623), and every lane forms its fragments in registers:
// no LDS image of the rows, no extra launch. The weight tiles are requested right after the x slices,
// so the statistics are computed while the weights stream in.
constexpr int GRL_MAXW = 10;  // waves per block: K <= GRL_MAXW * J * 32
template <int MODE, int MT, int J, int NT, bool STATS = true>
__global__ __launch_bounds__(GRL_MAXW * 64) void k_gemm_rows_ln(int M, int N, int K, const float * __restrict__ x,
                                                               const float * __restrict__ lnw,
                                                               const float * __restrict__ lnb, float eps,
                                                               const _Float16 * __restrict__ Wt, EpiParams ep) {
    __shared__ floatx4 red[GRL_MAXW][NT][MT][64];
    __shared__ double rs[2][GRL_MAXW][MT * 16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int ntiles = (N + 15) >> 4, t0 = blockIdx.x * NT;
    const int nsteps = K >> 5;
    const int ks0 = wave * J;
    const int nj = max(0, min(J, nsteps - ks0));
    const int cl = 8 * (lane >> 4);  // this lane's 8 columns inside a 32-wide k-step
    // x slices of this wave: rows i*16 + (lane & 15), columns (ks0 + j) * 32 + cl .. + 7
    float4 xv[MT][J][2];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const float * xr = x + (size_t) min(i * 16 + (lane & 15), M - 1) * K + cl;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const float4 * p = (const float4 *) (xr + min(ks0 + j, nsteps - 1) * 32);
            xv[i][j][0] = p[0];
            xv[i][j][1] = p[1];
        }
    }
    half8 b[NT][J];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const _Float16 * wp = Wt + ((size_t) min(t0 + t, ntiles - 1) * nsteps) * 512 + lane * 8;
#pragma unroll
        for (int j = 0; j < J; ++j)
            b[t][j] = __builtin_nontemporal_load((const half8 *) (wp + (size_t) min(ks0 + j, nsteps - 1) * 512));
    }
    __builtin_amdgcn_sched_barrier(0);
    const half8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < J; ++j)
            if (j >= nj) b[t][j] = z8;

    // row sums: this lane's 8 columns x nj k-steps, then the 4 lanes of a row, then the waves
    auto lane_group_sum = [&](double v) {
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        return v;
    };
    float mean[MT], scale[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) mean[i] = 0.0f, scale[i] = 1.0f;
    if constexpr (STATS) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (j < nj) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float4 v = xv[i][j][h];
                    s += ((double) v.x + (double) v.y) + ((double) v.z + (double) v.w);
                }
            }
        }
        s = lane_group_sum(s);
        if (lane < 16) rs[0][wave][i * 16 + lane] = s;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        double s = 0.0;
        for (int w = 0; w < nw; ++w) s += rs[0][w][i * 16 + (lane & 15)];
        mean[i] = (float) s / (float) K;
        double v = 0.0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (j < nj) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float4 q = xv[i][j][h];
                    const float tx = q.x - mean[i], ty = q.y - mean[i], tz = q.z - mean[i], tw = q.w - mean[i];
                    v += ((double) (tx * tx) + (double) (ty * ty)) + ((double) (tz * tz) + (double) (tw * tw));
                }
            }
        }
        v = lane_group_sum(v);
        if (lane < 16) rs[1][wave][i * 16 + lane] = v;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        double v = 0.0;
        for (int w = 0; w < nw; ++w) v += rs[1][w][i * 16 + (lane & 15)];
        const float var = (float) (v / (double) K);
        scale[i] = 1.0f / sqrtf(var + eps);
    }
    }
    // A fragments: f16((x - mean) * scale * w + b), the reference's separate roundings
    half8 a[MT][J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = min(ks0 + j, nsteps - 1) * 32 + cl;
        const float4 w0 = *(const float4 *) (lnw + c), w1 = *(const float4 *) (lnw + c + 4);
        const float4 b0 = *(const float4 *) (lnb + c), b1 = *(const float4 *) (lnb + c + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const float xs[8] = {xv[i][j][0].x, xv[i][j][0].y, xv[i][j][0].z, xv[i][j][0].w,
                                 xv[i][j][1].x, xv[i][j][1].y, xv[i][j][1].z, xv[i][j][1].w};
            half8 h;
#pragma unroll
            for (int e = 0; e < 8; ++e) h[e] = (_Float16) ((xs[e] - mean[i]) * scale[i] * wv[e] + bv[e]);
            a[i][j] = j < nj ? h : z8;
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        floatx4 acc[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int i = 0; i < MT; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][j], b[t][j], acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MT; ++i) red[wave][t][i][lane] = acc[i];
    }
    __syncthreads();
    for (int o = tid; o < NT * MT * 256; o += blockDim.x) {
        const int t = o / (MT * 256), q = o - t * (MT * 256);
        const int r = q >> 4, cc = q & 15;
        const int i = r >> 4, rr = r & 15;
        const int ln = 16 * (rr >> 2) + cc, e = rr & 3;
        float sum = ((const float *) &red[0][t][i][ln])[e];
        for (int w = 1; w < nw; ++w) sum += ((const float *) &red[w][t][i][ln])[e];
        const int c = (t0 + t) * 16 + cc;
        if (r < M && c < N) epi_store<MODE>(ep, r, c, sum);
    }
}

// ---------------------------------------------------------------------------------
// Whole-K forms of the decoder's chain for passes of <= 16 rows that reproduce the split chain BIT FOR
// BIT (a clip's result must not depend on how many rows share its decode pass):
//   k_gemm_rows_res: the residual matmul (attn.out, cross_attn.out, mlp.2) in one launch. Its waves
//     play the split-K plan's (k split y, wave w) roles -- same k-steps, same MFMA chains -- and the
//     epilogue adds the wave partials of each split in wave order, the splits in split order, then
//     bias and residual: exactly the EPI_PARTIAL launch + resid_layernorm's x update.
//   k_gemm_rows_lnx: the next matmul with the LayerNorm in its prologue, its statistics formed in the
//     order of the kernel that wrote the f16 rows in the split chain (ORDER 0: resid_layernorm's 256
//     threads x 2 float4 and its wave trees; ORDER 1: layernorm_f16's wave per row, 8 float4 per lane,
//     every lane its own butterfly sum) from per-float4 pair sums exchanged in LDS, and the GEMM's
//     waves, k-steps and MFMA chains those of the full-epilogue decode-row plan (rows_plan).
// ---------------------------------------------------------------------------------
constexpr int LNX_MAX_ROWS = 16, LNX_MAX4 = 320;  // rows per pass, float4 per row (d <= 1280)

template <int J, int KS>
__global__ __launch_bounds__(GR_MAXW * 64) void k_gemm_rows_res(int M, int N, int K, const _Float16 * __restrict__ A,
                                                                const _Float16 * __restrict__ Wt,
                                                                const float * __restrict__ bias, float * __restrict__ x) {
    __shared__ floatx4 red[KS][GR_MAXW][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int tile = blockIdx.x, n0 = tile * 16;
    const int nsteps = K >> 5;
    const half8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    const _Float16 * wp = Wt + ((size_t) tile * nsteps) * 512 + lane * 8;
    half8 b[KS][J], a[KS][J];
#pragma unroll
    for (int y = 0; y < KS; ++y)
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int ks = (y * nw + wave) * J + j;
            const half8 t = __builtin_nontemporal_load((const half8 *) (wp + (size_t) min(ks, nsteps - 1) * 512));
            b[y][j] = ks < nsteps ? t : z8;
        }
    __builtin_amdgcn_sched_barrier(0);
    const _Float16 * ap = A + (size_t) min(lane & 15, M - 1) * K + 8 * (lane >> 4);
#pragma unroll
    for (int y = 0; y < KS; ++y)
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int ks = (y * nw + wave) * J + j;
            const half8 t = *(const half8 *) (ap + min(ks, nsteps - 1) * 32);
            a[y][j] = ks < nsteps ? t : z8;
        }
#pragma unroll
    for (int y = 0; y < KS; ++y) {
        floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < J; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[y][j], b[y][j], acc, 0, 0, 0);
        red[y][wave][lane] = acc;
    }
    __syncthreads();
    for (int o = tid; o < 256; o += blockDim.x) {
        const int r = o >> 4, cc = o & 15;
        const int ln = 16 * (r >> 2) + cc, e = r & 3;
        float a_sum = 0.0f;
#pragma unroll
        for (int y = 0; y < KS; ++y) {
            float sy = ((const float *) &red[y][0][ln])[e];
            for (int w = 1; w < nw; ++w) sy += ((const float *) &red[y][w][ln])[e];
            a_sum = y == 0 ? sy : a_sum + sy;
        }
        const int c = n0 + cc;
        if (r < M && c < N) {
            const size_t oi = (size_t) r * N + c;
            x[oi] = x[oi] + (a_sum + bias[c]);
        }
    }
}

__device__ __forceinline__ double pair_sum_d(const float4 v) {
    return ((double) v.x + (double) v.y) + ((double) v.z + (double) v.w);
}
__device__ __forceinline__ double pair_sq_d(const float4 v, float m) {
    const float tx = v.x - m, ty = v.y - m, tz = v.z - m, tw = v.w - m;
    return ((double) (tx * tx) + (double) (ty * ty)) + ((double) (tz * tz) + (double) (tw * tw));
}
__device__ __forceinline__ double wave_bfly_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int MODE, int J, int NT, int ORDER>
__global__ __launch_bounds__(GR_MAXW * 64) void k_gemm_rows_lnx(int M, int N, int K, const float * __restrict__ x,
                                                                const float * __restrict__ lnw,
                                                                const float * __restrict__ lnb, float eps,
                                                                const _Float16 * __restrict__ Wt, EpiParams ep) {
    __shared__ floatx4 red[GR_MAXW][NT][64];
    __shared__ double pd[LNX_MAX_ROWS][LNX_MAX4];
    __shared__ double rs[LNX_MAX_ROWS][4];
    __shared__ float mrow[LNX_MAX_ROWS][64], srow[LNX_MAX_ROWS][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int ntiles = (N + 15) >> 4, t0 = blockIdx.x * NT;
    const int nsteps = K >> 5, n4 = K >> 2;
    const int ks0 = wave * J;
    const int nj = max(0, min(J, nsteps - ks0));
    const int g = lane >> 4, row = lane & 15;
    const bool own = row < M;  // lanes of clamped rows only read
    float4 xv[J][2];
    {
        const float * xr = x + (size_t) min(row, M - 1) * K + 8 * g;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const float4 * p = (const float4 *) (xr + min(ks0 + j, nsteps - 1) * 32);
            xv[j][0] = p[0];
            xv[j][1] = p[1];
        }
    }
    half8 b[NT][J];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const _Float16 * wp = Wt + ((size_t) min(t0 + t, ntiles - 1) * nsteps) * 512 + lane * 8;
#pragma unroll
        for (int j = 0; j < J; ++j)
            b[t][j] = __builtin_nontemporal_load((const half8 *) (wp + (size_t) min(ks0 + j, nsteps - 1) * 512));
    }
    __builtin_amdgcn_sched_barrier(0);
    // float4 index of (j, h) in the row: k-step * 8 + 2 g + h
    auto f4 = [&](int j, int h) { return (ks0 + j) * 8 + 2 * g + h; };
    // 1. pair sums of every float4 of the rows
#pragma unroll
    for (int j = 0; j < J; ++j)
        if (j < nj && own)
#pragma unroll
            for (int h = 0; h < 2; ++h) pd[row][f4(j, h)] = pair_sum_d(xv[j][h]);
    __syncthreads();
    // 2. the mean, in the partition of the split chain's LayerNorm kernel
    if constexpr (ORDER == 0) {
        for (int task = wave; task < M * 4; task += nw) {
            const int r = task >> 2, vw = task & 3, t = vw * 64 + lane;
            double s = 0.0;
            s += t < n4 ? pd[r][t] : 0.0;
            s += t + 256 < n4 ? pd[r][t + 256] : 0.0;
            s = wave_bfly_sum_d(s);
            if (lane == 0) rs[r][vw] = s;
        }
    } else {
        for (int r = wave; r < M; r += nw) {
            double s = 0.0;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) s += lane + 64 * jj < n4 ? pd[r][lane + 64 * jj] : 0.0;
            s = wave_bfly_sum_d(s);
            mrow[r][lane] = (float) s / (float) K;
        }
    }
    __syncthreads();
    float mean_r = 0.0f;
    if constexpr (ORDER == 0)
        mean_r = (float) ((rs[min(row, M - 1)][0] + rs[min(row, M - 1)][1]) +
                          (rs[min(row, M - 1)][2] + rs[min(row, M - 1)][3])) / (float) K;
    auto mean_of = [&](int i) { return ORDER == 0 ? mean_r : mrow[min(row, M - 1)][i & 63]; };
    // 3. centred squares (f32 difference and square, as the LayerNorm kernels), same partitions
#pragma unroll
    for (int j = 0; j < J; ++j)
        if (j < nj && own)
#pragma unroll
            for (int h = 0; h < 2; ++h) pd[row][f4(j, h)] = pair_sq_d(xv[j][h], mean_of(f4(j, h)));
    __syncthreads();
    if constexpr (ORDER == 0) {
        for (int task = wave; task < M * 4; task += nw) {
            const int r = task >> 2, vw = task & 3, t = vw * 64 + lane;
            double v = 0.0;
            if (t < n4) v += pd[r][t];
            if (t + 256 < n4) v += pd[r][t + 256];
            v = wave_bfly_sum_d(v);
            if (lane == 0) rs[r][vw] = v;
        }
    } else {
        for (int r = wave; r < M; r += nw) {
            double v = 0.0;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj)
                if (lane + 64 * jj < n4) v += pd[r][lane + 64 * jj];
            v = wave_bfly_sum_d(v);
            srow[r][lane] = 1.0f / sqrtf((float) (v / (double) K) + eps);
        }
    }
    __syncthreads();
    float scale_r = 0.0f;
    if constexpr (ORDER == 0) {
        const int rr = min(row, M - 1);
        const float var = (float) (((rs[rr][0] + rs[rr][1]) + (rs[rr][2] + rs[rr][3])) / (double) K);
        scale_r = 1.0f / sqrtf(var + eps);
    }
    auto scale_of = [&](int i) { return ORDER == 0 ? scale_r : srow[min(row, M - 1)][i & 63]; };
    // 4. A fragments f16((x - mean) * scale * w + b)
    const half8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    half8 a[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = min(ks0 + j, nsteps - 1) * 32 + 8 * g;
        const float4 w0 = *(const float4 *) (lnw + c), w1 = *(const float4 *) (lnw + c + 4);
        const float4 b0 = *(const float4 *) (lnb + c), b1 = *(const float4 *) (lnb + c + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        const float xs[8] = {xv[j][0].x, xv[j][0].y, xv[j][0].z, xv[j][0].w, xv[j][1].x, xv[j][1].y, xv[j][1].z, xv[j][1].w};
        half8 hv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int i = f4(j, e >> 2);
            hv[e] = (_Float16) ((xs[e] - mean_of(i)) * scale_of(i) * wv[e] + bv[e]);
        }
        a[j] = j < nj ? hv : z8;
        if (j >= nj)
#pragma unroll
            for (int t = 0; t < NT; ++t) b[t][j] = z8;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < J; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[j], b[t][j], acc, 0, 0, 0);
        red[wave][t][lane] = acc;
    }
    __syncthreads();
    for (int o = tid; o < NT * 256; o += blockDim.x) {
        const int t = o >> 8, q = o & 255;
        const int r = q >> 4, cc = q & 15;
        const int ln = 16 * (r >> 2) + cc, e = r & 3;
        float sum = ((const float *) &red[0][t][ln])[e];
        for (int w = 1; w < nw; ++w) sum += ((const float *) &red[w][t][ln])[e];
        const int c = (t0 + t) * 16 + cc;
        if (r < M && c < N) epi_store<MODE>(ep, r, c, sum);
    }
}

template <int MODE, bool STATS = true> struct LaunchRowsLn {
    static void run(hipStream_t s, int M, int N, int K, const float * x, const float * lnw, const float * lnb, float eps,
                    const _Float16 * Wt, const EpiParams & ep) {
        const int nsteps = K / 32;
        const int J = nsteps <= 2 * GRL_MAXW ? 2 : 4;
        const int nw = (nsteps + J - 1) / J;
        const int tiles = (N + 15) / 16;
        // two column tiles per block where that still gives >= 128 blocks (QKV, MLP0); one otherwise
        const int nt = (tiles + 1) / 2 >= 128 ? 2 : 1;
        const dim3 g((tiles + nt - 1) / nt);
        const bool one = M <= 16;
#define OWK_ROWS_LN_GO(MT_, J_, NT_) \
    OWK_LAUNCH((k_gemm_rows_ln<MODE, MT_, J_, NT_, STATS>), g, dim3(nw * 64), 0, s, M, N, K, x, lnw, lnb, eps, Wt, ep)
        if (J == 4) {
            if (nt == 2) { if (one) OWK_ROWS_LN_GO(1, 4, 2); else OWK_ROWS_LN_GO(2, 4, 2); }
            else { if (one) OWK_ROWS_LN_GO(1, 4, 1); else OWK_ROWS_LN_GO(2, 4, 1); }
        } else {
            if (nt == 2) { if (one) OWK_ROWS_LN_GO(1, 2, 2); else OWK_ROWS_LN_GO(2, 2, 2); }
            else { if (one) OWK_ROWS_LN_GO(1, 2, 1); else OWK_ROWS_LN_GO(2, 2, 1); }
        }
#undef OWK_ROWS_LN_GO
    }
};

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
// partial (EPI_PARTIAL) launches split K for free (resid_layernorm adds the splits), so
// they take shorter k ranges per wave and twice the blocks; full-epilogue launches avoid
// a second (reduce) launch unless K is very long (tools/gemm_sweep.py measurements)
static RowsPlan rows_plan(int K, bool partial) {
    const int nsteps = K / 32;
    RowsPlan p;
    // full epilogues take the whole K in one block up to 160 k-steps (K = 5120, the MLP's second
    // matmul: J = 10 x 16 waves), so no reduce launch follows
    if (partial) p.J = nsteps <= 64 ? 2 : 4;
    else p.J = nsteps <= 32 ? 2 : nsteps <= 64 ? 4 : nsteps <= 128 ? 8 : 10;
    p.KS = (nsteps + GR_MAXW * p.J - 1) / (GR_MAXW * p.J);
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
        OWK_LAUNCH(k_gemm_big<MODE>, dim3(nbm * nbn), dim3(256), 0, s, M, N, K, A, lda, W, ldw, ep);
    }
};
static int mid_tile(int M, int N);
template <int MODE> struct LaunchMid {
    static void run(hipStream_t s, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
                    const EpiParams & ep) {
        if (mid_tile(M, N) == 32)
            OWK_LAUNCH((k_gemm_mid<MODE, 32>), dim3(((M + 31) / 32) * ((N + 31) / 32)), dim3(128), 0, s, M, N, K, A, lda, W,
                       ldw, ep);
        else
            OWK_LAUNCH((k_gemm_mid<MODE, 64>), dim3(((M + 63) / 64) * ((N + 63) / 64)), dim3(256), 0, s, M, N, K, A, lda, W,
                       ldw, ep);
    }
};
// 256x256 kernel: the 8-phase k_gemm_8p (K % 64 == 0; other shapes take the 128x128 tile). The
// debug hooks override the choice per thread (gemm_set_256: 0 = the 128x128 tile, GEMM_MID_FORCED /
// GEMM_MID32_FORCED = the ring tiles for every shape) so a hook never changes another thread's engine
static thread_local int t_gemm256 = -1;  // -1: no override
static int gemm256_mode() { return t_gemm256 >= 0 ? t_gemm256 : 8; }
template <int MODE> struct Launch256 {
    static void run(hipStream_t s, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
                    const EpiParams & ep) {
        const int nbm = (M + G2_M - 1) / G2_M, nbn = (N + G2_N - 1) / G2_N;
        EpiParams e = ep;
        e.vec = epi_vec_ok(MODE, ep, N) ? 1 : 0;
        // EPI_QKV_ENC: C tiles (its V columns are written transposed, 4 consecutive key positions per
        // lane); every other epilogue: C^T tiles with 16-byte vector stores
        if (MODE == EPI_QKV_ENC)
            OWK_LAUNCH((k_gemm_8p<MODE, false>), dim3(nbm * nbn), dim3(512), 0, s, M, N, K, A, lda, W, ldw, e);
        else
            OWK_LAUNCH((k_gemm_8p<MODE, true>), dim3(nbm * nbn), dim3(512), 0, s, M, N, K, A, lda, W, ldw, e);
    }
};
template <int MODE> struct Launch256Q {
    static void run(hipStream_t s, int M, int N, int K, const _Float16 * q16, const float * dat, int mpad, const Q5W & w,
                    const EpiParams & ep) {
        const int nbm = (M + GQ16_M - 1) / GQ16_M, nbn = (N + G2_N - 1) / G2_N;
        EpiParams e = ep;
        e.vec = epi_vec_ok(MODE, ep, N) ? 1 : 0;
        e.qs_da = dat;
        e.qs_dw = w.dwt;
        e.qs_mpad = mpad;
        e.qs_npad = w.npad;
        OWK_LAUNCH(k_gemm_q16<MODE>, dim3(nbm * nbn), dim3(512), 0, s, M, N, K, q16, w.wi, e);
    }
};
template <int MODE> struct LaunchSkinny {
    static void run(hipStream_t s, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
                    const EpiParams & ep) {
        OWK_LAUNCH(k_gemm_skinny<MODE>, dim3((N + 15) / 16), dim3(512), 0, s, M, N, K, A, lda, W, ldw, ep);
    }
};

template <int MODE> struct LaunchRows {
    template <int MT, int J>
    static void go(hipStream_t s, dim3 grid, int nw, int M, int N, int K, const _Float16 * A, int lda,
                   const _Float16 * Wt, const EpiParams & ep, float * part) {
        // non-temporal weight loads: every decode-step weight is read once per step (3.5 % off the
        // per-layer matmul chain, tools/chain_sweep.py: 51.6 -> 49.8 us)
        OWK_LAUNCH((k_gemm_rows<MODE, MT, J, true>), grid, dim3(nw * 64), 0, s, M, N, K, A, lda, Wt, ep, part);
        if (grid.y > 1 && MODE != EPI_PARTIAL)
            OWK_LAUNCH((k_gemm_rows_reduce<MODE, MT>), dim3(grid.x), dim3(MT * 64), 0, s, M, N, (int) grid.y,
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
        // full-epilogue launches with many column tiles take 2 per block (a wave's activation
        // fragments serve both): the logits GEMM 47.7 -> 37.0 us for 32 x 51866 x 1280
        // (profiles/archive/r03n_logits_gemm_nt.txt), MLP0 9.7 -> 8.0 us; where halving the grid would leave
        // fewer than 128 blocks (cross-Q, attn.out: N = 1280 -> 40 blocks) one tile per block is faster
        // (r04: cross-Q 7.1 us with 2, 5.7 with 1); split-K partial launches measured slower with 2
        // (r04b A/B, large-v3 RTF 1017 vs 1026)
        if (MODE != EPI_PARTIAL && pl.KS == 1 && (pl.J == 4 || pl.J == 2) && (tiles + 1) / 2 >= 128) {
            const dim3 g((tiles + 1) / 2, 1);
#define OWK_ROWS_NT_GO(MT_, J_) \
    OWK_LAUNCH((k_gemm_rows_nt<MODE, MT_, J_, 2>), g, dim3(pl.nw * 64), 0, s, M, N, K, A, lda, Wt, ep, part)
            if (pl.J == 4) { if (one) OWK_ROWS_NT_GO(1, 4); else OWK_ROWS_NT_GO(2, 4); }
            else { if (one) OWK_ROWS_NT_GO(1, 2); else OWK_ROWS_NT_GO(2, 2); }
#undef OWK_ROWS_NT_GO
            return;
        }
        switch (pl.J) {
            case 2: one ? go<1, 2>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part)
                        : go<2, 2>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part); break;
            case 4: one ? go<1, 4>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part)
                        : go<2, 4>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part); break;
            case 8: one ? go<1, 8>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part)
                        : go<2, 8>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part); break;
            case 10: one ? go<1, 10>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part)
                         : go<2, 10>(s, grid, pl.nw, M, N, K, A, lda, Wt, ep, part); break;
            default: throw std::runtime_error("gemm_rows: no kernel for this plan");
        }
    }
};

// ---------------------------------------------------------------------------------
// Q5_0 x Q8_0 (see kernels.h). Activation rows -> Q8_0 with the x86 rounding of
// quantize_row_q8_0: d = amax / 127 (stored f16), q = rne(x * (127 / amax)).
// One 32-lane half-wave per block.
// ---------------------------------------------------------------------------------
template <typename TA>
__global__ __launch_bounds__(256) void k_quantize_q8(const TA * __restrict__ A, int lda, int M, int K,
                                                     int8_t * __restrict__ q, float * __restrict__ dq) {
    const int nb = K >> 5;
    const size_t total = (size_t) M * nb;
    const int lane = threadIdx.x & 31;
    for (size_t blk = ((size_t) blockIdx.x * blockDim.x + threadIdx.x) >> 5; blk < total;
         blk += ((size_t) gridDim.x * blockDim.x) >> 5) {
        const int r = (int) (blk / nb), b = (int) (blk - (size_t) r * nb);
        const float x = (float) A[(size_t) r * lda + b * 32 + lane];
        float am = fabsf(x);
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 32));
        const float dd = am / 127.f;
        const float id = am != 0.0f ? 127.f / am : 0.0f;
        q[(size_t) r * K + b * 32 + lane] = (int8_t) rintf(x * id);
        if (lane == 0) dq[(size_t) r * nb + b] = dd;  // raw f32 d: consumers round to f16 (kernels.h QFmt)
    }
}

void quantize_q8(hipStream_t s, const float * A32, const _Float16 * A16, int lda, int M, int K, int8_t * q, float * dq) {
    if (M <= 0) return;
    if (K % 32) throw std::runtime_error("quantize_q8: K % 32");
    const size_t blocks = (size_t) M * (K / 32);
    const int grid = (int) std::min<size_t>((blocks * 32 + 255) / 256, 65536);
    if (A32)
        OWK_LAUNCH(k_quantize_q8<float>, dim3(grid), dim3(256), 0, s, A32, lda, M, K, q, dq);
    else
        OWK_LAUNCH(k_quantize_q8<_Float16>, dim3(grid), dim3(256), 0, s, A16, lda, M, K, q, dq);
}

// Q8_0 rows of A as exact f16 integers for gemm_q16 (same rounding as k_quantize_q8) and the
// block scales block-major: dat[b * mpad + perm(r)] = (float) (f16) (amax / 127), perm = the row order
// k_gemm_q16 reads (within a 128-row tile: (t & 64) | (t & 15) << 2 | (t >> 4) & 3)
template <typename TA>
__global__ __launch_bounds__(256) void k_quantize_q8_f16(const TA * __restrict__ A, int lda, int M, int K,
                                                         _Float16 * __restrict__ q, float * __restrict__ dat, int mpad) {
    const int nb = K >> 5;
    const size_t total = (size_t) M * nb;
    const int lane = threadIdx.x & 31;
    for (size_t blk = ((size_t) blockIdx.x * blockDim.x + threadIdx.x) >> 5; blk < total;
         blk += ((size_t) gridDim.x * blockDim.x) >> 5) {
        const int r = (int) (blk / nb), b = (int) (blk - (size_t) r * nb);
        const float x = (float) A[(size_t) r * lda + b * 32 + lane];
        float am = fabsf(x);
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 32));
        const float dd = am / 127.f;
        const float id = am != 0.0f ? 127.f / am : 0.0f;
        q[(size_t) r * K + b * 32 + lane] = (_Float16) (float) (int) (int8_t) rintf(x * id);
        if (lane == 0) {
            const int t = r & 127;
            const int pr = (r & ~127) | (t & 64) | ((t & 15) << 2) | ((t >> 4) & 3);
            dat[(size_t) b * mpad + pr] = (float) (_Float16) dd;
        }
    }
}

// the same with 8 consecutive elements per lane (one 16/32-byte load, one 16-byte store; four lanes
// per block, amax over the quad): the per-element version moved 2.3 TB/s (f32 rows, 163 us for the
// 48000 x 1280 encoder operand, profiles/archive/r03g_q5_kernel_stats.txt)
template <typename TA>
__global__ __launch_bounds__(256) void k_quantize_q8_f16_v8(const TA * __restrict__ A, int lda, int M, int K,
                                                            _Float16 * __restrict__ q, float * __restrict__ dat, int mpad) {
    const int nb = K >> 5;
    const size_t total = (size_t) M * nb * 4;  // quads of 8 elements
    const int sub = threadIdx.x & 3;
    for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t) gridDim.x * blockDim.x) {
        const size_t blk = i >> 2;
        const int r = (int) (blk / nb), b = (int) (blk - (size_t) r * nb);
        const TA * src = A + (size_t) r * lda + b * 32 + sub * 8;
        float x[8];
        if constexpr (sizeof(TA) == 4) {
            const float4 u = ((const float4 *) src)[0], v = ((const float4 *) src)[1];
            x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w; x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
        } else {
            const half8 h = *(const half8 *) src;
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = (float) h[e];
        }
        float am = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(x[e]));
        am = fmaxf(am, __shfl_xor(am, 1, 64));
        am = fmaxf(am, __shfl_xor(am, 2, 64));
        const float dd = am / 127.f;
        const float id = am != 0.0f ? 127.f / am : 0.0f;
        half8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (_Float16) (float) (int) (int8_t) rintf(x[e] * id);
        *(half8 *) (q + (size_t) r * K + b * 32 + sub * 8) = o;
        if (sub == 0) {
            const int t = r & 127;
            const int pr = (r & ~127) | (t & 64) | ((t & 15) << 2) | ((t >> 4) & 3);
            dat[(size_t) b * mpad + pr] = (float) (_Float16) dd;
        }
    }
}

void quantize_q8_f16(hipStream_t s, const float * A32, const _Float16 * A16, int lda, int M, int K, _Float16 * q16,
                     float * dat, int mpad) {
    if (M <= 0) return;
    if (K % 32 || mpad < (M + 127) / 128 * 128) throw std::runtime_error("quantize_q8_f16: shape");
    const size_t blocks = (size_t) M * (K / 32);
    if (lda % 8 == 0 && ((uintptr_t) (A32 ? (const void *) A32 : (const void *) A16) & 31) == 0 && ((uintptr_t) q16 & 15) == 0) {
        const int grid = (int) std::min<size_t>((blocks * 4 + 255) / 256, 65536);
        if (A32)
            OWK_LAUNCH(k_quantize_q8_f16_v8<float>, dim3(grid), dim3(256), 0, s, A32, lda, M, K, q16, dat, mpad);
        else
            OWK_LAUNCH(k_quantize_q8_f16_v8<_Float16>, dim3(grid), dim3(256), 0, s, A16, lda, M, K, q16, dat, mpad);
        return;
    }
    const int grid = (int) std::min<size_t>((blocks * 32 + 255) / 256, 65536);
    if (A32)
        OWK_LAUNCH(k_quantize_q8_f16<float>, dim3(grid), dim3(256), 0, s, A32, lda, M, K, q16, dat, mpad);
    else
        OWK_LAUNCH(k_quantize_q8_f16<_Float16>, dim3(grid), dim3(256), 0, s, A16, lda, M, K, q16, dat, mpad);
}

// Q8_K rows for the K-quant formats (kernels.h quantize_q8k_f16; ref quantize_row_q8_K_ref,
// ggml-quants.c:2555-2592) in the virtual-block layout of kquant.h: one 256-thread block per
// (row, super-block). LAY 0: 8 blocks of q + one block [16 bsums | 16 zeros]; 1: 8 blocks of q;
// 2: 16 blocks [16 q | 16 zeros]. Every virtual block of the super-block carries d = 1 / iscale.
// Rounding: quantize_row_q8_K_ref's nearest_int(iscale * x) is `iscale * x + 12582912.f` and its bits,
// which gcc (-std=gnu11: -ffp-contract=fast, the reference's CMake default) contracts into ONE fused
// multiply-add -- the exact product rounded once. rmul[r] != 0 selects the x86 repack quantizer
// instead (ggml_quantize_mat_q8_K_4x8, ggml-cpu/arch/x86/repack.cpp:290-420: the rows of complete
// groups of 4 of a Q4_K / Q2_K matmul): the product rounded to f32 first, then to nearest even, and
// iscale = -127 / amax when some element equals +amax, else 127 / amax.
template <typename TA, int LAY>
__global__ __launch_bounds__(256) void k_quantize_q8k_f16(const TA * __restrict__ A, int lda, int M, int K,
                                                          _Float16 * __restrict__ q, float * __restrict__ dat,
                                                          int mpad, const uint8_t * __restrict__ rmul) {
    __shared__ uint32_t s_key[256];
    __shared__ float s_x[256];
    const int nsb = K >> 8;
    const int r = blockIdx.x / nsb, sb = blockIdx.x - r * nsb;
    if (r >= M) return;
    const int t = threadIdx.x;
    const float x = (float) A[(size_t) r * lda + sb * 256 + t];
    s_x[t] = x;
    // the FIRST element of largest |x| (the reference's scan keeps the earliest on ties): a tree
    // reduction of (|x| bits, index) pairs
    __shared__ int s_idx[256];
    s_key[t] = __float_as_uint(fabsf(x));
    s_idx[t] = t;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) {
            const uint32_t a = s_key[t], b = s_key[t + o];
            const int ia = s_idx[t], ib = s_idx[t + o];
            if (b > a || (b == a && ib < ia)) {
                s_key[t] = b;
                s_idx[t] = ib;
            }
        }
        __syncthreads();
    }
    const float amax = __uint_as_float(s_key[0]);
    const float mx = s_x[s_idx[0]];
    const bool mul_path = rmul && rmul[r];
    const bool pos_max = __syncthreads_or(x == amax);  // uniform: every thread reaches it
    int qv = 0;
    float d = 0.0f;
    if (amax != 0.0f) {
        if (mul_path) {
            const float iscale = pos_max ? -127.f / amax : 127.f / amax;
            float p = x * iscale;
            asm volatile("" : "+v"(p));  // the rounded product (no contraction into the rounding)
            qv = min(127, (int) rintf(p));
            d = 1.0f / iscale;
        } else {
            const float iscale = -127.f / mx;
            const float v = __builtin_fmaf(iscale, x, 12582912.f);
            qv = min(127, (__float_as_int(v) & 0x007fffff) - 0x00400000);
            d = 1.0f / iscale;
        }
    }
    // sums of 16 (one group of 16 lanes of a wave)
    int bs = qv;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) bs += __shfl_xor(bs, o, 16);
    const int kx = LAY == 0 ? (K >> 8) * 288 : LAY == 1 ? K : (K >> 8) * 512;
    _Float16 * out = q + (size_t) r * kx;
    const int g = t >> 4, e = t & 15;
    int kb0, nblk;
    if (LAY == 0) {
        out += sb * 288;
        out[t] = (_Float16) (float) qv;
        if (e == 0) out[256 + g] = (_Float16) (float) bs;
        if (t < 16) out[272 + t] = (_Float16) 0.0f;
        kb0 = sb * 9;
        nblk = 9;
    } else if (LAY == 1) {
        out += sb * 256;
        out[t] = (_Float16) (float) qv;
        kb0 = sb * 8;
        nblk = 8;
    } else {
        out += sb * 512;
        out[g * 32 + e] = (_Float16) (float) qv;
        out[g * 32 + 16 + e] = (_Float16) 0.0f;
        kb0 = sb * 16;
        nblk = 16;
    }
    if (t < nblk) {
        const int tt = r & 127;
        const int pr = (r & ~127) | (tt & 64) | ((tt & 15) << 2) | ((tt >> 4) & 3);
        dat[(size_t) (kb0 + t) * mpad + pr] = d;
    }
}

void quantize_q8k_f16(hipStream_t s, const float * A32, const _Float16 * A16, int lda, int M, int K, int fmt,
                      _Float16 * q16, float * dat, int mpad, const uint8_t * rmul) {
    if (M <= 0) return;
    if (K % 256 || !qf_is_k(fmt) || mpad < (M + 127) / 128 * 128) throw std::runtime_error("quantize_q8k_f16: shape");
    const int lay = fmt == QF_Q3_K ? 1 : fmt == QF_Q6_K ? 2 : 0;
    const size_t blocks = (size_t) M * (K / 256);
    if (blocks > 0x7fffffff) throw std::runtime_error("quantize_q8k_f16: too many rows");
#define OWK_Q8K(T, P, L) OWK_LAUNCH((k_quantize_q8k_f16<T, L>), dim3((unsigned) blocks), dim3(256), 0, s, P, lda, M, K, q16, dat, mpad, rmul)
    if (A32) {
        if (lay == 0) OWK_Q8K(float, A32, 0);
        else if (lay == 1) OWK_Q8K(float, A32, 1);
        else OWK_Q8K(float, A32, 2);
    } else {
        if (lay == 0) OWK_Q8K(_Float16, A16, 0);
        else if (lay == 1) OWK_Q8K(_Float16, A16, 1);
        else OWK_Q8K(_Float16, A16, 2);
    }
#undef OWK_Q8K
}

typedef int intx4 __attribute__((ext_vector_type(4)));

// 8 consecutive weights (group g = elements 8g..8g+7) of one block as int8, the B/A operand of
// mfma_i32_16x16x32_i8. 4/5-bit formats: nibbles of bytes 8(g&1)..+7 (low for g < 2, high
// otherwise), 5th bits qh >> 8g; the offset (Q5_0 -16, Q4_0 -8, none for the "_1" formats, whose
// minimum enters through m) by bytewise SWAR (v | 0x80) - off ^ 0x80. Q8_0: the bytes as stored.
template <int FMT>
__device__ __forceinline__ uint64_t unpack_group(uint64_t raw, uint32_t qh, int g) {
    if constexpr (FMT == QF_Q8_0) {
        return raw;
    } else {
        uint64_t v = (g < 2 ? raw : (raw >> 4)) & 0x0F0F0F0F0F0F0F0FULL;
        if constexpr (qf_has_qh(FMT)) {
            const uint32_t h8 = (qh >> (8 * g)) & 0xFFu;
#pragma unroll
            for (int e = 0; e < 8; ++e) v |= (uint64_t) ((h8 >> e) & 1u) << (8 * e + 4);
        }
        if constexpr (FMT == QF_Q5_0) v = ((v | 0x8080808080808080ULL) - 0x1010101010101010ULL) ^ 0x8080808080808080ULL;
        if constexpr (FMT == QF_Q4_0) v = ((v | 0x8080808080808080ULL) - 0x0808080808080808ULL) ^ 0x8080808080808080ULL;
        return v;
    }
}

// group g of K block kb of weight row n from the split arrays (runtime format)
__device__ __forceinline__ long wq_group(const Q5W & w, int n, int kb, int g, int K, int nb) {
    const size_t bi = (size_t) n * nb + kb;
    if (w.fmt == QF_Q8_0) return *(const long *) (w.qs + (size_t) n * K + kb * 32 + 8 * g);
    const uint64_t raw = *(const uint64_t *) (w.qs + bi * 16 + (g & 1) * 8);
    switch (w.fmt) {
        case QF_Q4_0: return (long) unpack_group<QF_Q4_0>(raw, 0u, g);
        case QF_Q4_1: return (long) unpack_group<QF_Q4_1>(raw, 0u, g);
        case QF_Q5_1: return (long) unpack_group<QF_Q5_1>(raw, w.qh[bi], g);
        default: return (long) unpack_group<QF_Q5_0>(raw, w.qh[bi], g);
    }
}

// the Q8_1 block sum term of a "_1" format: f16(d_f32 * sum(q)) (quantize_row_q8_1's y.s). The f32
// product is rounded first (the reference's two roundings): the empty asm keeps hipcc from folding
// multiply and conversion into one v_mad_mixlo_f16, whose single rounding of the exact product
// breaks f16 ties the other way (measured: 2 of 14 400 block sums)
__device__ __forceinline__ float q8_1_sum(float d_raw, int isum) {
    float p = d_raw * (float) isum;
    asm volatile("" : "+v"(p));
    return (float) (_Float16) p;
}

// Q5W block arrays -> exact f16 integers [N][K] and block scales [K/32][npad] (rows past N: 0)
__global__ void k_expand_q16(Q5W w, int N, int K, _Float16 * __restrict__ wi, float * __restrict__ dwt, int npad) {
    const int nb = K >> 5;
    const size_t total = (size_t) npad * nb * 4;  // (n, kb, group of 8)
    for (size_t p = (size_t) blockIdx.x * blockDim.x + threadIdx.x; p < total; p += (size_t) gridDim.x * blockDim.x) {
        const int g = (int) (p & 3);
        const size_t nk = p >> 2;
        const int n = (int) (nk / nb), kb = (int) (nk - (size_t) n * nb);
        if (n >= N) {
            if (g == 0) dwt[(size_t) kb * npad + n] = 0.0f;
            continue;
        }
        const long v = wq_group(w, n, kb, g, K, nb);
        half8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (_Float16) (float) (int8_t) (uint8_t) ((uint64_t) v >> (8 * e));
        *(half8 *) (wi + (size_t) n * K + kb * 32 + 8 * g) = h;
        if (g == 0) dwt[(size_t) kb * npad + n] = (float) w.d[(size_t) n * nb + kb];
    }
}

void quant_expand_f16(hipStream_t s, const Q5W & w, int N, int K, _Float16 * wi, float * dwt, int npad) {
    if (K % 32 || npad < N || qf_has_m(w.fmt)) throw std::runtime_error("quant_expand_f16: shape or format");
    OWK_LAUNCH(k_expand_q16, dim3(2048), dim3(256), 0, s, w, N, K, wi, dwt, npad);
}

// skinny: M <= 64 rows; one 16-column tile per block, 8 waves split the K blocks, partial
// tiles reduced through LDS in fixed wave order. "_1" formats: a second MFMA against an
// all-ones operand gives every row's block sum in the accumulator layout.
template <int MODE>
__global__ __launch_bounds__(512) void k_gemm_q5_skinny(int M, int N, int K, const int8_t * __restrict__ qa,
                                                        const float * __restrict__ da, Q5W w, EpiParams ep) {
    __shared__ floatx4 red[8][4][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = blockIdx.x * 16;
    const int MT = (M + 15) >> 4;
    const int nb = K >> 5;
    const int kb0 = (wave * nb) >> 3, kb1 = ((wave + 1) * nb) >> 3;
    const int g = lane >> 4;
    const int n = min(n0 + (lane & 15), N - 1);
    const bool has_m = qf_has_m(w.fmt);
    const long ones = 0x0101010101010101L;
    floatx4 acc[4], accm[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = accm[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int kb = kb0; kb < kb1; ++kb) {
        const long b = wq_group(w, n, kb, g, K, nb);
        const float dw = (float) w.d[(size_t) n * nb + kb];
        const float mw = has_m ? (float) w.m[(size_t) n * nb + kb] : 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i < MT) {
                const int ra = min(i * 16 + (lane & 15), M - 1);
                const long a = *(const long *) (qa + (size_t) ra * K + kb * 32 + 8 * g);
                const intx4 z = {0, 0, 0, 0};
                const intx4 iv = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, z, 0, 0, 0);
                intx4 is = z;
                if (has_m) is = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, ones, z, 0, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = min(i * 16 + 4 * g + e, M - 1);
                    const float dr = da[(size_t) r * nb + kb];
                    acc[i][e] += (float) iv[e] * ((float) (_Float16) dr * dw);
                    if (has_m) accm[i][e] += mw * q8_1_sum(dr, is[e]);
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][i][lane] = has_m ? acc[i] + accm[i] : acc[i];
    __syncthreads();
    if (tid < 256) {
        const int i = tid >> 6, ln = tid & 63;
        if (i < MT) {
            floatx4 sum = red[0][i][ln];
#pragma unroll
            for (int ww = 1; ww < 8; ++ww) sum += red[ww][i][ln];
            const int c = n0 + (ln & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = i * 16 + 4 * (ln >> 4) + e;
                if (r < M && c < N) epi_store<MODE>(ep, r, c, sum[e]);
            }
        }
    }
}

// decode rows (M <= 32): one 16-column tile per block, wave w takes J consecutive K blocks
// and issues ALL its weight (packed Q5_0) and activation (int8) loads before the first
// MFMA -- like k_gemm_rows, a launch is one memory round trip. The activation scales: in the QKV, MLP0,
// cross-Q and logits launches each lane loads its own outputs' scales directly (QKV 8.67 -> 7.67 us, MLP0
// 11.12 -> 9.61, cross-Q 7.83 -> 6.79, logits 61.8 -> 50.1); the split-K partial launches stage the whole
// A's (M x K/32 floats) in LDS behind a barrier, because direct loads there made every later layer's cross
// attention 48 -> 56 us on identical outputs (round 6, per-mode A/B: profiles/r06x_q5_direct_scales_by_mode.txt;
// the first all-launch trial profiles/r06i_q5_direct_scales_ab.txt). Every K block's exact integer dot
// (v_mfma_i32_16x16x32_i8) is scaled by d_a * d_w into the f32 accumulator; wave partial
// tiles are summed in fixed wave order. K up to GQ_MAXW * J * 32 (5120 at J = 10).
constexpr int GQ_MAXW = 16;
constexpr int GQ_JMAX = 10;  // K up to GQ_MAXW * GQ_JMAX * 32; short K uses 3 blocks per wave
constexpr int GQ_MAX_SCALES = 32 * 160;  // M x K/32 activation scales in LDS
// activation scales per thread: M * nb <= 32 * nb over blockDim = 64 * ceil(nb / J) threads
// -> at most 32 * J / 64 + 1

// NT column tiles per block (full epilogues, one k split): a wave's activation fragments and scales
// serve NT weight tiles (the MLP0 / logits launches, whose activation rows every block reads again);
// per output the same MFMA chain and the same wave order as NT = 1: bit-identical
template <int MODE, int MT, int FMT, int GQ_J, int NT = 1>  // FMT: QFmt; GQ_J K blocks per wave
__global__ __launch_bounds__(GQ_MAXW * 64) void k_gemm_q5_rows(int M, int N, int K, const int8_t * __restrict__ qa,
                                                               const float * __restrict__ da, Q5W w, EpiParams ep) {
    constexpr int GQ_DA_PER_THREAD = 32 * GQ_J / 64 + 1;
    constexpr bool HAS_M = qf_has_m(FMT), HAS_QH = qf_has_qh(FMT);
    constexpr int TB = qf_tile_bytes(FMT), QSB = qf_qs_bytes(FMT);
    // DIRECT: each lane loads its own activation scales with the operands (no LDS stage, no barrier before
    // the first MFMA) -- in the QKV, MLP0, cross-Q and logits launches (see above)
    constexpr bool DIRECT = MODE == EPI_QKV_DEC || MODE == EPI_GELU_F16 || MODE == EPI_F32 || MODE == EPI_F16;
    __shared__ floatx4 red[GQ_MAXW][NT][MT][64];
    __shared__ float sda[DIRECT ? 32 * 32 : GQ_MAX_SCALES];  // staged scales, or the GELU epilogue's f16 rows
    const int tid = threadIdx.x, lane = tid & 63, nw = blockDim.x >> 6;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: branch-free k range
    const int ntiles = (N + 15) >> 4, t0 = blockIdx.x * NT;
    const int nb = K >> 5;
    // split-K (gridDim.y > 1, EPI_PARTIAL): block y covers K blocks [kblo, kblo + nbl)
    const int kblo = blockIdx.y * nw * GQ_J;
    const int nbl = min(nw * GQ_J, nb - kblo);
    const int kb0 = kblo + wave * GQ_J;
    const int nj = max(0, min(GQ_J, nb - kb0));
    const int g = lane >> 4;
    const int c16 = lane & 15;
    uint64_t raw[NT][GQ_J];
    uint32_t qh[NT][GQ_J];
    _Float16 dw[NT][GQ_J], mw[NT][GQ_J];
    long a[MT][GQ_J];
    // the tile's blocks are contiguous records (qf_tile_bytes): coalesced loads. Blocks past this
    // wave's range load a valid record and a zero activation (adds exact zeros). Record format at
    // compile time: the load phase stays branch-free.
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint8_t * tb = w.tiled + (size_t) min(t0 + t, ntiles - 1) * nb * TB;
#pragma unroll
        for (int j = 0; j < GQ_J; ++j) {
            const int kb = min(kb0 + j, nb - 1);
            const uint8_t * rec = tb + (size_t) kb * TB;
            raw[t][j] = *(const uint64_t *) (rec + c16 * QSB + (QSB == 32 ? g * 8 : (g & 1) * 8));
            qh[t][j] = HAS_QH ? *(const uint32_t *) (rec + qf_tile_off_qh(FMT) + c16 * 4) : 0u;
            dw[t][j] = *(const _Float16 *) (rec + qf_tile_off_d(FMT) + c16 * 2);
            mw[t][j] = HAS_M ? *(const _Float16 *) (rec + qf_tile_off_m(FMT) + c16 * 2) : (_Float16) 0.0f;
        }
    }
#pragma unroll
    for (int j = 0; j < GQ_J; ++j) {
        const int kb = min(kb0 + j, nb - 1);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int ra = min(i * 16 + c16, M - 1);
            const long t = *(const long *) (qa + (size_t) ra * K + kb * 32 + 8 * g);
            a[i][j] = j < nj ? t : 0L;
        }
    }
    // activation scales of this block's K range (raw f32 d; at most GQ_DA_PER_THREAD per thread:
    // M <= 32, nbl <= nw * J) to LDS as [row][kb - kblo]; every load of the launch is issued before
    // the first wait (one round trip)
    if constexpr (!DIRECT) {
        float dv[GQ_DA_PER_THREAD];
#pragma unroll
        for (int u = 0; u < GQ_DA_PER_THREAD; ++u) {
            const int i = tid + u * blockDim.x;
            const int r = i / nbl;
            dv[u] = i < M * nbl ? da[(size_t) r * nb + kblo + (i - r * nbl)] : 0.0f;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < GQ_DA_PER_THREAD; ++u) {
            const int i = tid + u * blockDim.x;
            if (i < M * nbl) sda[i] = dv[u];
        }
        __syncthreads();
    }
    floatx4 acc[NT][MT], accm[NT][MT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[t][i] = accm[t][i] = floatx4{0.f, 0.f, 0.f, 0.f};
    const long ones = 0x0101010101010101L;
    // every activation scale of this wave first: unconditional LDS reads (in-array indices; a value past
    // the wave's K range is replaced by zero afterwards), so they go out together -- a guarded read per
    // scale made hipcc branch and wait on each one
    float drs[GQ_J][MT][4];
#pragma unroll
    for (int j = 0; j < GQ_J; ++j) {
        const int kb = min(kb0 + j, nb - 1);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = min(i * 16 + 4 * g + e, M - 1);
                drs[j][i][e] = DIRECT ? da[(size_t) r * nb + kb] : sda[min(r * nbl + (kb - kblo), GQ_MAX_SCALES - 1)];
            }
    }
#pragma unroll
    for (int j = 0; j < GQ_J; ++j) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const intx4 z = {0, 0, 0, 0};
            intx4 is = z;
            if constexpr (HAS_M) is = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[i][j], ones, z, 0, 0, 0);
            float dr[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) dr[e] = j < nj ? drs[j][i][e] : 0.0f;  // past the wave's range: zeros
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const uint64_t v = unpack_group<FMT>(raw[t][j], qh[t][j], g);
                const float dwf = (float) dw[t][j];
                const intx4 iv = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[i][j], (long) v, z, 0, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    acc[t][i][e] += (float) iv[e] * ((float) (_Float16) dr[e] * dwf);
                    if constexpr (HAS_M) accm[t][i][e] += (float) mw[t][j] * q8_1_sum(dr[e], is[e]);
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < MT; ++i) red[wave][t][i][lane] = HAS_M ? acc[t][i] + accm[t][i] : acc[t][i];
    __syncthreads();
    for (int o = tid; o < NT * MT * 256; o += blockDim.x) {
        const int t = o / (MT * 256), q = o - t * (MT * 256);
        const int r = q >> 4, cc = q & 15;
        const int i = r >> 4, rr = r & 15;
        const int ln = 16 * (rr >> 2) + cc, e = rr & 3;
        const float sum = wave_order_sum<GQ_MAXW>((const float *) &red[0][t][i][ln] + e, NT * MT * 64 * 4, nw);
        const int c = (t0 + t) * 16 + cc;
        if (r < M && c < N) {
            if constexpr (MODE == EPI_PARTIAL) {
                ep.out32[((size_t) blockIdx.y * M + r) * N + c] = sum;  // [ks][M][N] for resid_layernorm
            } else if constexpr (MODE == EPI_GELU_F16 && NT == 2) {
                const _Float16 h = (_Float16) gelu_lookup(ep.gelu_tab, sum + ep.bias[c]);
                ep.out16[(size_t) r * ep.ldo + c] = h;
                sda[r * 32 + t * 16 + cc] = (float) h;  // the scales are read: sda is free
            } else {
                epi_store<MODE>(ep, r, c, sum);
            }
        }
    }
    if constexpr (MODE == EPI_GELU_F16 && NT == 2) {
        // ep.q8: the block's 32 columns are one Q8_0 block of each row -- the next GEMM's operand rounded
        // here (k_quantize_q8's arithmetic on the same f16 values) instead of in a launch of its own
        if (ep.q8) {
            __syncthreads();
            for (int o = tid; o < M * 32; o += blockDim.x) {  // half-waves stay whole: M * 32, blockDim % 64 == 0
                const int r = o >> 5, cl = o & 31;
                const float x = sda[o];
                float am = fabsf(x);
#pragma unroll
                for (int sh = 16; sh > 0; sh >>= 1) am = fmaxf(am, __shfl_xor(am, sh, 32));
                const float id = am != 0.0f ? 127.f / am : 0.0f;
                ep.q8[(size_t) r * N + blockIdx.x * 32 + cl] = (int8_t) rintf(x * id);
                if (cl == 0) ep.q8d[(size_t) r * (N >> 5) + blockIdx.x] = am / 127.f;
            }
        }
    }
}

// tiles: 64 x 64 per block, 4 waves of 32 x 32; per 32-wide K block the int8 operands are
// staged in LDS (the Q5 weights expanded to int8 on the way), one MFMA per 16 x 16 tile,
// then the per-block scale d_a * d_w folds the integer dot into the f32 accumulator
template <int MODE>
__global__ __launch_bounds__(256) void k_gemm_q5_big(int M, int N, int K, const int8_t * __restrict__ qa,
                                                     const float * __restrict__ da, Q5W w, EpiParams ep) {
    __shared__ __attribute__((aligned(16))) int8_t sA[2][64][40], sB[2][64][40];
    __shared__ float sdA[2][64], sdB[2][64], sdS[2][64], sdM[2][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nbn = (N + 63) / 64;
    const int bm = blockIdx.x / nbn, bn = blockIdx.x - bm * nbn;
    const int m0 = bm * 64, n0 = bn * 64;
    const int nb = K >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    const int g = lane >> 4;
    floatx4 acc[2][2], accm[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = accm[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int srow = tid >> 2, sq = tid & 3;  // staging: row, 8-element group
    const int ra = min(m0 + srow, M - 1), rb = min(n0 + srow, N - 1);
    const bool has_m = qf_has_m(w.fmt);
    auto stage = [&](int buf, int kb) {
        const long av = *(const long *) (qa + (size_t) ra * K + kb * 32 + sq * 8);
        *(long *) &sA[buf][srow][sq * 8] = av;
        *(long *) &sB[buf][srow][sq * 8] = wq_group(w, rb, kb, sq, K, nb);
        // "_1" formats: the Q8_1 block sum of the activation row (its 4 groups sit in adjacent lanes)
        int isum = 0;
        if (has_m) {
#pragma unroll
            for (int e = 0; e < 8; ++e) isum += (int) (int8_t) (uint8_t) ((uint64_t) av >> (8 * e));
            isum += __shfl_xor(isum, 1, 64);
            isum += __shfl_xor(isum, 2, 64);
        }
        if (sq == 0) {
            const float dr = da[(size_t) ra * nb + kb];
            sdA[buf][srow] = (float) (_Float16) dr;
            sdB[buf][srow] = (float) w.d[(size_t) rb * nb + kb];
            if (has_m) {
                sdS[buf][srow] = q8_1_sum(dr, isum);
                sdM[buf][srow] = (float) w.m[(size_t) rb * nb + kb];
            }
        }
    };
    stage(0, 0);
    __syncthreads();
    for (int kb = 0; kb < nb; ++kb) {
        const int cur = kb & 1;
        if (kb + 1 < nb) stage(cur ^ 1, kb + 1);
        long a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            a[i] = *(const long *) &sA[cur][wm * 32 + i * 16 + (lane & 15)][8 * g];
            b[i] = *(const long *) &sB[cur][wn * 32 + i * 16 + (lane & 15)][8 * g];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const intx4 z = {0, 0, 0, 0};
                const intx4 iv = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[i], b[j], z, 0, 0, 0);
                const float dw = sdB[cur][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    acc[i][j][e] += (float) iv[e] * (sdA[cur][wm * 32 + i * 16 + 4 * g + e] * dw);
                if (has_m) {  // the m_w * s_a terms in their own sum (ggml's summs), added at the end
                    const float mw = sdM[cur][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
                    for (int e = 0; e < 4; ++e) accm[i][j][e] += mw * sdS[cur][wm * 32 + i * 16 + 4 * g + e];
                }
            }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = m0 + wm * 32 + i * 16 + 4 * g + e;
                if (r < M && c < N) epi_store<MODE>(ep, r, c, has_m ? acc[i][j][e] + accm[i][j][e] : acc[i][j][e]);
            }
        }
}

// k splits of a partial (EPI_PARTIAL) quantized decode-row GEMM: ~20-40 K blocks per split, 3 per
// wave (K 1280: 2 splits of 7 waves; K 5120: 4 splits of 14 waves)
int q5_partial_splits(int K) { return std::min(4, std::max(1, (K / 32 + 19) / 20)); }
size_t q5_partial_floats(int N, int K) { return (size_t) q5_partial_splits(K) * 32 * N; }

template <int MODE> struct LaunchQ5 {
    static void run(hipStream_t s, int M, int N, int K, const int8_t * qa, const float * da, const Q5W & w,
                    const EpiParams & ep) {
        const int nb = K / 32;
        if (MODE == EPI_PARTIAL && !(M <= 32 && w.tiled)) throw std::runtime_error("gemm_q5: EPI_PARTIAL needs the decode-row path");
        if (M <= 32 && w.tiled && nb <= GQ_MAXW * GQ_JMAX && M * nb <= GQ_MAX_SCALES) {
            // more, shorter waves when K allows: 3 K blocks per wave up to K = 1536; partial launches
            // (EPI_PARTIAL, summed by resid_layernorm) split K over gridDim.y (q5_partial_splits)
            const int KS = MODE == EPI_PARTIAL ? q5_partial_splits(K) : 1;
            const int J = (KS > 1 || nb <= GQ_MAXW * 3) ? 3 : GQ_JMAX;
            const int per = (nb + KS - 1) / KS;
            const int nw = (per + J - 1) / J;
            if (nw > GQ_MAXW) throw std::runtime_error("gemm_q5: decode-row plan");
            // full-epilogue launches with many column tiles take 2 per block (as LaunchRows: the activation
            // rows are read once per 2 tiles): MLP0 and the logits
            const int tiles = (N + 15) / 16;
            // ep.q8 (GELU rows): 2 tiles per block are one Q8_0 block per row, quantized in the epilogue
            const bool fq = MODE == EPI_GELU_F16 && ep.q8 && N % 32 == 0;
            const bool nt2 = MODE != EPI_PARTIAL && KS == 1 && (fq || (tiles + 1) / 2 >= 128);
            const dim3 grid(nt2 ? (tiles + 1) / 2 : tiles, KS), block(nw * 64);
#define OWK_Q_ROWS(MT_, F_, J_)                                                                                 \
    do {                                                                                                        \
        if (nt2) OWK_LAUNCH((k_gemm_q5_rows<MODE, MT_, F_, J_, 2>), grid, block, 0, s, M, N, K, qa, da, w, ep); \
        else OWK_LAUNCH((k_gemm_q5_rows<MODE, MT_, F_, J_, 1>), grid, block, 0, s, M, N, K, qa, da, w, ep);     \
    } while (0)
#define OWK_Q_ROWS_J(MT_, F_) do { if (J == 3) OWK_Q_ROWS(MT_, F_, 3); else OWK_Q_ROWS(MT_, F_, GQ_JMAX); } while (0)
#define OWK_Q_ROWS_F(MT_)                                                 \
    switch (w.fmt) {                                                      \
        case QF_Q8_0: OWK_Q_ROWS_J(MT_, QF_Q8_0); break;                  \
        case QF_Q4_0: OWK_Q_ROWS_J(MT_, QF_Q4_0); break;                  \
        case QF_Q4_1: OWK_Q_ROWS_J(MT_, QF_Q4_1); break;                  \
        case QF_Q5_1: OWK_Q_ROWS_J(MT_, QF_Q5_1); break;                  \
        default: OWK_Q_ROWS_J(MT_, QF_Q5_0); break;                       \
    }
            if (M <= 16) OWK_Q_ROWS_F(1) else OWK_Q_ROWS_F(2)
#undef OWK_Q_ROWS_F
#undef OWK_Q_ROWS_J
#undef OWK_Q_ROWS
            if (ep.q8 && !fq) quantize_q8(s, nullptr, ep.out16, ep.ldo, M, N, ep.q8, ep.q8d);
            return;
        }
        if (M <= 64)
            OWK_LAUNCH(k_gemm_q5_skinny<MODE>, dim3((N + 15) / 16), dim3(512), 0, s, M, N, K, qa, da, w, ep);
        else
            OWK_LAUNCH(k_gemm_q5_big<MODE>, dim3(((M + 63) / 64) * ((N + 63) / 64)), dim3(256), 0, s, M, N, K,
                               qa, da, w, ep);
        // Q8_0 rows of an f16 output requested by the caller: a launch of their own on these paths
        if (ep.q8) quantize_q8(s, nullptr, ep.out16, ep.ldo, M, N, ep.q8, ep.q8d);
    }
};

int qf_block_bytes(int f) {
    switch (f) {
        case QF_Q5_0: return 22;  // block_q5_0: d, qh[4], qs[16]
        case QF_Q8_0: return 34;  // block_q8_0: d, qs[32]
        case QF_Q4_0: return 18;  // block_q4_0: d, qs[16]
        case QF_Q4_1: return 20;  // block_q4_1: d, m, qs[16]
        case QF_Q5_1: return 24;  // block_q5_1: d, m, qh[4], qs[16]
    }
    throw std::runtime_error("quant: bad format");
}
int qf_ggml_type(int f) {
    static const int t[] = {6, 8, 2, 3, 7};
    if (f < 0 || f > QF_Q5_1) throw std::runtime_error("quant: bad format");
    return t[f];
}

size_t quant_tiled_bytes(int fmt, int N, int K) { return (size_t) ((N + 15) / 16) * (K / 32) * qf_tile_bytes(fmt); }

void quant_split_host(int fmt, const uint8_t * blocks, int N, int K, uint8_t * qs, uint32_t * qh, uint16_t * d,
                      uint16_t * m) {
    const int nb = K / 32, bb = qf_block_bytes(fmt), qsb = qf_qs_bytes(fmt);
    for (size_t i = 0; i < (size_t) N * nb; ++i) {
        const uint8_t * b = blocks + i * bb;
        int o = 0;
        memcpy(&d[i], b, 2);
        o += 2;
        if (qf_has_m(fmt)) {
            memcpy(&m[i], b + o, 2);
            o += 2;
        }
        if (qf_has_qh(fmt)) {
            memcpy(&qh[i], b + o, 4);
            o += 4;
        }
        memcpy(qs + i * qsb, b + o, qsb);
    }
}

void quant_tile_host(int fmt, const uint8_t * qs, const uint32_t * qh, const uint16_t * d, const uint16_t * m, int N,
                     int K, uint8_t * out) {
    const int nb = K / 32, nt = (N + 15) / 16, tb = qf_tile_bytes(fmt), qsb = qf_qs_bytes(fmt);
    memset(out, 0, quant_tiled_bytes(fmt, N, K));
    for (int t = 0; t < nt; ++t)
        for (int kb = 0; kb < nb; ++kb) {
            uint8_t * o = out + ((size_t) t * nb + kb) * tb;
            for (int c = 0; c < 16; ++c) {
                const int n = t * 16 + c;
                if (n >= N) break;
                const size_t bi = (size_t) n * nb + kb;
                memcpy(o + c * qsb, qs + bi * qsb, qsb);
                if (qf_has_qh(fmt)) memcpy(o + qf_tile_off_qh(fmt) + c * 4, &qh[bi], 4);
                memcpy(o + qf_tile_off_d(fmt) + c * 2, &d[bi], 2);
                if (qf_has_m(fmt)) memcpy(o + qf_tile_off_m(fmt) + c * 2, &m[bi], 2);
            }
        }
}

static void check_shape(int M, int N, int K, int lda, int ldw, int kmul) {
    if (M <= 0 || N <= 0 || K <= 0 || K % kmul != 0 || lda < K || ldw < K || (lda % 8) || (ldw % 8))
        throw std::runtime_error("gemm: unsupported shape M=" + std::to_string(M) + " N=" + std::to_string(N) +
                                 " K=" + std::to_string(K));
}

// large GEMMs (the batched encoder, cross-KV, conv) take the 256x256 ring kernel; the rest
// (small models, SortFormer chunks) the 128x128 tile. OWK_GEMM256=0 forces the 128x128 path.
int gemm_set_256(int on) {
    const int prev = t_gemm256;
    t_gemm256 = on;
    return prev;
}
static bool use_256(int M, int N, int K) {
    const int m = gemm256_mode();
    return m && m != GEMM_MID_FORCED && m != GEMM_MID32_FORCED && M >= 2048 && N >= 1024 && K % G8_K == 0;
}
// the 64x64 ring tile where the 128x128 grid would not give every CU a block (the override 0 keeps
// the 128x128 tile; the overrides GEMM_MID_FORCED / GEMM_MID32_FORCED take a ring tile always)
static bool use_mid(int M, int N) {
    const int m = gemm256_mode();
    if (m == 0) return false;
    if (m == GEMM_MID_FORCED || m == GEMM_MID32_FORCED) return true;
    return ((M + GB_M - 1) / GB_M) * ((N + GB_N - 1) / GB_N) < 256;
}
// tile edge of the ring kernel: 32 where the 64x64 grid would still leave CUs idle (SortFormer chunk
// shapes at M = 413, tests/test_gpu_kernels.py::test_gemm_mid_speed: 32x32 4.6-15.7 us against 64x64
// 6.2-21.7 us, N = 2048 included, whose 64x64 grid is 224 blocks; profiles/archive/r03h_gemm_mid_speed.txt)
static int mid_tile(int M, int N) {
    const int m = gemm256_mode();
    if (m == GEMM_MID_FORCED || m == GEMM_MID32_FORCED) return m == GEMM_MID32_FORCED ? 32 : 64;
    return ((M + 63) / 64) * ((N + 63) / 64) < 256 ? 32 : 64;
}

void gemm_f16(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W, int ldw,
              const EpiParams & ep) {
    check_shape(M, N, K, lda, ldw, GB_K);
    if (use_256(M, N, K)) dispatch_mode<Launch256>(mode, s, M, N, K, A, lda, W, ldw, ep);
    else if (use_mid(M, N)) dispatch_mode<LaunchMid>(mode, s, M, N, K, A, lda, W, ldw, ep);
    else dispatch_mode<LaunchBig>(mode, s, M, N, K, A, lda, W, ldw, ep);
}

void gemm_f16_skinny(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda, const _Float16 * W,
                     int ldw, const EpiParams & ep) {
    check_shape(M, N, K, lda, ldw, 32);
    if (M > 64) throw std::runtime_error("gemm_skinny: M > 64");
    dispatch_mode<LaunchSkinny>(mode, s, M, N, K, A, lda, W, ldw, ep);
}

void gemm_q5(hipStream_t s, int mode, int M, int N, int K, const int8_t * qa, const float * da, const Q5W & w,
             const EpiParams & ep) {
    if (M <= 0 || N <= 0 || K <= 0 || K % 32) throw std::runtime_error("gemm_q5: unsupported shape");
    if (!w) throw std::runtime_error("gemm_q5: no Q5_0 weights");
    if (mode == EPI_PARTIAL) {
        if (!ep.out32) throw std::runtime_error("gemm_q5: EPI_PARTIAL needs the partial workspace in out32");
        LaunchQ5<EPI_PARTIAL>::run(s, M, N, K, qa, da, w, ep);
        return;
    }
    dispatch_mode<LaunchQ5>(mode, s, M, N, K, qa, da, w, ep);
}

bool gemm_q16_applies(const Q5W & w, int M, int N, int K) {
    if (qf_is_k(w.fmt)) return w.wi && w.dwt && K % G2_K == 0;  // K-quants: every shape, K = the virtual K
    return w.wi && w.dwt && use_256(M, N, K) && !qf_has_m(w.fmt);
}

void gemm_q16(hipStream_t s, int mode, int M, int N, int K, const _Float16 * q16, const float * dat, int mpad,
              const Q5W & w, const EpiParams & ep) {
    if (!gemm_q16_applies(w, M, N, K) || mpad < (M + GQ16_M - 1) / GQ16_M * GQ16_M || w.npad < (N + G2_N - 1) / G2_N * G2_N)
        throw std::runtime_error("gemm_q16: unsupported shape");
    check_shape(M, N, K, K, K, G2_K);
    dispatch_mode<Launch256Q>(mode, s, M, N, K, q16, dat, mpad, w, ep);
}

size_t gemm_ws_floats(int N, int K) {
    const RowsPlan p = rows_plan(K, false);
    return p.KS > 1 ? (size_t) p.KS * ((N + 15) / 16) * 2 * 64 * 4 : 0;
}
size_t gemm_partial_floats(int N, int K) { return (size_t) rows_plan(K, true).KS * ((N + 15) / 16) * 2 * 64 * 4; }
int gemm_partial_splits(int K) { return rows_plan(K, true).KS; }

bool gemm_rows_exact_applies(int M, int d) {
    if (M < 1 || M > LNX_MAX_ROWS || d % 32 || d / 4 > LNX_MAX4) return false;
    const RowsPlan pf = rows_plan(d, false), pr = rows_plan(4 * d, true), po = rows_plan(d, true);
    return pf.KS == 1 && (pf.J == 2 || pf.J == 4) && pr.KS <= 3 && po.KS <= 3;
}

void gemm_rows_res(hipStream_t s, int M, int N, int K, const _Float16 * A, const _Float16 * Wt, const float * bias,
                   float * x) {
    const RowsPlan p = rows_plan(K, true);
    if (M < 1 || M > 16 || N % 16 || K % 32 || p.KS > 3 || !Wt || !A || !bias || !x)
        throw std::runtime_error("gemm_rows_res: unsupported shape");
    const dim3 g((N + 15) / 16);
#define OWK_RES_GO(J_, KS_) OWK_LAUNCH((k_gemm_rows_res<J_, KS_>), g, dim3(p.nw * 64), 0, s, M, N, K, A, Wt, bias, x)
    if (p.J == 2) {
        if (p.KS == 1) OWK_RES_GO(2, 1); else if (p.KS == 2) OWK_RES_GO(2, 2); else OWK_RES_GO(2, 3);
    } else {
        if (p.KS == 1) OWK_RES_GO(4, 1); else if (p.KS == 2) OWK_RES_GO(4, 2); else OWK_RES_GO(4, 3);
    }
#undef OWK_RES_GO
}

template <int MODE> static void launch_lnx(hipStream_t s, int order, int M, int N, int K, const float * x, const float * lnw,
                                           const float * lnb, float eps, const _Float16 * Wt, const EpiParams & ep) {
    const RowsPlan p = rows_plan(K, false);
    const int tiles = (N + 15) / 16;
    // column tiles per block as the split chain's full-epilogue dispatch (LaunchRows): no effect on bits
    const int nt = (p.J == 4 || p.J == 2) && (tiles + 1) / 2 >= 128 ? 2 : 1;
    const dim3 g((tiles + nt - 1) / nt);
#define OWK_LNX_GO(J_, NT_, O_) \
    OWK_LAUNCH((k_gemm_rows_lnx<MODE, J_, NT_, O_>), g, dim3(p.nw * 64), 0, s, M, N, K, x, lnw, lnb, eps, Wt, ep)
    if (p.J == 4) {
        if (nt == 2) { if (order) OWK_LNX_GO(4, 2, 1); else OWK_LNX_GO(4, 2, 0); }
        else { if (order) OWK_LNX_GO(4, 1, 1); else OWK_LNX_GO(4, 1, 0); }
    } else {
        if (nt == 2) { if (order) OWK_LNX_GO(2, 2, 1); else OWK_LNX_GO(2, 2, 0); }
        else { if (order) OWK_LNX_GO(2, 1, 1); else OWK_LNX_GO(2, 1, 0); }
    }
#undef OWK_LNX_GO
}

void gemm_rows_lnx(hipStream_t s, int mode, int order, int M, int N, int K, const float * x, const float * lnw,
                   const float * lnb, float eps, const _Float16 * Wt, const EpiParams & ep) {
    if (!gemm_rows_exact_applies(M, K) || N % 16 || !Wt || !x || !lnw || !lnb) throw std::runtime_error("gemm_rows_lnx: unsupported shape");
    switch (mode) {
        case EPI_F16: launch_lnx<EPI_F16>(s, order, M, N, K, x, lnw, lnb, eps, Wt, ep); break;
        case EPI_GELU_F16: launch_lnx<EPI_GELU_F16>(s, order, M, N, K, x, lnw, lnb, eps, Wt, ep); break;
        case EPI_QKV_DEC: launch_lnx<EPI_QKV_DEC>(s, order, M, N, K, x, lnw, lnb, eps, Wt, ep); break;
        default: throw std::runtime_error("gemm_rows_lnx: epilogue not instantiated");
    }
}

bool gemm_rows_ln_applies(int M, int N, int K) {
    return M >= 1 && M <= 32 && K % 32 == 0 && K % 8 == 0 && N % 16 == 0 && K / 32 <= GRL_MAXW * 4;
}

void gemm_rows_ln(hipStream_t s, int mode, int M, int N, int K, const float * x, const float * lnw, const float * lnb,
                  float eps, const _Float16 * Wt, const EpiParams & ep, bool debug_no_stats) {
    if (!gemm_rows_ln_applies(M, N, K) || !Wt || !x || !lnw || !lnb) throw std::runtime_error("gemm_rows_ln: unsupported shape");
    if (debug_no_stats) {  // timing experiments only: the LayerNorm statistics skipped (mean 0, scale 1)
        switch (mode) {
            case EPI_F16: LaunchRowsLn<EPI_F16, false>::run(s, M, N, K, x, lnw, lnb, eps, Wt, ep); return;
            case EPI_GELU_F16: LaunchRowsLn<EPI_GELU_F16, false>::run(s, M, N, K, x, lnw, lnb, eps, Wt, ep); return;
            case EPI_QKV_DEC: LaunchRowsLn<EPI_QKV_DEC, false>::run(s, M, N, K, x, lnw, lnb, eps, Wt, ep); return;
            default: throw std::runtime_error("gemm_rows_ln: epilogue not instantiated");
        }
    }
    switch (mode) {
        case EPI_F16: LaunchRowsLn<EPI_F16>::run(s, M, N, K, x, lnw, lnb, eps, Wt, ep); break;
        case EPI_GELU_F16: LaunchRowsLn<EPI_GELU_F16>::run(s, M, N, K, x, lnw, lnb, eps, Wt, ep); break;
        case EPI_QKV_DEC: LaunchRowsLn<EPI_QKV_DEC>::run(s, M, N, K, x, lnw, lnb, eps, Wt, ep); break;
        default: throw std::runtime_error("gemm_rows_ln: epilogue not instantiated");
    }
}

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
