// Persistent decode chain for passes of <= CH_MAXR rows (kernels.h ChainArgs), gfx950.
//
// A decoder layer of a few-row pass (configs[4]'s one-row greedy steps, a single clip's beam search) is
// ~15 launches of 2-8 us that each move 0.1-13 MB: latency, not bytes (profiles/r05a_c4seq_graph_kernel_stats.txt:
// 75 us per layer for 46 MB of weights). Between two attention launches the layer is a chain of decode-row
// GEMMs and residual + LayerNorm steps (whisper.cpp:2458-2836 per layer):
//   A: attn.out (split-K partials) -> residual + cross_attn_ln -> cross_attn.query
//   B: cross_attn.out (partials) -> residual + mlp_ln -> mlp.0 + GELU -> mlp.2 (partials)
//      -> residual + the next layer's attn_ln -> its fused Q/K/V (K/V into the self-attention cells)
// Each chain is ONE launch of one 16-wave block per item (a 16-column tile group and k split of a stage):
//   * a block streams its item's weight tiles into LDS (global_load_lds, non-temporal) BEFORE it waits for
//     the previous stage: the one thing a kernel boundary cannot do (profiles/archive/r03s_lab_prefetch.txt);
//   * stage hand-off (cdna_hip_programming.md Guideline 16, R1; MI355X_MICROARCH.md visibility table,
//     first row): every handed-off value is stored write-through (agent-scope atomic stores) and drained
//     (vmcnt(0)) before one lane adds the block's arrival to its XCD shard of the stage's count; a consumer
//     block polls the 8 shards from one wave, joins a block barrier, and reads handed-off values with
//     agent-scope (L1-bypassing) loads only;
//   * a stage with a LayerNorm prologue recomputes, in every block, the residual row x + (split-K partials
//     in k order + bias) and its LayerNorm exactly as k_resid_layernorm (rln_row.h) does -- block 0 stores
//     the new residual row -- and feeds its MFMAs from the LayerNorm rows in LDS;
//   * per output the same MFMA chain (wave w: k-steps (ks * nw + w) * J ..), the same wave order of the
//     partial sums and the same epilogue as k_gemm_rows: bit-identical to the launch chain it replaces
//     (tests/test_gpu_chain.py).
// Every wait is bounded (a give-up sets the host-mapped error word the engine checks after each pass).
// Residency: a consumer waits on every item of the previous stage, so all blocks of the launch must be
// resident together: grid <= CUs, one 1024-thread block per CU, and at most one chain launch in flight
// per device (the engine takes a process-wide per-device lock for the whole whisper_full call).
// The arrival counts are left at zero by the last block to exit (no memset node before each launch).
//
// Measured (tools/chain_trace.py realtime stamps, profiles/r05_chain_stamps.txt; large-v3 one-row steps):
// chain A spans 9.4 us and chain B 24.2 us from first block entry to last publish (+ ~3 us launch ramp each);
// a stage with a LayerNorm prologue costs ~4.4 us of hand-off (drain 0.8, arrival + poll 2.0-2.4, 16-B
// write-through loads + LayerNorm 2.8) -- the allgather row of MI355X_MICROARCH.md's price list -- against a
// kernel boundary plus the same work as launches in a graph replay. configs[4] sequential (2 min) ran at
// RTF 16.98 with the chain and 18.10 without, so the engine leaves it off (dec_chain_mode() == 0) and the
// tests keep it bit-identical. Every stage is at its hand-off price; what is left is fewer seams (the
// attention kernels inside the same launch), not cheaper ones.
#include "kernels.h"
#include "gemm_epi.h"
#include "rln_row.h"

#include <algorithm>

namespace owk {

constexpr int CH_THREADS = 1024;        // 16 waves: every decode-row plan has nw <= GR_MAXW = 16
constexpr int CH_LDA = CH_MAXD + 8;     // LDS row stride of the LayerNorm rows (halves; 16 B apart across rows)
constexpr int CH_LINE = 32;             // words per counter (one 128-B line each)
constexpr unsigned CH_SPIN_MAX = 1u << 18;  // polls before a wait gives up (~0.3 s)
constexpr int CH_WSLOTS = 80;           // 1-KB weight slots (nw * tpi * J per item: mlp.0 10 * 2 * 4)
constexpr int CH_KSMAX = 3;             // k splits a LayerNorm prologue adds (decode-row plans: <= 3)
typedef __attribute__((address_space(3))) void * lds_ptr_t;

// counter of stage s, XCD shard x: sync[(s * 8 + x) * CH_LINE]; exit count: sync[CH_MAXST * 8 * CH_LINE]
size_t dec_chain_sync_words() { return (size_t) (CH_MAXST * 8 + 1) * CH_LINE; }

__device__ __forceinline__ float ld_ag(const float * p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned ld_ag(const unsigned * p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag(float * p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_ag(unsigned * p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte write-through (sc1) buffer accesses of handed-off rows: base = a kernel argument (wave-uniform),
// byte offsets < 2 GB (the chain's row buffers)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int CH_SC1 = 16;  // cache-policy bits of an sc1 buffer access
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ch_rsrc(const void * p) {
    return __builtin_amdgcn_make_buffer_rsrc((void *) p, (short) 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ u32x4 ld16_sc1(const void * base, size_t byte_off) {
    return __builtin_amdgcn_raw_buffer_load_b128(ch_rsrc(base), (int) byte_off, 0, CH_SC1);
}
__device__ __forceinline__ void st16_sc1(void * base, size_t byte_off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, ch_rsrc(base), (int) byte_off, 0, CH_SC1);
}

__device__ __forceinline__ int chain_items(const ChainStage & st) {
    if (st.N <= 0) return 1;
    const int tiles = (st.N + 15) >> 4;
    return ((tiles + st.tpi - 1) / st.tpi) * st.KS;
}

// one wave polls the 8 shards of stage s's arrival count until `need` items have published; the block
// barrier after it orders every wave's loads behind the matched poll
__device__ __forceinline__ void chain_wait(unsigned * sync, int s, unsigned need, unsigned * err) {
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        for (unsigned spins = 0;; ++spins) {
            unsigned v = lane < 8 ? ld_ag(sync + (s * 8 + lane) * CH_LINE) : 0u;
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            if (__shfl(v, 0) >= need) break;
            if (spins >= CH_SPIN_MAX) {
                if (lane == 0 && err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

// sum over the 4 waves of row group g (rln_row.h block_sum4_d for the group's 256 threads)
__device__ __forceinline__ double group_sum4_d(double v, double (*red)[4]) {
    v = wave_sum_d(v);
    const int g = threadIdx.x >> 8, wl = (threadIdx.x >> 6) & 3;
    if ((threadIdx.x & 63) == 0) red[g][wl] = v;
    __syncthreads();
    const double t = (red[g][0] + red[g][1]) + (red[g][2] + red[g][3]);
    __syncthreads();
    return t;
}

// the LayerNorm prologue: rows in groups of 4 (256 threads each), every row exactly resid_ln_row's
// arithmetic (rln_row.h); block 0 (writer) stores the new residual rows write-through
__device__ __forceinline__ void chain_ln(const ChainStage & st, int M, int N, float eps, bool writer, _Float16 * sA,
                                         double (*red)[4]) {
    const int g = threadIdx.x >> 8, t = threadIdx.x & 255;
    const int n4 = N >> 2, KS = st.ln_ks;
    const float4 z4 = float4{0.f, 0.f, 0.f, 0.f};
    const float4 * b4p = (const float4 *) st.ln_bias;
    const float4 * w4p = (const float4 *) (st.lnw ? st.lnw : st.ln_bias);
    const float4 * lb4p = (const float4 *) (st.lnw ? st.lnb : st.ln_bias);
    for (int r0 = 0; r0 < M; r0 += 4) {
        const int row = r0 + g;
        const bool act = row < M;
        const int rr = min(row, M - 1);
        float4 pv[RL_V4][CH_KSMAX], bv[RL_V4], rv[RL_V4], wv[RL_V4], lbv[RL_V4];
        // one 16-byte write-through load per split and residual float4 (the groups past the last row load
        // nothing: their values are computed and discarded)
#pragma unroll
        for (int j = 0; j < RL_V4; ++j) {
            const int i = min(t + 256 * j, n4 - 1);
#pragma unroll
            for (int ks = 0; ks < CH_KSMAX; ++ks)
                pv[j][ks] = act ? __builtin_bit_cast(float4, ld16_sc1(st.ln_part, (((size_t) min(ks, KS - 1) * M + rr) * n4 + i) * 16))
                                : z4;
            bv[j] = b4p[i];
            rv[j] = act ? __builtin_bit_cast(float4, ld16_sc1(st.x_in, ((size_t) rr * n4 + i) * 16)) : z4;
            wv[j] = w4p[i];
            lbv[j] = lb4p[i];
        }
        float4 xv[RL_V4];
#pragma unroll
        for (int j = 0; j < RL_V4; ++j) {
            const int i = t + 256 * j;
            float4 r = z4;
            if (i < n4) {
                float4 a = pv[j][0];
#pragma unroll
                for (int ks = 1; ks < CH_KSMAX; ++ks) {
                    if (ks < KS) {
                        const float4 q = pv[j][ks];
                        a.x += q.x; a.y += q.y; a.z += q.z; a.w += q.w;
                    }
                }
                const float4 bb = bv[j], res = rv[j];
                r.x = res.x + (a.x + bb.x);
                r.y = res.y + (a.y + bb.y);
                r.z = res.z + (a.z + bb.z);
                r.w = res.w + (a.w + bb.w);
                if (writer && act) st16_sc1(st.x_out, ((size_t) rr * n4 + i) * 16, __builtin_bit_cast(u32x4, r));
            }
            xv[j] = r;
        }
        if (!st.lnw) continue;
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < RL_V4; ++j)
            s += ((double) xv[j].x + (double) xv[j].y) + ((double) xv[j].z + (double) xv[j].w);
        s = group_sum4_d(s, red);
        const float mean = (float) s / (float) N;
        double v = 0.0;
#pragma unroll
        for (int j = 0; j < RL_V4; ++j) {
            if (t + 256 * j < n4) {
                const float tx = xv[j].x - mean, ty = xv[j].y - mean, tz = xv[j].z - mean, tw = xv[j].w - mean;
                v += ((double) (tx * tx) + (double) (ty * ty)) + ((double) (tz * tz) + (double) (tw * tw));
            }
        }
        v = group_sum4_d(v, red);
        const float var = (float) (v / (double) N);
        const float scale = 1.0f / sqrtf(var + eps);
#pragma unroll
        for (int j = 0; j < RL_V4; ++j) {
            const int i = t + 256 * j;
            if (act && i < n4) {
                const float4 ww = wv[j], bb = lbv[j];
                float4 y;
                y.x = (xv[j].x - mean) * scale * ww.x + bb.x;
                y.y = (xv[j].y - mean) * scale * ww.y + bb.y;
                y.z = (xv[j].z - mean) * scale * ww.z + bb.z;
                y.w = (xv[j].w - mean) * scale * ww.w + bb.w;
                half4 h;
                h[0] = (_Float16) y.x;
                h[1] = (_Float16) y.y;
                h[2] = (_Float16) y.z;
                h[3] = (_Float16) y.w;
                *(half4 *) (sA + (size_t) row * CH_LDA + 4 * i) = h;
            }
        }
    }
    __syncthreads();
}

// stage S of the launch (S a constant after unrolling, so the stage's fields are read from the kernel
// arguments directly)
__device__ __forceinline__ void chain_stage(const ChainArgs & a, const ChainStage & st, int s, _Float16 * sA, char * sW,
                                            floatx4 (*red)[CH_TPI][64], double (*lnred)[4]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int M = a.M;
    const int items = chain_items(st);
    const int item = blockIdx.x;
    if (item >= items) return;  // block-uniform
    const bool gemm = st.N > 0;
    const int tiles = (st.N + 15) >> 4;
    const int ntg = gemm ? (tiles + st.tpi - 1) / st.tpi : 1;
    const int tg = item % ntg, ks = item / ntg;
    const int nsteps = st.K >> 5;
    const int ks0 = (ks * st.nw + wave) * st.J;
    const int nj = max(0, min(st.J, nsteps - ks0));
    const bool cw = gemm && wave < st.nw;  // a computing wave
    const half8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long * ts = a.ts ? a.ts + ((size_t) blockIdx.x * CH_MAXST + s) * CH_TS : nullptr;
    auto stamp = [&](int k) {
        if (ts && tid == 0) ts[k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);

    // 1. this item's weight tiles, streamed into LDS (global_load_lds, non-temporal: read once per pass)
    // while the block waits for the previous stage; wave w's tiles land in its own slots
    char * wslot = sW + (size_t) wave * st.tpi * st.J * 1024;
    if (cw) {
#pragma unroll
        for (int t = 0; t < CH_TPI; ++t) {
            if (t >= st.tpi) break;
            const int tile = min(tg * st.tpi + t, tiles - 1);
            const _Float16 * wp = st.Wt + (size_t) tile * nsteps * 512 + lane * 8;
#pragma unroll
            for (int j = 0; j < CH_J; ++j) {
                if (j >= st.J) break;
                __builtin_amdgcn_global_load_lds((const void *) (wp + (size_t) min(ks0 + j, nsteps - 1) * 512),
                                                 (lds_ptr_t) (wslot + (t * st.J + j) * 1024), 16, 0, 2);
            }
        }
    }
    stamp(1);
    // 2. the previous stage's outputs
    if (s > 0) chain_wait(a.sync, s - 1, (unsigned) chain_items(a.st[s - 1]), a.err);
    stamp(2);

    // 3. the A operand: LayerNorm rows in LDS, or rows from memory
    half8 av[CH_J];
    if (st.ln_part) {
        chain_ln(st, M, a.d, a.eps, blockIdx.x == 0, sA, lnred);
        if (cw) {
            const _Float16 * ap = sA + (size_t) min(lane & 15, M - 1) * CH_LDA + 8 * (lane >> 4);
#pragma unroll
            for (int j = 0; j < CH_J; ++j) av[j] = j < nj ? *(const half8 *) (ap + (ks0 + j) * 32) : z8;
        }
    } else if (cw) {
        const _Float16 * ap = st.A + (size_t) min(lane & 15, M - 1) * st.K + 8 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < CH_J; ++j) {
            const _Float16 * p = ap + (size_t) min(ks0 + j, nsteps - 1) * 32;
            const half8 v = st.a_handoff ? __builtin_bit_cast(half8, ld16_sc1(st.A, (size_t) (p - st.A) * 2)) : *(const half8 *) p;
            av[j] = j < nj ? v : z8;
        }
    }

    stamp(3);
    if (gemm) {
        // 4. k_gemm_rows's per-wave MFMA chain over its k-steps, partials to LDS
        if (cw) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight tiles have landed
#pragma unroll
            for (int t = 0; t < CH_TPI; ++t) {
                if (t >= st.tpi) break;
                floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < CH_J; ++j) {
                    if (j >= st.J) break;
                    const half8 w = *(const half8 *) (wslot + (t * st.J + j) * 1024 + lane * 16);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[j], j < nj ? w : z8, acc, 0, 0, 0);
                }
                red[wave][t][lane] = acc;
            }
        }
        __syncthreads();
        stamp(4);
        // 5. the epilogue: one output (row r, column c) per thread, wave partials in wave order
        if (tid < st.tpi * 256) {
            const int t = tid >> 8, q = tid & 255;
            const int r = q >> 4, cc = q & 15;
            const int ln = 16 * (r >> 2) + cc, e = r & 3;
            const float sum = wave_order_sum<16>((const float *) &red[0][t][ln] + e, CH_TPI * 64 * 4, st.nw);
            const int c = (tg * st.tpi + t) * 16 + cc;
            const bool ok = r < M && c < st.N;
            if (st.mode == EPI_PARTIAL) {
                if (ok) st_ag(st.part + ((size_t) ks * M + r) * st.N + c, sum);
            } else if (st.mode == EPI_GELU_F16) {
                // handed to the next stage: column pairs as one 4-byte write-through store
                const float v = sum + st.ep.bias[min(c, st.N - 1)];
                const _Float16 h = (_Float16) gelu_lookup(st.ep.gelu_tab, v);
                const unsigned u = __builtin_bit_cast(uint16_t, h);
                const unsigned pu = __shfl_xor(u, 1);
                if (ok && !(cc & 1)) st_ag((unsigned *) (st.ep.out16 + (size_t) r * st.ep.ldo + c), u | (pu << 16));
            } else if (st.mode == EPI_F16) {
                if (ok) epi_store<EPI_F16>(st.ep, r, c, sum);
            } else if (st.mode == EPI_QKV_DEC) {
                if (ok) epi_store<EPI_QKV_DEC>(st.ep, r, c, sum);
            }
        }
    }
    // 6. publish: every thread's stores have landed, then one arrival for the block (the last stage's
    // outputs are read by the next launch: no drain, no arrival)
    if (s + 1 < a.n_stages) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            __hip_atomic_fetch_add(a.sync + (s * 8 + (blockIdx.x & 7)) * CH_LINE, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    stamp(5);
}

__global__ __launch_bounds__(CH_THREADS) void k_dec_chain(const ChainArgs a) {
    __shared__ __attribute__((aligned(16))) _Float16 sA[CH_MAXR * CH_LDA];
    __shared__ floatx4 red[16][CH_TPI][64];
    __shared__ double lnred[4][4];
    __shared__ __attribute__((aligned(1024))) char sW[CH_WSLOTS * 1024];
#pragma unroll
    for (int s = 0; s < CH_MAXST; ++s) {
        if (s >= a.n_stages) break;
        chain_stage(a, a.st[s], s, sA, sW, red, lnred);
        __syncthreads();  // LDS (rows, partials) reused by the next stage
    }
    // the last block out leaves every count at zero for the next launch (all others have made their last poll)
    if (threadIdx.x == 0) {
        unsigned * ex = a.sync + CH_MAXST * 8 * CH_LINE;
        const unsigned old = __hip_atomic_fetch_add(ex, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            for (int i = 0; i < CH_MAXST * 8; ++i) st_ag(a.sync + i * CH_LINE, 0u);
            st_ag(ex, 0u);
        }
    }
}

void dec_chain(hipStream_t s, const ChainArgs & a) {
    if (a.M < 1 || a.M > CH_MAXR || a.d < 32 || a.d > CH_MAXD || a.d % 32 || a.n_stages < 1 || a.n_stages > CH_MAXST ||
        !a.sync)
        throw std::runtime_error("dec_chain: unsupported pass");
    int grid = 1;
    for (int i = 0; i < a.n_stages; ++i) {
        const ChainStage & st = a.st[i];
        if (st.N > 0) {
            if (st.N % 16 || st.K % 32 || st.J < 1 || st.J > CH_J || st.nw < 1 || st.nw > 16 || st.KS < 1 ||
                st.tpi < 1 || st.tpi > CH_TPI || !st.Wt || (st.mode != EPI_PARTIAL && st.KS != 1) ||
                (st.mode == EPI_PARTIAL && !st.part) || (!st.ln_part && !st.A) || (st.ln_part && st.K != a.d) ||
                st.K / 32 > st.nw * st.J * st.KS || st.nw * st.tpi * st.J > CH_WSLOTS)
                throw std::runtime_error("dec_chain: bad stage");
            if (st.mode != EPI_PARTIAL && st.mode != EPI_F16 && st.mode != EPI_GELU_F16 && st.mode != EPI_QKV_DEC)
                throw std::runtime_error("dec_chain: bad epilogue");
        }
        if (st.ln_part && (st.ln_ks < 1 || st.ln_ks > CH_KSMAX || !st.ln_bias || !st.x_in || !st.x_out))
            throw std::runtime_error("dec_chain: bad LayerNorm prologue");
        if (st.N <= 0 && !st.ln_part) throw std::runtime_error("dec_chain: empty stage");
        const int tiles = (st.N + 15) / 16;
        const int items = st.N > 0 ? ((tiles + st.tpi - 1) / st.tpi) * st.KS : 1;
        grid = std::max(grid, items);
    }
    if (grid > dec_chain_grid()) throw std::runtime_error("dec_chain: more items than resident blocks");
    OWK_LAUNCH(k_dec_chain, dim3(grid), dim3(CH_THREADS), 0, s, a);
}

int dec_chain_grid() {
    static const int g = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        return std::min(cus, 256);
    }();
    return g;
}

}  // namespace owk
