// Logit filtering, log-softmax and token selection on the device, gfx950.
//
// One block per decoder row re-implements whisper_process_logits (ref
// src/whisper.cpp:6177-6445) and the greedy branch of whisper_sample_token
// (6460-6517) so a decode step returns ~32 bytes per sequence instead of the
// reference's 200 KB logits download and O(n_vocab) host loop per decoder.
// Masks are applied in the reference's order; log-sum-exp sums run in double.
#include "kernels.h"

namespace owk {

constexpr int LG_THREADS = 1024;
constexpr int LG_WAVES = LG_THREADS / 64;

enum : int {
    LF_INITIAL = 1, LF_LAST_TS = 2, LF_PENULT_TS = 4, LF_HAS_TS = 8, LF_SUPPRESS_BLANK = 16,
    LF_NO_TS = 32, LF_TDRZ = 64, LF_SUPPRESS_EOT = 128, LF_NEED_NOSP = 256, LF_MAX_INIT_TS = 512,
};

__device__ __forceinline__ float block_max(float v, float * red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < LG_WAVES; ++i) r = fmaxf(r, red[i]);
    return r;
}

__device__ __forceinline__ double block_sum(double v, double * red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double r = 0.0;
    for (int i = 0; i < LG_WAVES; ++i) r += red[i];
    return r;
}

// (value, index) max with the smallest index winning ties ("first max", whisper.cpp:6496-6502)
__device__ __forceinline__ void block_argmax(float & v, int & idx, float * redv, int * redi) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(idx, o, 64);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { redv[w] = v; redi[w] = idx; }
    __syncthreads();
    v = redv[0]; idx = redi[0];
    for (int i = 1; i < LG_WAVES; ++i)
        if (redv[i] > v || (redv[i] == v && redi[i] < idx)) { v = redv[i]; idx = redi[i]; }
}

__device__ __forceinline__ bool masked(int i, int f, int ts_min, const VocabInfo & vi) {
    if ((f & LF_SUPPRESS_BLANK) && (f & LF_INITIAL) && (i == vi.eot || i == vi.space)) return true;
    if (i == vi.not_) return true;
    if ((f & LF_NO_TS) && i >= vi.beg) return true;
    if (i == vi.sot || i == vi.nosp) return true;
    if (!(f & LF_TDRZ) && i == vi.solm) return true;
    if (i == vi.translate || i == vi.transcribe || i == vi.prev) return true;
    if (i >= vi.lang_begin && i < vi.lang_begin + vi.n_lang) return true;
    if ((f & LF_SUPPRESS_EOT) && i == vi.eot) return true;
    if (f & LF_LAST_TS) {
        if (f & LF_PENULT_TS) { if (i >= vi.beg) return true; }
        else if (i < vi.eot) return true;
    }
    if ((f & LF_INITIAL) && (f & LF_MAX_INIT_TS) && i >= vi.beg + vi.tid0_max + 1) return true;
    if ((f & LF_HAS_TS) && i >= vi.beg && i < vi.beg + ts_min) return true;
    return false;
}

__global__ __launch_bounds__(LG_THREADS) void k_process_logits(float * __restrict__ logits, int n_vocab,
                                                              const LogitJob * __restrict__ jobs, VocabInfo vi,
                                                              TokenOut * __restrict__ outv, float * __restrict__ lp_out,
                                                              float * __restrict__ pr_out) {
    __shared__ float redf[LG_WAVES];
    __shared__ double redd[LG_WAVES];
    __shared__ int redi[LG_WAVES];
    __shared__ int apply_ts_rule;
    const LogitJob job = jobs[blockIdx.x];
    float * L = logits + (size_t) job.row * n_vocab;
    const int f = job.flags;
    const int tid = threadIdx.x;
    TokenOut res;
    res.nosp_prob = 0.0f;

    // no_speech probability of the raw logits (whisper.cpp:7186-7196)
    if (f & LF_NEED_NOSP) {
        float mx = -INFINITY;
        for (int i = tid; i < n_vocab; i += LG_THREADS) mx = fmaxf(mx, L[i]);
        mx = block_max(mx, redf);
        double s = 0.0;
        for (int i = tid; i < n_vocab; i += LG_THREADS)
            if (L[i] > -INFINITY) s += (double) expf(L[i] - mx);
        s = block_sum(s, redd);
        const float lse = logf((float) s) + mx;
        res.nosp_prob = expf(L[vi.nosp] - lse);
    }

    // temperature + suppression masks (whisper.cpp:6200-6330)
    for (int i = tid; i < n_vocab; i += LG_THREADS) {
        float v = L[i];
        if (job.temperature > 0.0f) v /= job.temperature;
        if (masked(i, f, job.ts_min, vi)) v = -INFINITY;
        L[i] = v;
    }
    __syncthreads();
    for (int j = tid; j < vi.n_suppress; j += LG_THREADS) L[vi.suppress_list[j]] = -INFINITY;
    __syncthreads();

    // log_softmax (whisper_compute_logprobs, 6137-6157)
    float mx = -INFINITY;
    for (int i = tid; i < n_vocab; i += LG_THREADS) mx = fmaxf(mx, L[i]);
    mx = block_max(mx, redf);
    double s = 0.0;
    for (int i = tid; i < n_vocab; i += LG_THREADS)
        if (L[i] > -INFINITY) s += (double) expf(L[i] - mx);
    s = block_sum(s, redd);
    const float lse = logf((float) s) + mx;

    // timestamp mass vs best text token (6337-6361)
    float ts_max = -INFINITY, tx_max = -INFINITY;
    for (int i = tid; i < n_vocab; i += LG_THREADS) {
        const float lp = L[i] > -INFINITY ? L[i] - lse : -INFINITY;
        if (i >= vi.beg) ts_max = fmaxf(ts_max, lp); else tx_max = fmaxf(tx_max, lp);
    }
    ts_max = block_max(ts_max, redf);
    tx_max = block_max(tx_max, redf);
    double ts_sum = 0.0;
    for (int i = vi.beg + tid; i < n_vocab; i += LG_THREADS) {
        const float lp = L[i] > -INFINITY ? L[i] - lse : -INFINITY;
        if (lp > -INFINITY) ts_sum += (double) expf(lp - ts_max);
    }
    ts_sum = block_sum(ts_sum, redd);
    if (tid == 0) {
        const float ts_lp = ts_sum > 0.0 ? logf((float) ts_sum) + ts_max : -INFINITY;
        apply_ts_rule = ts_lp > tx_max;
    }
    __syncthreads();
    if (apply_ts_rule)
        for (int i = tid; i < vi.beg; i += LG_THREADS) L[i] = -INFINITY;
    __syncthreads();

    // probs + greedy pick (whisper_compute_probs 6159-6171, whisper_sample_token 6460-6517)
    float best = -1.0f;
    int best_i = 0x7fffffff;
    float tbest = -1.0f;
    int tbest_i = 0x7fffffff;
    double ts_psum = 0.0;
    for (int i = tid; i < n_vocab; i += LG_THREADS) {
        const float lp = L[i] > -INFINITY ? L[i] - lse : -INFINITY;
        const float p = L[i] == -INFINITY ? 0.0f : expf(lp);
        if (lp_out) lp_out[(size_t) blockIdx.x * n_vocab + i] = lp;
        if (pr_out) pr_out[(size_t) blockIdx.x * n_vocab + i] = p;
        if (p > best) { best = p; best_i = i; }
        if (i >= vi.beg) {
            ts_psum += (double) p;
            if (p > tbest) { tbest = p; tbest_i = i; }
        }
    }
    block_argmax(best, best_i, redf, redi);
    block_argmax(tbest, tbest_i, redf, redi);
    ts_psum = block_sum(ts_psum, redd);
    if (tid == 0) {
        res.id = best > 0.0f ? best_i : 0;
        res.p = best > 0.0f ? best : 0.0f;
        res.plog = L[res.id] > -INFINITY ? L[res.id] - lse : -INFINITY;
        // max_ts starts at 0 in the reference: tid stays 0 unless some ts prob > 0
        res.tid = tbest > 0.0f ? tbest_i : 0;
        const double max_ts = tbest > 0.0f ? (double) tbest : 0.0;
        res.pt = (float) (max_ts / (ts_psum + 1e-10));
        res.ptsum = (float) ts_psum;
        if (res.id >= vi.beg) {
            res.tid = res.id;
            res.pt = res.p;
        }
        res.pad_ = 0.0f;
        outv[blockIdx.x] = res;
    }
}

// ---------------------------------------------------------------------------------
// state->logits emulation for the no-speech probability. The reference computes it
// with whisper_compute_logprobs(state->logits, n_vocab, ...) (ref 7186-7196): the max
// is taken over the WHOLE [n_tokens][n_vocab] buffer (only the flagged rows of the
// last decode call are fresh, the others hold stale or zero-initialised values) while
// the soft-max runs over row 0. The engine keeps row 0 and per-row maxima per clip.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(LG_THREADS) void k_row_max(const float * __restrict__ logits, int n_vocab,
                                                       float * __restrict__ out) {
    __shared__ float redf[LG_WAVES];
    const float * L = logits + (size_t) blockIdx.x * n_vocab;
    float mx = -INFINITY;
    for (int i = threadIdx.x; i < n_vocab; i += LG_THREADS) mx = fmaxf(mx, L[i]);
    mx = block_max(mx, redf);
    if (threadIdx.x == 0) out[blockIdx.x] = mx;
}

void logits_row_max(hipStream_t s, const float * logits, int n_rows, int n_vocab, float * out_dev) {
    if (n_rows <= 0) return;
    OWK_LAUNCH(k_row_max, dim3(n_rows), dim3(LG_THREADS), 0, s, logits, n_vocab, out_dev);
}

// dst_rows[i] <- logits row src_rows[i]  (dst index -1: zero fill)
// row copies: CR_SPLIT blocks per row, 8-byte accesses (rows of an even n_vocab are 8-byte aligned;
// one 256-thread block of 4-byte copies per row took 27 us per decode pass)
constexpr int CR_SPLIT = 16;
__global__ void k_copy_rows(const float * __restrict__ logits, int n_vocab, const int2 * __restrict__ map,
                            float * __restrict__ dst) {
    const int2 m = map[blockIdx.x / CR_SPLIT];
    const int part = blockIdx.x % CR_SPLIT;
    float * d = dst + (size_t) m.y * n_vocab;
    const float * s = logits + (size_t) m.x * n_vocab;
    if ((n_vocab & 1) == 0) {
        const int n2 = n_vocab >> 1, per = (n2 + CR_SPLIT - 1) / CR_SPLIT;
        const int i0 = part * per, i1 = min(n2, i0 + per);
        for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x)
            ((float2 *) d)[i] = m.x >= 0 ? ((const float2 *) s)[i] : float2{0.0f, 0.0f};
    } else {
        const int per = (n_vocab + CR_SPLIT - 1) / CR_SPLIT;
        const int i0 = part * per, i1 = min(n_vocab, i0 + per);
        for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) d[i] = m.x >= 0 ? s[i] : 0.0f;
    }
}

void logits_copy_rows(hipStream_t s, const float * logits, int n_vocab, const int2 * map_dev, int n, float * dst) {
    if (n <= 0) return;
    OWK_LAUNCH(k_copy_rows, dim3(n * CR_SPLIT), dim3(256), 0, s, logits, n_vocab, map_dev, dst);
}

// Emulated state->logits row maxima (see whisper_full.cpp): entry (slot, row, logit_row,
// zero_fill) sets rmx[slot][row] to the max of logits row logit_row, or to 0 for a row
// that a resize of the reference buffer would have zero-filled, or leaves the stale value.
__global__ __launch_bounds__(LG_THREADS) void k_rowmax_update(const float * __restrict__ logits, int n_vocab,
                                                            const int4 * __restrict__ ent, float * __restrict__ rmx,
                                                            int stride) {
    __shared__ float redf[LG_WAVES];
    const int4 e = ent[blockIdx.x];
    float * dst = rmx + (size_t) e.x * stride + e.y;
    if (e.z < 0) {
        if (e.w && threadIdx.x == 0) *dst = 0.0f;
        return;
    }
    const float * L = logits + (size_t) e.z * n_vocab;
    // 8 loads in flight per thread (a max is exact in any order): a loop of single loads waited on
    // each one in turn (51 round trips per thread over a 51866-entry row)
    float mx = -INFINITY;
    int i = threadIdx.x;
    for (; i + 7 * LG_THREADS < n_vocab; i += 8 * LG_THREADS) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = L[i + u * LG_THREADS];
#pragma unroll
        for (int u = 0; u < 8; ++u) mx = fmaxf(mx, v[u]);
    }
    for (; i < n_vocab; i += LG_THREADS) mx = fmaxf(mx, L[i]);
    mx = block_max(mx, redf);
    if (threadIdx.x == 0) *dst = mx;
}

void rowmax_update(hipStream_t s, const float * logits, int n_vocab, const int4 * ent_dev, int n, float * rmx,
                   int stride) {
    if (n <= 0) return;
    OWK_LAUNCH(k_rowmax_update, dim3(n), dim3(LG_THREADS), 0, s, logits, n_vocab, ent_dev, rmx, stride);
}

// No-speech probability after a prefill (ref whisper.cpp:7185-7195): soft-max of the
// emulated buffer's row 0 with the max over the whole buffer (rows 0..n_rows of rmx),
// whisper_compute_logprobs' float sum taken in the reference's sequential order.
constexpr int NS_CHUNK = 4096;
__global__ __launch_bounds__(LG_THREADS) void k_nosp(const float * __restrict__ row0, int n_vocab,
                                                    const int2 * __restrict__ req, const float * __restrict__ rmx,
                                                    int stride, int nosp, float * __restrict__ out) {
    __shared__ float redf[LG_WAVES];
    __shared__ float ex[NS_CHUNK];
    const int2 q = req[blockIdx.x];
    const float * L = row0 + (size_t) q.x * n_vocab;
    const float * R = rmx + (size_t) q.x * stride;
    float m = -INFINITY;
    for (int i = threadIdx.x; i < q.y; i += LG_THREADS) m = fmaxf(m, R[i]);
    m = block_max(m, redf);
    float sum = 0.0f;  // meaningful in thread 0
    for (int c0 = 0; c0 < n_vocab; c0 += NS_CHUNK) {
        const int n = min(NS_CHUNK, n_vocab - c0);
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += LG_THREADS) {
            const float v = L[c0 + i];
            ex[i] = v > -INFINITY ? expf(v - m) : 0.0f;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int i = 0; i < n; ++i) sum += ex[i];
    }
    if (threadIdx.x == 0) {
        const float lse = logf(sum) + m;
        out[blockIdx.x] = L[nosp] == -INFINITY ? 0.0f : expf(L[nosp] - lse);
    }
}

void nosp_probs(hipStream_t s, const float * row0, int n_vocab, const int2 * req_dev, int n, const float * rmx,
                int stride, int nosp, float * out_dev) {
    if (n <= 0) return;
    OWK_LAUNCH(k_nosp, dim3(n), dim3(LG_THREADS), 0, s, row0, n_vocab, req_dev, rmx, stride, nosp, out_dev);
}

// ---------------------------------------------------------------------------------
// The same processing with every row split over LGS_B blocks (decode passes: 32 rows were 32 blocks
// on 256 CUs, each sweeping a 207 KB row six times at one CU's fetch rate: 63 us per pass). Five
// launches, each a short sweep of row / LGS_B, with per-block partials combined in fixed block order:
//   mask    temperature + masks + suppress list (in place); block maxima of the row, of its
//           timestamp range and of its text range
//   sum     M = max of the block maxima; block double sum of exp(L - M)
//   ts      (one block per row) lse = log(sum) + M; the timestamp-mass rule of 6337-6361 over the
//           timestamp range; its decision and lse to the row record
//   pick    the decision applied (text logits -inf, in place); logprobs / probs; block first-max of p,
//           of the timestamp p, block double sum of the timestamp p
//   final   the greedy record of whisper_sample_token from the partials
// max(L_i - lse) = fl(max(L_i) - lse) (rounding is monotonic), so the range maxima of the masked
// logits give the reference's ts_max / tx_max; argmax with first-index ties is order-independent;
// the double sums differ from the one-block order only below double precision. Rows that need the
// no-speech probability of the raw logits (prefill passes) take k_process_logits.
// ---------------------------------------------------------------------------------
constexpr int LGS_B = 16, LGS_T = 256, LGS_W = LGS_T / 64;
struct LgPart {
    float m, tsl, txl, best, tbest;
    int best_i, tbest_i, pad;
    double s, ts_psum;
};
struct LgRow {
    float lse;
    int apply;
};

template <int NW> __device__ __forceinline__ float bmax(float v, float * red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < NW; ++i) r = fmaxf(r, red[i]);
    return r;
}
template <int NW> __device__ __forceinline__ double bsum(double v, double * red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
    for (int i = 0; i < NW; ++i) r += red[i];
    return r;
}
template <int NW> __device__ __forceinline__ void bargmax(float & v, int & idx, float * redv, int * redi) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(idx, o, 64);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { redv[threadIdx.x >> 6] = v; redi[threadIdx.x >> 6] = idx; }
    __syncthreads();
    v = redv[0]; idx = redi[0];
    for (int i = 1; i < NW; ++i)
        if (redv[i] > v || (redv[i] == v && redi[i] < idx)) { v = redv[i]; idx = redi[i]; }
}

__device__ __forceinline__ void lgs_range(int n_vocab, int b, int & i0, int & i1) {
    const int per = (n_vocab + LGS_B - 1) / LGS_B;
    i0 = b * per;
    i1 = min(n_vocab, i0 + per);
}

__global__ __launch_bounds__(LGS_T) void k_lgs_mask(float * __restrict__ logits, int n_vocab,
                                                    const LogitJob * __restrict__ jobs, VocabInfo vi,
                                                    LgPart * __restrict__ part) {
    __shared__ float red[LGS_W];
    const int jb = blockIdx.x / LGS_B, b = blockIdx.x % LGS_B;
    const LogitJob job = jobs[jb];
    float * L = logits + (size_t) job.row * n_vocab;
    int i0, i1;
    lgs_range(n_vocab, b, i0, i1);
    for (int i = i0 + threadIdx.x; i < i1; i += LGS_T) {
        float v = L[i];
        if (job.temperature > 0.0f) v /= job.temperature;
        if (masked(i, job.flags, job.ts_min, vi)) v = -INFINITY;
        L[i] = v;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < vi.n_suppress; j += LGS_T) {
        const int t = vi.suppress_list[j];
        if (t >= i0 && t < i1) L[t] = -INFINITY;
    }
    __syncthreads();
    float m = -INFINITY, ts = -INFINITY, tx = -INFINITY;
    for (int i = i0 + threadIdx.x; i < i1; i += LGS_T) {
        const float v = L[i];
        m = fmaxf(m, v);
        if (i >= vi.beg) ts = fmaxf(ts, v); else tx = fmaxf(tx, v);
    }
    m = bmax<LGS_W>(m, red);
    ts = bmax<LGS_W>(ts, red);
    tx = bmax<LGS_W>(tx, red);
    if (threadIdx.x == 0) {
        LgPart & p = part[blockIdx.x];
        p.m = m;
        p.tsl = ts;
        p.txl = tx;
    }
}

__global__ __launch_bounds__(LGS_T) void k_lgs_sum(const float * __restrict__ logits, int n_vocab,
                                                   const LogitJob * __restrict__ jobs, LgPart * __restrict__ part) {
    __shared__ double red[LGS_W];
    const int jb = blockIdx.x / LGS_B, b = blockIdx.x % LGS_B;
    const float * L = logits + (size_t) jobs[jb].row * n_vocab;
    const LgPart * rp = part + (size_t) jb * LGS_B;
    float M = rp[0].m;
    for (int k = 1; k < LGS_B; ++k) M = fmaxf(M, rp[k].m);
    int i0, i1;
    lgs_range(n_vocab, b, i0, i1);
    double s = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += LGS_T)
        if (L[i] > -INFINITY) s += (double) expf(L[i] - M);
    s = bsum<LGS_W>(s, red);
    if (threadIdx.x == 0) part[blockIdx.x].s = s;
}

__global__ __launch_bounds__(LGS_T) void k_lgs_ts(const float * __restrict__ logits, int n_vocab,
                                                  const LogitJob * __restrict__ jobs, VocabInfo vi,
                                                  const LgPart * __restrict__ part, LgRow * __restrict__ rows) {
    __shared__ double red[LGS_W];
    const int jb = blockIdx.x;
    const float * L = logits + (size_t) jobs[jb].row * n_vocab;
    const LgPart * rp = part + (size_t) jb * LGS_B;
    float M = rp[0].m, tsl = rp[0].tsl, txl = rp[0].txl;
    double S = rp[0].s;
    for (int k = 1; k < LGS_B; ++k) {
        M = fmaxf(M, rp[k].m);
        tsl = fmaxf(tsl, rp[k].tsl);
        txl = fmaxf(txl, rp[k].txl);
        S += rp[k].s;
    }
    const float lse = logf((float) S) + M;
    const float ts_max = tsl > -INFINITY ? tsl - lse : -INFINITY;
    const float tx_max = txl > -INFINITY ? txl - lse : -INFINITY;
    double ts_sum = 0.0;
    for (int i = vi.beg + threadIdx.x; i < n_vocab; i += LGS_T) {
        const float lp = L[i] > -INFINITY ? L[i] - lse : -INFINITY;
        if (lp > -INFINITY) ts_sum += (double) expf(lp - ts_max);
    }
    ts_sum = bsum<LGS_W>(ts_sum, red);
    if (threadIdx.x == 0) {
        const float ts_lp = ts_sum > 0.0 ? logf((float) ts_sum) + ts_max : -INFINITY;
        rows[jb].lse = lse;
        rows[jb].apply = ts_lp > tx_max;
    }
}

__global__ __launch_bounds__(LGS_T) void k_lgs_pick(float * __restrict__ logits, int n_vocab,
                                                    const LogitJob * __restrict__ jobs, VocabInfo vi,
                                                    const LgRow * __restrict__ rows, LgPart * __restrict__ part,
                                                    float * __restrict__ lp_out, float * __restrict__ pr_out) {
    __shared__ float redf[LGS_W];
    __shared__ int redi[LGS_W];
    __shared__ double redd[LGS_W];
    const int jb = blockIdx.x / LGS_B, b = blockIdx.x % LGS_B;
    float * L = logits + (size_t) jobs[jb].row * n_vocab;
    const LgRow row = rows[jb];
    int i0, i1;
    lgs_range(n_vocab, b, i0, i1);
    float best = -1.0f, tbest = -1.0f;
    int best_i = 0x7fffffff, tbest_i = 0x7fffffff;
    double ts_psum = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += LGS_T) {
        float v = L[i];
        if (row.apply && i < vi.beg) {
            v = -INFINITY;
            L[i] = v;
        }
        const float lp = v > -INFINITY ? v - row.lse : -INFINITY;
        const float p = v == -INFINITY ? 0.0f : expf(lp);
        if (lp_out) lp_out[(size_t) jb * n_vocab + i] = lp;
        if (pr_out) pr_out[(size_t) jb * n_vocab + i] = p;
        if (p > best) { best = p; best_i = i; }
        if (i >= vi.beg) {
            ts_psum += (double) p;
            if (p > tbest) { tbest = p; tbest_i = i; }
        }
    }
    bargmax<LGS_W>(best, best_i, redf, redi);
    bargmax<LGS_W>(tbest, tbest_i, redf, redi);
    ts_psum = bsum<LGS_W>(ts_psum, redd);
    if (threadIdx.x == 0) {
        LgPart & p = part[blockIdx.x];
        p.best = best;
        p.best_i = best_i;
        p.tbest = tbest;
        p.tbest_i = tbest_i;
        p.ts_psum = ts_psum;
    }
}

__global__ void k_lgs_final(const float * __restrict__ logits, int n_vocab, const LogitJob * __restrict__ jobs,
                            VocabInfo vi, const LgRow * __restrict__ rows, const LgPart * __restrict__ part,
                            TokenOut * __restrict__ outv) {
    const int jb = blockIdx.x;
    const LgPart * rp = part + (size_t) jb * LGS_B;
    float best = rp[0].best, tbest = rp[0].tbest;
    int best_i = rp[0].best_i, tbest_i = rp[0].tbest_i;
    double ts_psum = rp[0].ts_psum;
    for (int k = 1; k < LGS_B; ++k) {
        if (rp[k].best > best || (rp[k].best == best && rp[k].best_i < best_i)) { best = rp[k].best; best_i = rp[k].best_i; }
        if (rp[k].tbest > tbest || (rp[k].tbest == tbest && rp[k].tbest_i < tbest_i)) {
            tbest = rp[k].tbest;
            tbest_i = rp[k].tbest_i;
        }
        ts_psum += rp[k].ts_psum;
    }
    const float * L = logits + (size_t) jobs[jb].row * n_vocab;
    const float lse = rows[jb].lse;
    TokenOut res;
    res.nosp_prob = 0.0f;
    res.id = best > 0.0f ? best_i : 0;
    res.p = best > 0.0f ? best : 0.0f;
    res.plog = L[res.id] > -INFINITY ? L[res.id] - lse : -INFINITY;
    res.tid = tbest > 0.0f ? tbest_i : 0;
    const double max_ts = tbest > 0.0f ? (double) tbest : 0.0;
    res.pt = (float) (max_ts / (ts_psum + 1e-10));
    res.ptsum = (float) ts_psum;
    if (res.id >= vi.beg) {
        res.tid = res.id;
        res.pt = res.p;
    }
    res.pad_ = 0.0f;
    outv[jb] = res;
}

size_t process_logits_ws_bytes(int n_jobs) {
    return (size_t) n_jobs * LGS_B * sizeof(LgPart) + (size_t) n_jobs * sizeof(LgRow) + 64;
}

void process_logits(hipStream_t s, float * logits, int n_vocab, const LogitJob * jobs_dev, int n_jobs,
                    const VocabInfo & vi, TokenOut * out_dev, float * logprobs_out, float * probs_out, bool any_nosp,
                    void * ws, size_t ws_bytes) {
    if (n_jobs <= 0) return;
    // (turbo bench, interleaved on one box: 3819-3844 one block per row, 3897-3916 split;
    // profiles/archive/r03l_ab_logits_split_turbo.txt)
    if (any_nosp || !ws || ws_bytes < process_logits_ws_bytes(n_jobs)) {
        OWK_LAUNCH(k_process_logits, dim3(n_jobs), dim3(LG_THREADS), 0, s, logits, n_vocab, jobs_dev, vi, out_dev,
                   logprobs_out, probs_out);
        return;
    }
    LgPart * part = (LgPart *) ws;
    LgRow * rows = (LgRow *) (part + (size_t) n_jobs * LGS_B);
    const dim3 g(n_jobs * LGS_B);
    OWK_LAUNCH(k_lgs_mask, g, dim3(LGS_T), 0, s, logits, n_vocab, jobs_dev, vi, part);
    OWK_LAUNCH(k_lgs_sum, g, dim3(LGS_T), 0, s, logits, n_vocab, jobs_dev, part);
    OWK_LAUNCH(k_lgs_ts, dim3(n_jobs), dim3(LGS_T), 0, s, logits, n_vocab, jobs_dev, vi, part, rows);
    OWK_LAUNCH(k_lgs_pick, g, dim3(LGS_T), 0, s, logits, n_vocab, jobs_dev, vi, rows, part, logprobs_out, probs_out);
    OWK_LAUNCH(k_lgs_final, dim3(n_jobs), dim3(1), 0, s, logits, n_vocab, jobs_dev, vi, rows, part, out_dev);
}

} // namespace owk
