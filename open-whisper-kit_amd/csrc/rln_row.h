// The row of resid_layernorm (kernels.h): the k splits of an EPI_PARTIAL decode-row GEMM summed in
// order, bias and residual added (x[r] += sum + bias, whisper.cpp's ggml_add(mul_mat + b, inpL)), the
// new residual row written, then its LayerNorm as f16 rows (and optional Q8_0 rows) for the next matmul.
// k_resid_layernorm (k_misc.hip) runs one 256-thread block per row. SC1: the partial tiles come from
// other blocks of the same launch (agent-scope loads) -- the form an in-launch finish of the partial
// GEMM used (measured slower). The LayerNorm statistics are the same double sums
// as ln_row_regs.
#pragma once

namespace owk {

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int) (uint32_t) u, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int) (uint32_t) (u >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((uint64_t) (uint32_t) hi << 32) | (uint32_t) lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((int) (uint32_t) u, l);
    const uint32_t hi = __builtin_amdgcn_readlane((int) (uint32_t) (u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t) hi << 32) | lo);
}

// the xor butterfly's sum over the wave (offsets 1, 2, 4, 8, 16, 32; every lane ends with the same
// bits): offsets 1 and 2 as DPP quad permutes, 4 and 8 as the half-row / row mirrors (after the quad
// steps every lane of a quad holds the quad's sum, so the mirror partner carries the xor partner's
// bits), then the four row sums broadcast and added as the butterfly's last two steps add them at
// lane 0 -- no LDS-crossbar permutes. Bit-identical to the butterfly in every lane.
__device__ __forceinline__ double wave_sum_d(double v) {
    v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
    v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
    v += dpp_d<0x141>(v);  // row_half_mirror: the other quad of the 8
    v += dpp_d<0x140>(v);  // row_mirror: the other 8 of the row
    return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

constexpr int RL_V4 = 2;     // float4 per thread -> N <= 2048
constexpr int RL_KSMAX = 4;  // k splits (gemm_partial_splits <= 3, q5_partial_splits <= 4)

// sum over the block's first four waves (the row's 256 threads); every thread of the block calls it
__device__ __forceinline__ double block_sum4_d(double v, double * red) {
    v = wave_sum_d(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0 && w < 4) red[w] = v;
    __syncthreads();
    const double t = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return t;
}

template <bool SC1>
__device__ __forceinline__ float4 rln_part_load(const float4 * p) {
    if constexpr (SC1) {
        const float * f = (const float *) p;
        return float4{__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load(f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load(f + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load(f + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
    } else {
        return *p;
    }
}

// row `row` of the pass; red: a 4-double LDS array; every thread of the block calls it
template <bool SC1>
__device__ __forceinline__ void resid_ln_row(int row, int M, int N, int KS, const float * part, const float * bias,
                                             float * x, const float * w, const float * b, float eps, _Float16 * xn,
                                             int ldo, int8_t * q8, float * q8d, double * red) {
    const int t = threadIdx.x & 255;
    const bool act = threadIdx.x < 256;  // the row's 256 threads (a larger block: the rest only meet the barriers)
    const int n4 = N >> 2;
    float4 * xr = (float4 *) (x + (size_t) row * N);
    // every load of the block is issued before the first add (the k splits, bias, residual and the
    // LayerNorm gains): one memory round trip instead of one per split (a runtime split loop waits
    // on each load before the next is issued)
    const float4 z4 = float4{0.f, 0.f, 0.f, 0.f};
    // branch-free: indices clamped into the row / the last split, unused values discarded below
    const float4 * p4 = (const float4 *) part;
    const float4 * w4 = (const float4 *) (w ? w : bias);
    const float4 * b4 = (const float4 *) (w ? b : bias);
    float4 pv[RL_V4][RL_KSMAX], bv[RL_V4], rv[RL_V4], wv[RL_V4], lbv[RL_V4];
#pragma unroll
    for (int j = 0; j < RL_V4; ++j) {
        const int i = min(t + 256 * j, n4 - 1);
#pragma unroll
        for (int ks = 0; ks < RL_KSMAX; ++ks) pv[j][ks] = rln_part_load<SC1>(p4 + ((size_t) min(ks, KS - 1) * M + row) * n4 + i);
        bv[j] = ((const float4 *) bias)[i];
        rv[j] = xr[i];
        wv[j] = w4[i];
        lbv[j] = b4[i];
    }
    float4 xv[RL_V4];
#pragma unroll
    for (int j = 0; j < RL_V4; ++j) {
        const int i = t + 256 * j;
        float4 r = z4;
        if (i < n4) {
            float4 a = pv[j][0];  // the splits in k order, as before
#pragma unroll
            for (int ks = 1; ks < RL_KSMAX; ++ks) {
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
            if (act) xr[i] = r;
        }
        xv[j] = r;
    }
    if (!w) return;
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < RL_V4; ++j)
        s += ((double) xv[j].x + (double) xv[j].y) + ((double) xv[j].z + (double) xv[j].w);
    s = block_sum4_d(s, red);
    const float mean = (float) s / (float) N;
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < RL_V4; ++j) {
        if (t + 256 * j < n4) {
            const float tx = xv[j].x - mean, ty = xv[j].y - mean, tz = xv[j].z - mean, tw = xv[j].w - mean;
            v += ((double) (tx * tx) + (double) (ty * ty)) + ((double) (tz * tz) + (double) (tw * tw));
        }
    }
    v = block_sum4_d(v, red);
    const float var = (float) (v / (double) N);
    const float scale = 1.0f / sqrtf(var + eps);
    _Float16 * o = xn + (size_t) row * ldo;
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
            *(half4 *) (o + 4 * i) = h;
            if (q8) {
                // Q8_0 rows of the f32 LayerNorm output (quantized GEMM operand; x86 quantize_row_q8_0):
                // a 32-block is the float4s of 8 consecutive threads (N % 32 == 0)
                float m = fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w)));
#pragma unroll
                for (int sh = 1; sh < 8; sh <<= 1) m = fmaxf(m, __shfl_xor(m, sh, 8));
                const float id = m != 0.0f ? 127.f / m : 0.0f;
                char4 qv;
                qv.x = (signed char) rintf(y.x * id);
                qv.y = (signed char) rintf(y.y * id);
                qv.z = (signed char) rintf(y.z * id);
                qv.w = (signed char) rintf(y.w * id);
                *(char4 *) (q8 + (size_t) row * N + 4 * i) = qv;
                if ((i & 7) == 0) q8d[(size_t) row * (N / 32) + (i >> 3)] = m / 127.f;  // raw f32 d (kernels.h QFmt)
            }
        }
    }
}

}  // namespace owk
