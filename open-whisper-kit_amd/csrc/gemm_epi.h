// Device helpers of the f16 GEMMs (k_gemm.hip): the fused epilogue values
// (gelu_lookup, f16_rn, epi_store) and the fixed wave order of the decode-row reductions.
#pragma once

#include "kernels.h"

namespace owk {

__device__ __forceinline__ float gelu_lookup(const uint16_t * tab, float x) {
    // ggml_vec_gelu_f32 with GGML_GELU_FP16 (ggml-cpu/vec.h:995-1009)
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    const _Float16 h = (_Float16) x;
    const uint16_t r = tab[__builtin_bit_cast(uint16_t, h)];
    return (float) __builtin_bit_cast(_Float16, r);
}

// f32 -> f16 after the f32 value is rounded: the empty asm keeps hipcc from folding a preceding
// multiply into v_mad_mixlo_f16 (one rounding of the exact product), which differs from the
// reference's f32 op followed by its F16 conversion on ties (measured: 1 f16 ulp on scaled outputs)
__device__ __forceinline__ _Float16 f16_rn(float v) {
    asm volatile("" : "+v"(v));
    return (_Float16) v;
}

template <int MODE>
__device__ __forceinline__ void epi_store(const EpiParams & p, int r, int c, float acc) {
    if constexpr (MODE == EPI_F16) {
        float v = acc;
        if (p.bias) v += p.bias[c];
        v *= p.scale;
        p.out16[(size_t) r * p.ldo + c] = f16_rn(v);
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
        // head-major cache [slot][head][t][64]: one (row, head) of a decode step streams its
        // keys (and values) as one contiguous run
        const size_t base = (size_t) (p.slot_map ? p.slot_map[clip] : clip) * p.T * d + (size_t) t * 64;
        if (c < d) {
            p.out16b[base + (size_t) (c >> 6) * p.T * 64 + (c & 63)] = f16_rn(acc * p.scale);
        } else {
            const int cv = c - d;
            p.out16c[base + (size_t) (cv >> 6) * p.T * 64 + (cv & 63)] = (_Float16) (acc + p.bias2[cv]);
        }
    } else if constexpr (MODE == EPI_QKV_DEC) {
        const int d = p.d;
        if (c < d) {
            p.out16[(size_t) r * p.ldo + c] = f16_rn((acc + p.bias[c]) * p.scale);
        } else if (c < 2 * d) {
            // head-major self-attention cache [slot][head][cell][64]; Tpad = cells * 64
            const int cc = c - d;
            p.out16b[p.row_off[r] + (size_t) (cc >> 6) * p.Tpad + (cc & 63)] = f16_rn(acc * p.scale);
        } else {
            const int cc = c - 2 * d;
            p.out16c[p.row_off[r] + (size_t) (cc >> 6) * p.Tpad + (cc & 63)] = (_Float16) (acc + p.bias2[cc]);
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
        // out32 (optional): the f32 value too, the operand a quantized consumer matmul rounds to Q8
        const float v = acc + p.bias[c];
        const float y = v / (1.0f + expf(-v));
        if (p.out16) p.out16[(size_t) r * p.ldo + c] = (_Float16) y;
        if (p.out32) p.out32[(size_t) r * p.ldo + c] = y;
    } else if constexpr (MODE == EPI_HALF_RESID) {
        // ggml_add(x, b) -> ggml_scale(0.5) -> ggml_add(residual, .) (sortformer.cpp:1163-1167)
        const float v = (acc + p.bias[c]) * 0.5f;
        const size_t o = (size_t) r * p.ldo + c;
        p.out32[o] = p.resid[o] + v;
    } else if constexpr (MODE == EPI_RELU_F16) {
        const float v = acc + p.bias[c];
        const float y = v > 0.0f ? v : 0.0f;
        if (p.out16) p.out16[(size_t) r * p.ldo + c] = (_Float16) y;
        if (p.out32) p.out32[(size_t) r * p.ldo + c] = y;
    } else if constexpr (MODE == EPI_SIGMOID_F32) {
        const float v = acc + p.bias[c];
        p.out32[(size_t) r * p.ldo + c] = 1.0f / (1.0f + expf(-v));
    }
}
template <> __device__ __forceinline__ void epi_store<EPI_PARTIAL>(const EpiParams &, int, int, float) {}

// one output's wave partials summed in wave order 0 .. nw-1 (the decode-row GEMMs' fixed order), every
// LDS read issued before the first add: rp[w * stride] for w < MAXW stays inside the MAXW-row
// reduction array; rows past nw are read and not used
template <int MAXW>
__device__ __forceinline__ float wave_order_sum(const float * rp, int stride, int nw) {
    float v[MAXW];
#pragma unroll
    for (int w = 0; w < MAXW; ++w) v[w] = rp[w * stride];
    float s = v[0];
#pragma unroll
    for (int w = 1; w < MAXW; ++w)
        if (w < nw) s += v[w];
    return s;
}

}  // namespace owk
