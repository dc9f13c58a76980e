// K-quant weights (q2_K .. q6_K, 256-weight super-blocks; ref ggml/src/ggml-common.h block_q*_K,
// ggml/src/ggml-quants.c:784-1877) for the f16-MFMA ring GEMM (k_gemm_q16): host expansion at load.
//
// The reference multiplies a K-quant row with Q8_K activation rows (quantize_row_q8_K_ref: one f32
// d per 256, int8 q, int16 sums per 16) as   d_x*d_y * SUM_j s_j * dot(q_x, q_y)_j
//                                            - dmin_x*d_y * SUM_j m_j * bsum_j
// (ggml-cpu/arch/x86/quants.c ggml_vec_dot_q*_K_q8_K; the 4-bit sub-scales s_j / mins m_j and the
// integer dots are exact). Here each super-block becomes a run of 32-wide "virtual" K blocks whose
// MFMA dot is an exact integer (|partial| < 2^24 in the f32 accumulator) scaled by one f32 factor
// (the kernel's acc = fma(dot, dw * da, acc)):
//   q2_K, q4_K, q5_K  8 blocks of s_j * q (sub-scale folded into the f16 weight: <= 15*3, 63*15,
//                     63*31 < 2048, exact)  with dw = d, then ONE min block: 16 weights -m_j per
//                     16-sum (m of the 16- or 32-wide sub-block) against the 16 bsums, dw = dmin;
//                     288 virtual K per 256
//   q3_K              8 blocks of (s_j - 32) * q (|.| <= 128) with dw = d; 256 per 256
//   q6_K              16 blocks, each one 16-wide sub-block (q - 32) and 16 zeros, dw = d * s_j
//                     (exact f32 product: s_j * (q-32) reaches 4096, not exact in f16); 512 per 256
// The activation side (k_quantize_q8k_f16) writes the matching layout. The products and sums are
// the reference's integers; the f32 combination order differs from its 8-lane AVX2 accumulators
// (last-ulp level, as the Q5_0 path).
#pragma once

#include <cstddef>
#include <cstdint>

namespace owk {

int kq_block_bytes(int fmt);     // bytes per 256-weight super-block (84 / 110 / 144 / 176 / 210)
int kq_ggml_type(int fmt);       // GGML_TYPE_Q2_K .. Q6_K (10 .. 14)
int kq_kx(int fmt, int K);       // virtual K of a K-long row
int kq_layout(int fmt);          // 0: 8 + min block, 1: 8 blocks, 2: 16 half blocks (k_quantize_q8k_f16)

// rows [N][K/256 super-blocks] -> wi [N][kx] f16 (exact integers, as uint16 bits) and the virtual
// block scales dwt[kb][npad] f32 (columns n >= N: 0)
void kq_expand_host(int fmt, const uint8_t * blocks, int N, int K, uint16_t * wi, float * dwt, int npad);
// one row -> f32 exactly as the reference's dequantize_row_q*_K as built by gcc (-ffp-contract=fast
// contracts `d * q - m` into one fused multiply-add; tests/test_kquant.py pins it bit for bit)
void kq_dequant_row_host(int fmt, const uint8_t * blocks, int K, float * y);

} // namespace owk
