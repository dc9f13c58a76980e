// Launch interfaces of the streaming-SortFormer gfx950 kernels (k_sortformer.hip).
// Dense linears reuse the MFMA GEMM of k_gemm.hip (kernels.h) with the SortFormer epilogues.
#pragma once

#include "kernels.h"

namespace owk {
namespace sf {

// NeMo log-mel (ref sortformer.cpp:779-894): pre-emphasis 0.97, zero pad n_fft/2 both sides,
// Hann(400) centred in 512, radix-2 float FFT (twiddle recurrence, ref 217-263), power,
// mel = fb . P (float), ln(mel + 2^-24). Frames [0, n_compute) of mel[n_mels][n_frames_out].
// tw: per-stage twiddles [511][2] as the reference's recurrence produces them (host-built).
void mel(hipStream_t s, const float * pcm, int n_samples, const float * win512, const float * tw, const float * fb,
         int n_mels, int n_compute, int n_frames_out, float * mel);

// pre-encoder stage 1: Conv2d(1 -> C, 3x3, s2, p1) + bias, ReLU over the chunk mel window
// mel[f][c0 + t] (f < 128, t < T_in, row stride ld). out [T1][F1][C] f32.
void conv0(hipStream_t s, const float * mel, int ld, int c0, int T_in, int n_mels, const float * w, const float * b,
           int C, float * out, int T1, int F1);
// depthwise Conv2d(C, 3x3, s2, p1) + bias: in [Ti][Fi][C] -> out [To][Fo][C] (ops.cpp:7035-7070 order)
void dwconv(hipStream_t s, const float * in, int Ti, int Fi, int C, const float * w, const float * b, float * out,
            int To, int Fo);
// pointwise Conv2d(C -> C, 1x1) + bias, ReLU as an f32 GEMM over positions: in [P][C] -> out.
// flatten == 0: out32 [P][C];  flatten == 1: out16 [t][c * Fo + f] (the permute/flatten of
// sortformer.cpp:1002-1003 feeding pre_encode.out), P = t * Fo + f.
void pwconv(hipStream_t s, const float * in, int P, int C, const float * w, const float * b, int flatten, int Fo,
            float * out32, _Float16 * out16, int ld16);

// x_out = x * s (ggml_scale)
void scale(hipStream_t s, const float * x, size_t n, float sc, float * out);
// out16 = f16(relu(x)) (ggml_relu before an F16 mul_mat)
void relu_f16(hipStream_t s, const float * x, size_t n, _Float16 * out);
// out16 = f16(x) (the activation rounding of a mul_mat with F16 weights)
void to_f16(hipStream_t s, const float * x, size_t n, _Float16 * out);

// Multi-head attention over T keys, f32 (ggml_mul_mat F32 x F32 + ggml_soft_max):
//   score[i][j] = ((q_i + u) . k_j + [REL] (q_i + v) . P[T-1-i+j]) * sc, softmax over j, out = sum_j p_ij v_j
// qkv: [T][ldq] f32 with Q at column 0, K at kcol, V at vcol (head h at h*dh); u, v: [H][dh]
// (REL only, else null); P: [2T-1][H*dh] f32 (REL only). out: [T][H*dh] f16, or f32 into out32 when
// given (the operand a quantized linear_out / out_projection rounds to Q8 itself); ldP: P's row stride
// (0: H*dh; the conformer passes every layer's P side by side)
void attention(hipStream_t s, int dh, bool rel, const float * qkv, int ldq, int kcol, int vcol, int T, int H,
               const float * u, const float * v, const float * P, float sc, _Float16 * out, float * out32 = nullptr,
               int ldP = 0);

// conformer conv module middle: GLU over pw1 output x [T][2C] (a * sigmoid(g)), depthwise conv
// (k taps, zero padded (k-1)/2, ggml_ssm_conv order) + bias, SiLU -> out16 [T][C]
void glu_dwconv(hipStream_t s, const float * x, int T, int C, const float * w, int k, const float * b, _Float16 * out);

}  // namespace sf
}  // namespace owk
