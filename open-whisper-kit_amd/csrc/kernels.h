// Launch interfaces of the gfx950 kernels (implemented in k_*.hip).
#pragma once

#include "common.h"

namespace owk {

// ---------------------------------------------------------------------------------
// GEMM epilogues. Every dense op of the Whisper graph is C[M,N] = A[M,K] * W[N,K]^T
// with A = f16 activations (the reference rounds every mul_mat activation to F16,
// ggml-cpu vec_dot_type F16) and W = f16 weights, f32 accumulate; what differs is the
// fused epilogue (bias / scale / GELU / residual / layout scatter).
// ---------------------------------------------------------------------------------
enum EpiMode : int {
    EPI_F16 = 0,        // out16[r*ldo+c] = f16((acc + bias[c]) * scale)
    EPI_GELU_F16 = 1,   // out16 = gelu_tab(acc + bias)                   (mlp.0, conv1)
    EPI_RESID_F32 = 2,  // out32[r*ldo+c] = resid[r*ldo+c] + (acc + bias)  (attn.out, mlp.2)
    EPI_CONV2 = 3,      // out32[r*ldo+c] = pos[(r%T)*ldo+c] + gelu(acc + bias)  (conv2 + e_pe)
    EPI_QKV_ENC = 4,    // Q/K/V split; V written transposed per (clip, head) for attention
    EPI_KV_CROSS = 5,   // cross K (scaled) / V (+bias) split into the cross-KV cache
    EPI_QKV_DEC = 6,    // decoder self-attn: Q (bias, scale), K (scale), V (bias) -> KV cells
    EPI_F32 = 7,        // out32[r*ldo+c] = acc  (logits)
    EPI_PARTIAL = 8,    // decode-row GEMM only: raw partial tiles to the workspace, finished by
                        // resid_layernorm (bias + residual + next LayerNorm in one pass)
    // SortFormer (streaming-sortformer/src/sortformer.cpp) epilogues
    EPI_BIAS_F32 = 9,   // out32 = acc (+ bias[c]); out16 (optional) = f16 of the same value
    EPI_SILU_F16 = 10,  // out16 = f16(silu(acc + bias)); out32 (optional) the f32 value (conformer FFN linear1)
    EPI_HALF_RESID = 11,// out32 = resid + (acc + bias) * 0.5         (macaron FFN half step)
    EPI_RELU_F16 = 12,  // out16 = f16(relu(acc + bias)); out32 (optional) (transformer FFN, head)
    EPI_SIGMOID_F32 = 13,// out32 = sigmoid(acc + bias)               (speaker head)
};

struct EpiParams {
    const float * bias = nullptr;   // [N] (or [d] slices for split modes)
    const float * bias2 = nullptr;  // second bias (V bias in split modes)
    float scale = 1.0f;
    const float * resid = nullptr;  // f32 residual input
    float * out32 = nullptr;
    _Float16 * out16 = nullptr;
    _Float16 * out16b = nullptr;    // K (split modes)
    _Float16 * out16c = nullptr;    // V (split modes)
    int ldo = 0;                    // leading dim of out32/out16/resid
    int d = 0;                      // model width for split modes
    int T = 0;                      // rows per clip (EPI_CONV2, EPI_QKV_ENC)
    int Tpad = 0;                   // padded key count of the transposed V (EPI_QKV_ENC)
    const float * pos = nullptr;    // EPI_CONV2 positional embedding [T][d]
    const uint16_t * gelu_tab = nullptr;  // 65536-entry f16 GELU table
    const int64_t * row_off = nullptr;    // EPI_QKV_DEC: element offset of each row's KV cell in head 0
                                          // (head h at + h * Tpad: the cache is head-major)
    const int * slot_map = nullptr;       // EPI_KV_CROSS: clip index -> cross-KV slot (null = identity)
    int vec = 0;                          // set by the large-tile launcher: 16-byte vector epilogue allowed
    // quantized large-tile GEMM (gemm_q16): per-32-block scales, block-major [K/32][pad]
    const float * qs_da = nullptr;        // activation d (f16-rounded), rows permuted per 256-row tile
    const float * qs_dw = nullptr;        // weight d
    int qs_mpad = 0, qs_npad = 0;
    int c_off = 0;                        // large-tile launch over a column range: its first column
    // gemm_q5 with an f16 output (EPI_GELU_F16 decode rows fuse it): its Q8_0 rows [M][N] and raw f32
    // block d [M][N/32], the next quantized GEMM's operand (must not alias that GEMM's own operand)
    int8_t * q8 = nullptr;
    float * q8d = nullptr;
};

// large tiles (encoder / conv / cross-KV / long prefill): A [M,lda] f16, W [N,ldw] f16
void gemm_f16(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda,
              const _Float16 * W, int ldw, const EpiParams & ep);
// skinny (decode steps, M <= 64): split-K across the waves of a block, LDS reduction
// this thread's large-GEMM override (-1 none, 0 force 128x128, 8 the 8-phase 256x256 kernel (the
// default), GEMM_MID_FORCED / GEMM_MID32_FORCED the 64x64 / 32x32 ring tile for every shape);
// returns the previous override (debug hooks restore it with GemmOverride)
constexpr int GEMM_MID_FORCED = 16, GEMM_MID32_FORCED = 17;
int gemm_set_256(int on);
struct GemmOverride {
    int prev;
    explicit GemmOverride(int on) : prev(gemm_set_256(on)) {}
    ~GemmOverride() { gemm_set_256(prev); }
};
void gemm_f16_skinny(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda,
                     const _Float16 * W, int ldw, const EpiParams & ep);
// split-K workspace of the decode-row GEMM (owned by the caller: one per stream)
struct GemmWs {
    float * partial = nullptr;  // partial tiles [k split][column tile][rows][16]
    size_t partial_floats = 0;
};
size_t gemm_ws_floats(int N, int K);  // partial floats a (N, K) decode-row GEMM needs (0 = no split)
size_t gemm_partial_floats(int N, int K);  // workspace of an EPI_PARTIAL decode-row GEMM
int gemm_partial_splits(int K);            // its k splits (rows of partial tiles)
// x[r][c] += sum_ks partial + bias[c]  (the reference's mul_mat + bias + residual add), then
// LayerNorm of the updated row -> xn (f16), unless lnw == nullptr (residual only).
// `part` holds `ks` splits [ks][M][N] of an EPI_PARTIAL GEMM with M rows (M <= 32) and N columns.
// q8/q8d (optional): the f32 LayerNorm output as Q8_0 rows too (a quantized model's next GEMM operand)
void resid_layernorm(hipStream_t s, int M, int N, int ks, const float * part, const float * bias, float * x,
                     const float * lnw, const float * lnb, float eps, _Float16 * xn, int ldo,
                     int8_t * q8 = nullptr, float * q8d = nullptr);
// decode-row GEMM whose A operand is f16(LayerNorm(x)) of the f32 residual stream x [M][K] (lnw / lnb
// the LayerNorm gain / bias [K]): the LayerNorm runs in the GEMM's prologue (M <= 32, K <= 1280,
// epilogues EPI_F16 / EPI_GELU_F16 / EPI_QKV_DEC); Wt the tiled weight copy
// the bit-exact whole-K chain of passes with <= 16 rows (k_gemm.hip): residual matmul in one launch
// (x += A W^T + bias, the split-K partials + resid_layernorm's order) and the LayerNorm-prologue matmul
// (order 0: the statistics of resid_layernorm, 1: of layernorm_f16 -- the kernel whose f16 rows it replaces)
bool gemm_rows_exact_applies(int M, int d);
void gemm_rows_res(hipStream_t s, int M, int N, int K, const _Float16 * A, const _Float16 * Wt, const float * bias,
                   float * x);
void gemm_rows_lnx(hipStream_t s, int mode, int order, int M, int N, int K, const float * x, const float * lnw,
                   const float * lnb, float eps, const _Float16 * Wt, const EpiParams & ep);
bool gemm_rows_ln_applies(int M, int N, int K);
void gemm_rows_ln(hipStream_t s, int mode, int M, int N, int K, const float * x, const float * lnw, const float * lnb,
                  float eps, const _Float16 * Wt, const EpiParams & ep, bool debug_no_stats = false);
// dispatch on M: <= 32 rows decode-row GEMM (needs the tiled copy Wt), <= 64 skinny,
// else 128x128 tiles (row-major W)
void gemm(hipStream_t s, int mode, int M, int N, int K, const _Float16 * A, int lda,
          const _Float16 * W, int ldw, const EpiParams & ep, const GemmWs * ws = nullptr,
          const _Float16 * Wt = nullptr);
// tiled weight copy for the decode-row GEMM: [ceil(N/16)][K/32][64 lanes][8] f16
size_t tiled_weight_elems(int N, int K);
void tile_weights(hipStream_t s, const _Float16 * W, int N, int K, _Float16 * out);

// ---------------------------------------------------------------------------------
// Q5_0 weights x Q8_0 activations (ggml MOSTLY_Q5_0 models, ftype 2008). The reference
// quantizes every mul_mat activation row to Q8_0 per 32 (x86 quantize_row_q8_0,
// ggml-cpu/arch/x86/quants.c:290-360) and takes the integer dot with the Q5_0 block
// (ggml_vec_dot_q5_0_q8_0, quants.c:845) scaled by d_w * d_a per block. Here the dot is
// v_mfma_i32_16x16x32_i8 per 32-block (exact integers), scaled and accumulated in f32.
// ---------------------------------------------------------------------------------
// Weight formats of the quantized pipeline (ggml block types; whisper-quantize ftypes):
//   Q5_0 (ftype 8)  w = d * (q5 - 16)       x Q8_0 activations
//   Q8_0 (ftype 7)  w = d * q8              x Q8_0
//   Q4_0 (ftype 2)  w = d * (q4 - 8)        x Q8_0
//   Q4_1 (ftype 3)  w = d * q4 + m          x Q8_1 (ggml_vec_dot_q4_1_q8_1, x86 quants.c:701)
//   Q5_1 (ftype 9)  w = d * q5 + m          x Q8_1 (ggml_vec_dot_q5_1_q8_1, x86 quants.c:925)
// A "_1" block's dot is d_w d_a sum(qw qa) + m_w s_a with s_a = f16(d_a_f32 * sum(qa)) the
// Q8_1 block sum (quantize_row_q8_1, x86 quants.c:388): the GEMMs form it from the int8
// activations and the UNROUNDED f32 scale, so activation producers store the raw f32
// d = amax / 127 and every consumer rounds it to f16 itself (the stored block_q8_*.d).
//   Q2_K .. Q6_K (ftype 10-14): 256-weight super-blocks x Q8_K activations (kquant.h): the
//   f16-MFMA ring kernel (gemm_q16) over "virtual" 32-blocks, at every row count
enum QFmt : int { QF_Q5_0 = 0, QF_Q8_0 = 1, QF_Q4_0 = 2, QF_Q4_1 = 3, QF_Q5_1 = 4,
                  QF_Q2_K = 5, QF_Q3_K = 6, QF_Q4_K = 7, QF_Q5_K = 8, QF_Q6_K = 9 };
__host__ __device__ constexpr bool qf_is_k(int f) { return f >= QF_Q2_K && f <= QF_Q6_K; }
__host__ __device__ constexpr bool qf_has_qh(int f) { return f == QF_Q5_0 || f == QF_Q5_1; }
__host__ __device__ constexpr bool qf_has_m(int f) { return f == QF_Q4_1 || f == QF_Q5_1; }
__host__ __device__ constexpr int qf_qs_bytes(int f) { return f == QF_Q8_0 ? 32 : 16; }  // per 32 weights
// column-tiled decode record per (16-row tile, 32-wide K block): qs (16 x 16 or 16 x 32 B) |
// qh (16 x 4 B, 5-bit formats) | d (16 x 2 B) | m (16 x 2 B, "_1" formats)
__host__ __device__ constexpr int qf_tile_bytes(int f) {
    return 16 * qf_qs_bytes(f) + (qf_has_qh(f) ? 64 : 0) + 32 + (qf_has_m(f) ? 32 : 0);
}
__host__ __device__ constexpr int qf_tile_off_qh(int f) { return 16 * qf_qs_bytes(f); }
__host__ __device__ constexpr int qf_tile_off_d(int f) { return 16 * qf_qs_bytes(f) + (qf_has_qh(f) ? 64 : 0); }
__host__ __device__ constexpr int qf_tile_off_m(int f) { return qf_tile_off_d(f) + 32; }
int qf_block_bytes(int f);  // ggml block size (18 / 20 / 22 / 24 / 34)
int qf_ggml_type(int f);    // GGML_TYPE_Q5_0 6, Q8_0 8, Q4_0 2, Q4_1 3, Q5_1 7

struct Q5W {
    const uint8_t * qs = nullptr;   // [N][K/2]: block b = 16 bytes, byte j = element j | element j+16 << 4
                                    // (Q8_0: [N][K] int8)
    const uint32_t * qh = nullptr;  // [N][K/32]: 5th bits, bit j = element j (Q5_0 / Q5_1)
    const _Float16 * d = nullptr;   // [N][K/32]: block scales
    const _Float16 * m = nullptr;   // [N][K/32]: block minimums (Q4_1 / Q5_1)
    // decode-step matrices: the column-tiled records (qf_tile_bytes), rows past N zero
    const uint8_t * tiled = nullptr;
    // large-tile (encoder / cross-KV) matrices of the symmetric formats (Q5_0 / Q8_0 / Q4_0): the
    // integer weights as exact f16 values [N][K] and the block scales transposed [K/32][npad] f32
    const _Float16 * wi = nullptr;
    const float * dwt = nullptr;
    int npad = 0;
    int fmt = QF_Q5_0;
    int kx = 0;  // K-quant formats: the virtual K of wi / dwt (kquant.h); only wi / dwt are set
    explicit operator bool() const { return qs != nullptr || (qf_is_k(fmt) && wi != nullptr); }
};
size_t quant_tiled_bytes(int fmt, int N, int K);
// ggml block rows -> the split arrays (qh / m may be null for formats without them)
void quant_split_host(int fmt, const uint8_t * blocks, int N, int K, uint8_t * qs, uint32_t * qh, uint16_t * d,
                      uint16_t * m);
void quant_tile_host(int fmt, const uint8_t * qs, const uint32_t * qh, const uint16_t * d, const uint16_t * m, int N,
                     int K, uint8_t * out);
// Q8_0 / Q8_1 rows of A (f32 if A32, else f16): q [M][K] int8, dq [M][K/32] (raw f32 d = amax / 127)
void quantize_q8(hipStream_t s, const float * A32, const _Float16 * A16, int lda, int M, int K, int8_t * q, float * dq);
// C[M,N] = Q8(A) . Q(W)^T with the fused epilogue `mode`; EPI_PARTIAL (M <= 32, tiled weights): raw
// split-K partial tiles [q5_partial_splits(K)][M][N] to ep.out32, finished by resid_layernorm
void gemm_q5(hipStream_t s, int mode, int M, int N, int K, const int8_t * qa, const float * da, const Q5W & w,
             const EpiParams & ep);
// the same product through the f16 MFMA ring kernel (M >= 2048 tiles): A = the Q8_0 integers of the
// activation as exact f16 values [M][K] + scales (quantize_q8_f16), W = Q5W::wi / dwt; every 32-block
// dot is exact, then acc = fma(dot, d_w * d_a, acc) in f32 (ggml_vec_dot_q5_0_q8_0's per-block term)
void quantize_q8_f16(hipStream_t s, const float * A32, const _Float16 * A16, int lda, int M, int K, _Float16 * q16,
                     float * dat, int mpad);
void gemm_q16(hipStream_t s, int mode, int M, int N, int K, const _Float16 * q16, const float * dat, int mpad,
              const Q5W & w, const EpiParams & ep);
bool gemm_q16_applies(const Q5W & w, int M, int N, int K);
// Q8_K rows of A (quantize_row_q8_K_ref, ggml-quants.c:2555-2592: per 256 the signed value of the
// first largest |x|, iscale = -127 / max, q = min(127, rne(iscale * x)), d = 1 / iscale, int sums
// per 16) laid out for the K-quant format `fmt` (kquant.h): q16 [M][kq_kx(fmt, K)] exact f16, dat
// [kx / 32][mpad] f32 (rows permuted like quantize_q8_f16). rmul (optional, [M]): rows quantized the
// way the reference's x86 repack path does (ggml_quantize_mat_q8_K_4x8: Q4_K / Q2_K weights, the rows
// of complete groups of 4 of each matmul; k_gemm.hip has the two roundings)
void quantize_q8k_f16(hipStream_t s, const float * A32, const _Float16 * A16, int lda, int M, int K, int fmt,
                      _Float16 * q16, float * dat, int mpad, const uint8_t * rmul = nullptr);
// the reference repacks these K-quant weights for its x86 matmuls (ggml-cpu/repack.cpp:3076-3097:
// Q4_K with AVX2, Q2_K with AVX-512; every whisper linear has N % 8 == 0)
__host__ __device__ constexpr bool qf_k_repacked(int f) { return f == QF_Q4_K || f == QF_Q2_K; }
// expand Q5W block arrays into wi / dwt (device buffers of N*K halves and K/32*npad floats)
void quant_expand_f16(hipStream_t s, const Q5W & w, int N, int K, _Float16 * wi, float * dwt, int npad);
// EPI_PARTIAL decode-row quantized GEMM whose activation rows are f16 (quantized to Q8_0 inside)
int q5_partial_splits(int K);
size_t q5_partial_floats(int N, int K);  // workspace floats of a partial quantized GEMM (M <= 32)

// ---------------------------------------------------------------------------------
// normalisation / elementwise
// ---------------------------------------------------------------------------------
// out16[r] = f16(LN(x[r]) * w + b); mean/variance accumulated in double (ref ops.cpp:3578-3623)
// row_idx (optional): output row i normalises input row row_idx[i]; out32 (optional) f32 copy
// q8/q8d (optional): the f32 output rows as Q8_0 ([row][d] int8, [row][d/32] raw f32 scales),
// the activation rounding of a quantized GEMM done in the producer
void layernorm_f16(hipStream_t s, const float * x, int rows, int d, const float * w, const float * b,
                   float eps, _Float16 * out, int ldo, const int * row_idx = nullptr, float * out32 = nullptr,
                   int8_t * q8 = nullptr, float * q8d = nullptr);
// y = LayerNorm1(x) -> out1 (f16) + out1_32 (f32), then LayerNorm2(y) -> out2 (f16) + out2_32 (f32, optional):
// bit-identical to the two layernorm_f16 calls (one launch; rows of width d, ldo = d)
void layernorm2_f16(hipStream_t s, const float * x, int rows, int d, const float * w1, const float * b1, _Float16 * out1,
                    float * out1_32, const float * w2, const float * b2, _Float16 * out2, float * out2_32, float eps);
// decoder input embedding: x[r] = f32(tok_emb[tok[r]]) + pos_emb[pos[r]]
void embed_tokens(hipStream_t s, const _Float16 * tok_emb, const float * pos_emb, const int * tokens,
                  const int * pos, int rows, int d, float * x);
// the same from a Q5_0 token embedding (ggml get_rows -> dequantize_row_q5_0: d * (q - 16))
void embed_tokens_f32(hipStream_t s, const float * tok_emb, const float * pos_emb, const int * tokens, const int * pos,
                      int rows, int d, float * x);
void embed_tokens_q5(hipStream_t s, const Q5W & te, const float * pos_emb, const int * tokens, const int * pos,
                     int rows, int d, float * x);

// ---------------------------------------------------------------------------------
// audio front-end
// ---------------------------------------------------------------------------------
struct MelJob {
    const float * pcm;   // device pointer to this clip's samples
    int n_samples;
    int n_len;           // frames (n_samples + 480000) / 160
    float * mel;         // device [n_mel][n_len]
};
// log10 power mel spectrogram, un-normalised (ref whisper.cpp:3104-3167), all jobs in one launch
// twiddle: cos[400] then sin[400] (double); hann: periodic window [400] (float, host-computed
// exactly as whisper_global_cache::fill_hann_window, whisper.cpp:3023-3031)
void mel_spectrogram(hipStream_t s, const MelJob * jobs_dev, int n_jobs, int max_frames,
                     const float * filters, const int * filter_rng, int n_mel, const double * twiddle,
                     const float * hann);
// per-job max, clamp to max-8, (x+4)/4 (ref whisper.cpp:3228-3244)
void mel_normalize(hipStream_t s, const MelJob * jobs_dev, int n_jobs, int n_mel);

// im2col for conv1 (k=3, s=1, p=1) from each clip's mel window: A[(clip*3000 + t)][c*3+k], f16
struct MelWindow {
    const float * mel;   // [n_mel][n_len]
    int n_len;
    int offset;          // seek (frames)
};
void conv1_im2col(hipStream_t s, const MelWindow * win_dev, int n_clips, int n_mel, int n_ctx2,
                  int kpad, _Float16 * A);
// im2col for conv2 (k=3, s=2, p=1) over the f16 conv1 output [clips*3000][d]
void conv2_im2col(hipStream_t s, const _Float16 * x, int n_clips, int t_in, int d, _Float16 * A);

// ---------------------------------------------------------------------------------
// attention
// ---------------------------------------------------------------------------------
// encoder self-attention (flash, MFMA) over T real keys + n_zero_pad all-zero keys
// (the reference's GGML_PAD(1500,256) kv_pad rows, whisper.cpp:2055,2145-2159).
// q, k: [clips*T][H*64] f16; vt: [clips][H][64][Tpad] f16; out: [clips*T][H*64] f16
// encoder attention of a flash_attn = false context (soft_max path, F16 probabilities)
// out32 (optional): write the f32 output instead of f16 (Q5_0 models quantize it to Q8_0)
void attn_encoder_softmax(hipStream_t s, const _Float16 * q, const _Float16 * k, const _Float16 * vt, int n_clips, int T,
                          int Tpad, int H, float scale, _Float16 * out, float * out32 = nullptr);
void attn_encoder(hipStream_t s, const _Float16 * q, const _Float16 * k, const _Float16 * vt,
                  int n_clips, int T, int Tpad, int H, float scale, int n_zero_pad, _Float16 * out,
                  float * out32 = nullptr);

// decoder attention row job: one query row attends over a list of KV rows in a given
// order with the reference flash-attention numerics (one_chunk: F16 V accumulator,
// ops.cpp:8140-8233; tiled: F32 accumulator, ops.cpp:8275-8546)
struct AttnRow {
    int q_row;          // row in q / out
    int kv_base;        // element offset of KV row 0 for this row's clip (layer-relative)
    int n_keys;         // number of listed key rows
    int key_list;       // offset into key_idx (cell indices, in reference visit order); -1 = 0..n_keys-1
    int n_zero_pad;     // trailing all-zero keys (cross attention padding)
    int mode;           // 0 = one_chunk (F16 accumulator), 1 = tiled (F32 accumulator), 2 = soft_max (no FA)
};
// ld_kv: elements between consecutive keys; hs: elements between consecutive heads (64 for
// the interleaved [cell][d] self-attention cache, n_keys * 64 for the head-major cross K/V)
void attn_decoder(hipStream_t s, const _Float16 * q, int ldq, const _Float16 * kbase, const _Float16 * vbase,
                  int ld_kv, int hs, const AttnRow * rows_dev, int n_rows, const int * key_idx, int H, float scale,
                  int max_keys, _Float16 * out, int ldo, bool any_one_chunk, bool any_tiled, float * out32 = nullptr,
                  bool oc_listed = true,  // false: every one_chunk row is a contiguous cell run
                  int8_t * q8 = nullptr, float * q8d = nullptr);  // one_chunk rows: Q8_0 of the f32 output
// rows with mode 2 (flash_attn = false contexts): soft_max attention, F16 probabilities;
// optional DTW capture of alignment-head probabilities cap[a][key][row] (amap: head -> a or -1)
void attn_decoder_softmax(hipStream_t s, const _Float16 * q, int ldq, const _Float16 * kbase, const _Float16 * vbase,
                          int ld_kv, int hs, const AttnRow * rows_dev, int n_rows, const int * key_idx, int H, float scale,
                          int max_keys, _Float16 * out, int ldo, const int * amap, float * cap, int cap_rows,
                          float * out32 = nullptr, float * ws = nullptr, size_t ws_floats = 0);
// workspace of the key-split soft_max form (ws non-null above): every (row, head) over ceil(keys / 128)
// blocks, probabilities bit-identical to the one-block kernel, P.V partials added in chunk order
size_t attn_softmax_ws_floats(int n_rows, int H);
// test hook: 256 / 1024 forces the single-block soft_max attention's width (0: by the pass size)
extern int attn_softmax_force_nt;
// test/bench hook: the one_chunk cross-attention kernels on contiguous head-major keys (ld 64):
// which = 1 the one-wave k_attn_step
void attn_cross_kernel(hipStream_t s, int which, const _Float16 * q, int ldq, const _Float16 * kbase,
                       const _Float16 * vbase, int hs, const AttnRow * rows_dev, int n_rows, int H, float scale,
                       _Float16 * out, int ldo);
int attn_max_listed_keys();  // per-row limit of the one_chunk kernel's key list
int attn_max_tiled_keys();   // per-row limit of the tiled decoder kernel

// ---------------------------------------------------------------------------------
// logits -> token (whisper_process_logits + whisper_sample_token, greedy)
// ---------------------------------------------------------------------------------
struct LogitJob {
    int row;               // logits row
    int flags;             // bit0 is_initial, bit1 last_was_ts, bit2 penult_was_ts, bit3 has_ts,
                           // bit4 suppress_blank, bit5 no_timestamps, bit6 tdrz, bit7 suppress_eot,
                           // bit8 need_nosp (no_speech prob of the raw logits)
    int ts_min;            // timestamps below token_beg + ts_min are masked (has_ts rule)
    float temperature;
};
struct VocabInfo {
    int n_vocab, eot, sot, solm, prev, nosp, not_, beg, translate, transcribe, space;
    int lang_begin, n_lang;
    int tid0_max;          // max initial timestamp index (max_initial_ts rule)
    const int * suppress_list; int n_suppress;  // suppress_nst token ids
};
struct TokenOut {
    int id, tid;
    float p, plog, pt, ptsum;
    float nosp_prob;
    float pad_;
};
// per-row maxima of raw logits rows
void logits_row_max(hipStream_t s, const float * logits, int n_rows, int n_vocab, float * out_dev);
void logits_copy_rows(hipStream_t s, const float * logits, int n_vocab, const int2 * map_dev, int n, float * dst);
void rowmax_update(hipStream_t s, const float * logits, int n_vocab, const int4 * ent_dev, int n, float * rmx,
                   int stride);
void nosp_probs(hipStream_t s, const float * row0, int n_vocab, const int2 * req_dev, int n, const float * rmx,
                int stride, int nosp, float * out_dev);
// processes logits in place (filters applied), writes logprobs/probs when requested. With a workspace of
// process_logits_ws_bytes(n_jobs) and no job needing the raw no-speech probability (any_nosp false),
// every row is split over several blocks (k_logits.hip); else one block per row.
size_t process_logits_ws_bytes(int n_jobs);
void process_logits(hipStream_t s, float * logits, int n_vocab, const LogitJob * jobs_dev, int n_jobs,
                    const VocabInfo & vi, TokenOut * out_dev, float * logprobs_out, float * probs_out,
                    bool any_nosp = true, void * ws = nullptr, size_t ws_bytes = 0);

// Silero VAD (k_vad.hip). Weights as the kernels read them: F16 conv weights transposed
// to [(ic * K + k)][OC] (im2col row order), W_ih transposed to [128][512], W_hh row-major.
struct VadWeights {
    const _Float16 * stft_T;    // [256][258]
    const _Float16 * enc_T[4];  // [(ic*3 + k)][OC]
    const float * enc_b[4];
    const float * ih_T;         // [128][512]
    const float * b_ih;
    const float * w_hh;         // [512][128]
    const float * b_hh;
    const _Float16 * wf;        // [128]
    const float * bf;           // [1]
};
// chunks of n_streams streams; chunk g reads pcm[pcm_off[s] + 512 * chunk_index[g] ...] of
// stream s = chunk_stream[g] (zero past pcm_len[s]); stream s owns chunks
// [stream_first[s], stream_first[s] + stream_n[s]) and LSTM state state[s][h(128) | c(128)]
void launch_vad(const VadWeights & w, const float * pcm, const int64_t * pcm_off, const int * pcm_len,
                const int * chunk_stream, const int * chunk_index, int n_chunks, const int * stream_first,
                const int * stream_n, int n_streams, float * ig, float * hist, float * state, float * probs,
                hipStream_t stream);

} // namespace owk
