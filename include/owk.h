/*
 * owk.h -- MI355X engine extensions beyond the reference whisper.h ABI.
 *
 * The reference processes one clip per whisper_full() call (ref src/whisper.cpp:7778).
 * The MI355X engine is batch-major: owk_full_batch() runs N independent clips
 * through one stage-major pipeline (batched mel -> conv -> encoder -> cross-KV ->
 * decoder steps), each clip with its own whisper_state holding results readable with
 * the standard whisper_full_*_from_state() getters. Per-clip decoding semantics are
 * exactly those of whisper_full_with_state (ref src/whisper.cpp:6827-7776).
 */
#ifndef OWK_H
#define OWK_H

#include "whisper.h"

#ifdef __cplusplus
extern "C" {
#endif

/* extra per-call options (all-zero = reference behaviour) */
struct owk_full_ext {
    /* fixed-work mode for throughput runs: mask <|endoftext|> on the device, equivalent
     * to a logits_filter_callback doing logits[eot] = -INF (ref whisper.cpp:6254-6256) */
    int suppress_eot;
    /* samples[i] are device pointers (f32, on the context's GPU) instead of host memory:
     * lets a caller keep the audio resident in HBM (bench.py times the pipeline this way) */
    int samples_on_device;
    int reserved[6];
};

/* run n_clips clips; states[i] receives clip i's segments. Returns 0 if every clip
 * succeeded, else the first non-zero whisper_full error code. */
WHISPER_API int owk_full_batch(struct whisper_context * ctx, struct whisper_state ** states,
                               struct whisper_full_params params, const struct owk_full_ext * ext,
                               const float * const * samples, const int * n_samples, int n_clips);

/* Silero VAD over n_streams independent streams in one device pass (all chunks encoded
 * together, one LSTM workgroup per stream, each stream from a zero state): probs_out[s]
 * receives ceil(n_samples[s] / 512) speech probabilities, the values
 * whisper_vad_detect_speech would give for that stream alone. Returns 0 on success. */
WHISPER_API int owk_vad_detect_batch(struct whisper_vad_context * vctx, const float * const * samples,
                                     const int * n_samples, int n_streams, float * const * probs_out);
/* test hook (host only): whisper_vad_segments_from_probs on a caller's probabilities;
 * writes [start_cs, end_cs] pairs (up to cap) and returns the segment count */
WHISPER_API int owk_vad_segments_raw(const float * probs, int n_probs, int n_window, struct whisper_vad_params params,
                                     int64_t * out_cs, int cap);

/* per-kernel-class device timing with HIP events recorded on the engine stream (eager launches
 * while enabled: captured graphs cannot carry timing events) */
WHISPER_API void owk_prof_enable(struct whisper_context * ctx, int enable);
/* time only these kernel classes (comma-separated; NULL or "" = all): the other launches carry no
 * events, so the host stays ahead of the device and each event pair brackets its kernel alone */
WHISPER_API void owk_prof_select(struct whisper_context * ctx, const char * classes);
WHISPER_API void owk_prof_reset(struct whisper_context * ctx);
/* total device milliseconds and launch count of one kernel class since reset;
 * returns 0 if the class is known */
WHISPER_API int owk_prof_read(struct whisper_context * ctx, const char * kernel_class, double * total_ms, long * launches);
/* algorithmic work (flops, bytes) the engine attributes to a kernel class since reset */
WHISPER_API int owk_prof_work(struct whisper_context * ctx, const char * kernel_class, double * flops, double * bytes);
/* comma-separated list of kernel classes seen since reset (owned by ctx) */
WHISPER_API const char * owk_prof_classes(struct whisper_context * ctx);

/* test hooks: intermediates of the last staged call on a state
 * (mel [n_mel][n_len] f32; encoder output [n_audio_ctx][d] f32; cross K/V f16 bits) */
WHISPER_API int owk_debug_mel(struct whisper_state * st, float * out, int cap);
WHISPER_API int owk_debug_enc(struct whisper_context * ctx, struct whisper_state * st, int index, float * out, int cap);
WHISPER_API int owk_debug_cross(struct whisper_context * ctx, struct whisper_state * st, int slot, int layer,
                                uint16_t * k, uint16_t * v);
WHISPER_API const uint16_t * owk_debug_gelu_table(void);
/* test hook (host only): whisper_tokenize on the vocabulary of the model file at path_model (only
 * its header, mel filters and vocabulary are read). Returns the token count (written to out when
 * it fits cap), -count when it does not, INT32_MIN when the file cannot be parsed. */
WHISPER_API int owk_debug_tokenize(const char * path_model, const char * text, int * out, int cap);
/* test hook (host only): the self-attention KV-cell allocator (csrc/kv_cells.h, the reference's
 * whisper_kv_cache_find_slot / _seq_rm / _seq_cp / _cell_max, ref whisper.cpp:1019-1137) driven by a
 * script of n_ops records of 5 ints (op, a, b, c, d) on n_ctx cells:
 *   0 find_slot of a tokens at positions c .. c + a - 1 of sequence b (result: first cell or -1)
 *   1 seq_rm(seq a, p0 b, p1 c)   2 seq_cp(src a, dst b, p0 c, p1 d)   3 cell_max (result)   4 clear
 * out: the n_ops results, the head, then (pos, sequence bitmask) per cell. Returns the ints written
 * (n_ops + 1 + 2 n_ctx), -1 if cap is too small, -2 on an invalid record. */
WHISPER_API int owk_debug_kv_cells(int n_ctx, const int * ops, int n_ops, int * out, int cap);
/* out[M][N] = A[M][K] . W[N][K]^T (f16 bits in, f32 out) through the engine's GEMM dispatch */
WHISPER_API int owk_debug_gemm(int device, int M, int N, int K, const uint16_t * a, const uint16_t * w, float * out);
// one large-tile epilogue mode through the 128x128 and 256x256 kernels on the same random operands: max |diff|
// (mode alone or | 0x800: the 8-phase 256x256 kernel; | 0x1000 / 0x2000: the 64x64 / 32x32 ring tile of
// mid-size GEMMs against the 128x128 tile)
WHISPER_API double owk_debug_gemm_epi_diff(int device, int mode, int M, int N, int K, int d, int T);
/* average microseconds per launch of `iters` back-to-back engine GEMMs (epilogue `mode`, zero data) */
/* test hook (host only): the DTW alignment of captured alignment-head attention
 * cap[(head * n_audio_ctx + j) * n_tok + t] (the reference's aheads_cross_QKs layout), as
 * the time index of each text token the reference's placement loop assigns, in order
 * (whisper_exp_compute_token_level_timestamps_dtw, ref src/whisper.cpp:8837-8998).
 * Returns the count written (<= cap_out) or -1. */
WHISPER_API int owk_debug_dtw(const float * cap, int n_ah, int n_audio_ctx, int n_tok, int sot_len, int n_frames,
                              int medfilt, int * out, int cap_out);
/* test hook (host only): the GBNF constraint of grammar.cpp (ref whisper.cpp:5498-5905) on a caller's
 * rules and vocabulary (vocab[id] = token text, ids < eot are the text tokens): accept the n_accept
 * tokens, then write the ids the constraint penalises (up to cap); returns their count, -1 on error */
WHISPER_API int owk_debug_grammar_rejects(const whisper_grammar_element ** rules, size_t n_rules, size_t i_start_rule,
                                          const char * const * vocab, int n_vocab, int eot, const int * accept,
                                          int n_accept, int * out, int cap);
/* test hook: alignment-head probabilities captured by the state's last DTW re-decode,
 * [head][n_audio_ctx][rows of that pass]; returns the float count (copies when out != NULL) */
WHISPER_API long owk_debug_capture(struct whisper_state * state, float * out, long cap);
/* test hook: out[M][N] = Q8_0(a) . Q5_0(w)^T through the engine's quantize + Q5 GEMM; a f32 [M][K],
 * w_blocks ggml block_q5_0 rows [N][K/32]; q_out / d_out (optional) receive the Q8_0 activations */
WHISPER_API int owk_debug_gemm_q5(int device, int M, int N, int K, const float * a, const uint8_t * w_blocks, float * out,
                                  int8_t * q_out, float * d_out);
/* the same for any block format fmt (0 Q5_0, 1 Q8_0, 2 Q4_0, 3 Q4_1, 4 Q5_1: w_blocks are ggml blocks
 * of that type; Q4_1 / Q5_1 take Q8_1 activations); d_out receives the raw f32 activation scales.
 * fmt 5..9 = Q2_K, Q3_K, Q4_K, Q5_K, Q6_K (K % 256 == 0; Q8_K activations, the K-quant model path at
 * every M): q_out receives the activation rows in the virtual-block layout [M][kx] (kx = K * 9/8 for
 * Q2_K / Q4_K / Q5_K, K for Q3_K, 2K for Q6_K), d_out the Q8_K scale per row and 256-block [M][K/256] */
WHISPER_API int owk_debug_gemm_quant(int device, int fmt, int M, int N, int K, const float * a, const uint8_t * w_blocks,
                                     float * out, int8_t * q_out, float * d_out);
// use_q16 = 1: the large-tile encoder path (expanded f16 integers, gemm_q16; M >= 2048, symmetric formats);
// use_q16 = 2: the MLP0 decode-row form (M <= 32, N % 32 == 0): EPI_GELU_F16 with an identity GELU table,
// out = the f16 outputs as f32, q_out [M][N] / d_out [M][N/32] = the Q8_0 rows its epilogue writes
WHISPER_API int owk_debug_gemm_quant2(int device, int fmt, int M, int N, int K, const float * a, const uint8_t * w_blocks,
                                      float * out, int8_t * q_out, float * d_out, int use_q16);
/* host-only test hook (no device): N rows of ggml K-quant blocks (fmt 5..9 as above) -> the virtual-block
 * expansion the GEMMs run on (wi [N][kx] f16 bits, dwt [kx/32][N] f32; either may be NULL) and the f32
 * row dequantization of the token embedding (deq [N][K], may be NULL); 0 on success */
WHISPER_API int owk_debug_kquant(int fmt, int N, int K, const uint8_t * w_blocks, uint16_t * wi, float * dwt, float * deq);
/* mode | 0x100: force the 128x128 large-GEMM kernel; (default, or | 0x800) the 8-phase 256x256 kernel; | 0x1000 / 0x2000: the 64x64 / 32x32 ring tile;
 * | 0x200: uniform random operands (else zeros) */
WHISPER_API double owk_debug_gemm_bench(int device, int mode, int M, int N, int K, int iters);
/* the decoder's per-layer matmul + residual/LayerNorm chain (no attention) of a large-v3-shaped model,
 * R rows, distinct random weights per layer, one captured hipGraph: device microseconds per layer */
WHISPER_API double owk_debug_decode_chain(int device, int R, int n_layers, int iters);
/* the same with the chain's form chosen by `variant` (whisper_api.cpp: 0 round-3 split-K + resid_layernorm,
 * 1 LayerNorm-prologue consumers + whole-K residual epilogues, 2 = 1 without the prologue statistics
 * (timing only), 3 / 4 mixed) */
WHISPER_API double owk_debug_decode_chain2(int device, int R, int n_layers, int iters, int variant);

/* test hook: the decoder's LayerNorm-prologue GEMM (M <= 32 rows, K <= 1280) against layernorm + GEMM, EPI_F16
 * with bias b (may be NULL), f16 bits out [M][N]; with w2 / resid (may be NULL): the whole-K residual epilogue of
 * an [N][4N] matmul against split-K partials + resid_layernorm, f32 [M][N] each (out_resid_* may be NULL) */
WHISPER_API int owk_debug_gemm_rows_ln(int device, int M, int N, int K, const float * x, const float * lnw,
                                       const float * lnb, const float * b, const uint16_t * w, uint16_t * out_fused,
                                       uint16_t * out_ref, const uint16_t * w2, const float * resid,
                                       float * out_resid_full, float * out_resid_split);
/* test hook: decode passes of at most n rows run the whole-K decoder chain (0 = never; bit-identical to the
 * split-K chain by construction); returns the previous limit */
WHISPER_API int owk_debug_set_whole_k_rows(int n);
/* soft_max decoder attention on random data: key-split form (split != 0) or single-block kernel; R rows x H
 * (>= 4) heads x T keys, heads 0..3 captured as alignment heads; out [R][H*64] f16, cap [4][T][R] f32
 * (either may be null); returns us per call over iters timed calls (-1: error) */
WHISPER_API double owk_debug_attn_softmax(int device, int split, int R, int H, int T, uint16_t * out, float * cap,
                                          int iters);
/* library identity: 1 when the gfx950 HIP code object is present and a device is usable */
WHISPER_API int owk_device_ok(int device);
WHISPER_API const char * owk_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* OWK_H */
