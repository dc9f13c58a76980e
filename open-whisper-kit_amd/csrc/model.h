// Whisper model: ggml-bin loader (host) and the device-resident weight set.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "whisper.h"

namespace owk {

struct HParams {
    int32_t n_vocab = 51864, n_audio_ctx = 1500, n_audio_state = 384, n_audio_head = 6, n_audio_layer = 4;
    int32_t n_text_ctx = 448, n_text_state = 384, n_text_head = 6, n_text_layer = 4, n_mels = 80, ftype = 1;
    float eps = 1e-5f;
};

enum ModelType { MODEL_UNKNOWN, MODEL_TINY, MODEL_BASE, MODEL_SMALL, MODEL_MEDIUM, MODEL_LARGE };

// special-token layout: whisper_model_load vocab section, ref src/whisper.cpp:1589-1675
struct Vocab {
    int n_vocab = 51864;
    std::map<std::string, int> token_to_id;
    std::vector<std::string> id_to_token;
    int eot = 50256, sot = 50257, translate = 50357, transcribe = 50358, solm = 50359, prev = 50360,
        nosp = 50361, not_ = 50362, beg = 50363;
    bool is_multilingual() const { return n_vocab >= 51865; }
    int num_languages() const { return n_vocab - 51765 - (is_multilingual() ? 1 : 0); }
};

// language table (ISO code -> id, English name); iteration order of std::map matters
// for whisper_lang_auto_detect tie behaviour (ref whisper.cpp:280-381, 4055-4066)
const std::map<std::string, std::pair<int, std::string>> & languages();

struct EncLayerW {
    const float *attn_ln_w, *attn_ln_b, *mlp_ln_w, *mlp_ln_b;
    const _Float16 *w_qkv;  // [3d][d]: query, key, value rows
    const float *b_q, *b_v;
    const _Float16 *w_o;
    const float *b_o;
    const _Float16 *w_mlp0, *w_mlp1;
    const float *b_mlp0, *b_mlp1;
    Q5W q_qkv, q_o, q_mlp0, q_mlp1;  // Q5_0 models (the F16 pointers are null then)
};

struct DecLayerW {
    const float *attn_ln_w, *attn_ln_b, *cross_ln_w, *cross_ln_b, *mlp_ln_w, *mlp_ln_b;
    const _Float16 *w_qkv;  // self attention [3d][d]
    const float *b_q, *b_v;
    const _Float16 *w_o;
    const float *b_o;
    const _Float16 *cw_q;   // cross query [d][d]
    const float *cb_q;
    const _Float16 *cw_kv;  // cross key + value [2d][d]
    const float *cb_v;
    const _Float16 *cw_o;
    const float *cb_o;
    const _Float16 *w_mlp0, *w_mlp1;
    const float *b_mlp0, *b_mlp1;
    // tiled copies for the decode-row GEMM (tile_weights layout)
    const _Float16 *t_qkv, *t_o, *t_cq, *t_co, *t_mlp0, *t_mlp1;
    Q5W q_qkv, q_o, q_cq, q_ckv, q_co, q_mlp0, q_mlp1;  // Q5_0 models
};

struct Model {
    HParams hp;
    ModelType type = MODEL_UNKNOWN;
    Vocab vocab;
    int n_filters_mel = 0, n_filters_fft = 0;
    std::vector<float> filters;  // host copy [n_mel][n_fft]
    int n_loaded = 0;
    int kpad_conv1 = 0;          // conv1 GEMM K padded to a multiple of 64

    // device weights: one allocation
    DevBuf blob;
    const _Float16 * conv1_w = nullptr;  // [d][kpad_conv1]
    const float * conv1_b = nullptr;
    const _Float16 * conv2_w = nullptr;  // [d][3d]
    const float * conv2_b = nullptr;
    const float * e_pe = nullptr;        // [n_audio_ctx][d]
    const float *e_ln_w = nullptr, *e_ln_b = nullptr;
    std::vector<EncLayerW> enc;
    bool q5 = false;                     // quantized model (MOSTLY_Q5_0/Q8_0/Q4_0/Q4_1/Q5_1): 2-D linears (and d_te) are Q5W
    int qfmt = 0;                        // their block format (kernels.h QFmt)
    DevBuf q5blob;
    DevBuf q16blob;  // Q5W::wi / dwt of the encoder and cross-K/V matrices (symmetric formats)
    bool kq = false;                     // K-quant model (MOSTLY_Q2_K .. Q6_K, kquant.h): every 2-D linear
                                         // as Q5W::wi / dwt in q16blob, the embedding rows dequantized
    DevBuf te32;                         // K-quants: token embedding [n_vocab][d] f32 (dequantize_row_q*_K)
    Q5W q_te;
    const _Float16 * d_te = nullptr;     // [n_vocab][d]
    const _Float16 * d_te_t = nullptr;   // tiled copy (logits of decode steps)
    DevBuf tiled;                        // all tiled decoder weights
    const float * d_pe = nullptr;        // [n_text_ctx][d]
    const float *d_ln_w = nullptr, *d_ln_b = nullptr;
    std::vector<DecLayerW> dec;

    // device constants
    const uint16_t * gelu_tab = nullptr;  // 65536 f16 entries
    const float * mel_filters = nullptr;  // [n_mel][201]
    const int * mel_rng = nullptr;        // [n_mel][2]: nonzero bin range [lo, hi) of each filter
    const double * twiddle = nullptr;     // cos[400], sin[400]
    const float * hann = nullptr;         // [400]
    int device = 0;
};

// parse a ggml-bin model through a whisper_model_loader and upload it to `device`.
// Returns nullptr (after logging) on malformed input, like whisper_model_load.
// vocab_only: stop after the header, mel filters and vocabulary (host only, no device touched)
Model * load_model(whisper_model_loader * loader, int device, std::string & err, bool vocab_only = false);

// whisper_tokenize's algorithm on a vocabulary (regex word split + greedy longest match,
// ref whisper.cpp:3272-3320)
std::vector<int> tokenize_text(const Vocab & v, const std::string & text);

void log_msg(ggml_log_level level, const char * fmt, ...) __attribute__((format(printf, 2, 3)));

} // namespace owk
