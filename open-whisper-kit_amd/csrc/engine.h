// Batch-major device engine: mel -> conv -> encoder -> cross-KV for many clips at once,
// and batched decoder passes over rows drawn from any number of clips / decoders.
#pragma once

#include <functional>
#include <map>
#include <string>
#include <vector>

#include "kernels.h"
#include "model.h"

namespace owk {

// decode passes of at most whole_k_rows() rows run the whole-K residual + LayerNorm-prologue chain
// (engine.cpp launch_decode; bit-identical to the split chain), larger passes the split-K +
// resid_layernorm chain. Default 0: the whole-K chain measured slower at every row count
// (tools/chain_ab.py, profiles/archive/r04h_chain_ab.txt); the test hook keeps it verified bit-identical.
constexpr int kWholeKRowsDefault = 0;
int whole_k_rows();           // the current limit (kWholeKRowsDefault unless a test hook changed it)
int set_whole_k_rows(int n);  // test hook (owk_debug_set_whole_k_rows); returns the previous limit


// per-kernel-class HIP-event timing + algorithmic work counters
// eager launches with an event pair around each kernel-class launch on the engine stream; with a
// class selection (owk_prof_select) only the selected classes carry events: the host then stays
// ahead of the device and an event pair brackets its kernel alone (no host launch gap inside)
struct Prof {
    bool on = false;
    std::vector<std::string> only;  // empty: every class
    struct Rec {
        int cls;
        hipEvent_t a, b;
        double flops, bytes;
    };
    std::vector<std::string> names;
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    struct Tot {
        double ms = 0, flops = 0, bytes = 0;
        long n = 0;
    };
    std::vector<Tot> tot;
    std::string classes_csv;
    int cls_id(const char * name);
    hipEvent_t ev();
    void flush();
    void reset();
    ~Prof();
};

struct ProfScope {
    Prof * p;
    hipStream_t s;
    int cls = -1;
    hipEvent_t a = nullptr;
    double flops, bytes;
    ProfScope(Prof * p_, hipStream_t s_, const char * name, double flops_ = 0, double bytes_ = 0);
    ~ProfScope();
};

struct DecodeRow {
    int slot;        // clip slot (cross-KV / self-KV / mel owner)
    int token;
    int pos;
    int cell;        // self-KV cell receiving this token's K/V
    int key_off;     // visible self-attention cells: key_list[key_off .. key_off+n_keys)
    int n_keys;
    int mode_self;   // 0 one_chunk (F16 acc), 1 tiled (F32 acc), 2 soft_max (flash_attn = false)
    int mode_cross;
    int logit_row;   // -1: no logits for this row
};

// what a decoder pass launches (the key of its captured graph)
struct DecShape {
    int R, n_logit;
    bool self_oc, self_tl, cross_oc, cross_tl;  // attention kernels needed (one_chunk / tiled)
    int max_keys;
    bool self_sm = false, cross_sm = false;     // soft_max rows (flash_attn = false contexts)
    bool capture = false;                       // DTW: capture alignment-head cross-attention
    bool self_list = false;                     // a one_chunk self row whose cells are not one run
    int n_clips = 0;                            // distinct clips (cross K/V slots) among the rows: the
                                                // cross K/V a pass must read is per clip, not per row
};

// per-step bookkeeping of the emulated reference state->logits buffer (no-speech prob)
struct StepPost {
    std::vector<int4> rowmax;  // (slot, row, logit_row or -1, zero_fill)
    std::vector<int2> row0;    // (logit_row or -1 = zeros, slot)
    std::vector<int2> nosp;    // (slot, n_rows): no-speech prob over the slot's buffer
};

class Engine {
public:
    Engine(const Model * m, Prof * prof);
    ~Engine();

    const Model * m;
    Prof * prof;
    hipStream_t stream = nullptr;

    int cap_slots = 0;   // clip slots with cross-KV storage
    int kv_cells = 0;    // self-KV cells per slot
    // whisper_context_params.flash_attn: false selects the reference's soft_max attention
    // (encoder and decoder) -- the numerics DTW timestamps are defined with
    bool flash_attn = true;
    // whisper_full_params.audio_ctx of the current call (state->exp_n_audio_ctx, ref whisper.cpp:921,
    // 6986): 0 = the model's n_audio_ctx. The encoder runs over n_ctx() positions (2 * n_ctx() mel
    // frames), cross K/V hold n_ctx() rows per slot and decoder cross-attention attends over them.
    int audio_ctx = 0;
    int n_ctx() const { return audio_ctx > 0 && audio_ctx < m->hp.n_audio_ctx ? audio_ctx : m->hp.n_audio_ctx; }

    void reserve(int slots, int cells);

    // ---- mel ----
    // computes normalised log-mel for clips into slots[i]
    void compute_mel(const std::vector<int> & slots, const std::vector<const float *> & pcm,
                     const std::vector<int> & n_samples, bool pcm_on_device = false);
    void set_mel(int slot, const float * host, int n_len, int n_mel);
    int mel_len(int slot) const { return slot < (int) mel_len_.size() ? mel_len_[slot] : 0; }
    void download_mel(int slot, float * host) const;

    // ---- encoder + cross KV ----
    void encode(const std::vector<int> & slots, const std::vector<int> & offsets);
    // debug: f32 encoder output of the last encode (row-major [n*1500][d]) and cross KV
    void download_enc(int index, float * host) const;
    void download_cross(int slot, int layer, uint16_t * k_host, uint16_t * v_host) const;

    // ---- decoder ----
    // runs all rows through the decoder; raw logits for rows with logit_row >= 0 are
    // left on the device in logits_dev() [n_logit_rows][n_vocab]
    void decode(const std::vector<DecodeRow> & rows, const std::vector<int> & key_list, int n_logit_rows,
                bool capture = false);
    // DTW alignment heads (whisper.cpp:1160-1273): amap[layer * n_head + head] = global alignment-head
    // index (layer-major, preset order) or -1. A decode(..., capture = true) pass stores the f32
    // cross-attention probabilities of those heads; download_capture returns them for rows
    // [row0, row0 + n) as [head][key][row] (the reference's aheads_cross_QKs layout).
    void set_alignment_heads(const std::vector<int> & amap, int n_aheads);
    int n_aheads() const { return n_ah_; }
    void download_capture(int row0, int n, std::vector<float> & out) const;
    int capture_rows() const { return cap_rows_; }
    float * logits_dev() const { return logits_.as<float>(); }
    void download_logits(int logit_row, float * host) const;
    void upload_logits(int logit_row, const float * host);
    // after a decoder pass, ONE upload + ONE synchronisation: state->logits emulation
    // (row maxima, row 0, no-speech probabilities) and on-device whisper_process_logits +
    // greedy pick for every job; probs/logprobs are downloaded only when requested
    void step_post(const StepPost & post, const std::vector<LogitJob> & jobs, const VocabInfo & vi,
                   std::vector<TokenOut> & out, std::vector<float> & nosp_out, float * probs_host,
                   float * logprobs_host);
    // the emulated buffer of a slot <-> host copies (it persists with the whisper_state)
    void save_logits_state(int slot, int n_rows, std::vector<float> & rowmax, std::vector<float> & row0);
    void load_logits_state(int slot, const std::vector<float> & rowmax, const std::vector<float> & row0);
    static constexpr int RMX = 512;  // rows of the emulated buffer tracked per slot (>= n_text_ctx)

    void sync();

private:

    void launch_decode(const DecShape & sh);
    // the F16 <= 32-row chain (embedding, every layer) of rows [r0, r0 + n) on stream s with GEMM
    // workspace ws; attention kernels address rows by their absolute index (AttnRow.q_row)
    void fused_part(const DecShape & sh, int r0, int n, hipStream_t s, const GemmWs * ws);
    void launch_logits(const DecShape & sh);  // final LayerNorm of the logit rows + logits GEMM
    void stage_layout(int C, int KC);
    void clear_graphs();
    uint64_t buffers_signature() const;

    DevBuf row0_, rmx_;         // emulated state->logits: row 0 [slot][n_vocab], row maxima [slot][RMX]
    PinnedBuf post_h_, post_out_h_;
    DevBuf post_d_, post_out_d_;
    // slot storage
    DevBuf cross_k_, cross_v_;   // [L][cap_slots][n_audio_ctx][d]
    DevBuf self_k_, self_v_;     // [L][cap_slots][head][kv_cells][64] (head-major)
    std::vector<DevBuf *> mel_;  // per slot [n_mel][n_len]
    std::vector<int> mel_len_;

    // encoder workspace
    DevBuf e_a1_, e_c1_, e_a2_, e_x_, e_xn_, e_q_, e_k_, e_vt_, e_ao_, e_h_, e_enc_, e_enc32_;
    DevBuf e_win_, e_slotmap_;
    DevBuf e_rmul_;                       // encoder rows' Q8_K rounding path (K-quants, repacked formats)
    const uint8_t * kq_rmul_ = nullptr;   // the rows' path of the linears being issued (null: all fma)
    int enc_rows_cap_ = 0;
    int last_enc_n_ = 0;
    int vt_T_ = 0;  // n_ctx() the transposed-V buffer was zeroed for

    // decoder workspace
    DevBuf d_x_, d_xn_, d_q_, d_ao_, d_h_, d_xl_;
    DevBuf logits_, lg_probs_, lg_lp_, lg_ws_;
    int dec_rows_cap_ = 0, dec_keys_cap_ = 0;
    PinnedBuf stg_;   // host image of the per-pass inputs
    DevBuf d_stg_;    // its device copy (fixed sections, see stage_layout)
    size_t st_tok_ = 0, st_pos_ = 0, st_rowoff_ = 0, st_rs_ = 0, st_rc_ = 0, st_lsel_ = 0, st_keys_ = 0, st_bytes_ = 0;
    size_t st_rmul_ = 0;  // K-quants (repacked formats): per-row Q8_K rounding path (quantize_q8k_f16)
    std::map<uint64_t, hipGraphExec_t> graphs_;
    uint64_t graphs_sig_ = 0;
    hipGraphExec_t graph_for(uint64_t key, hipStream_t s, const std::function<void()> & launch);

    // Q5_0 models: f32 activations feeding the quantized GEMMs and their Q8_0 copy
    void linear(const char * cls, int mode, int M, int N, int K, const _Float16 * A16, const float * A32, int lda,
                const _Float16 * W, const Q5W & q, const EpiParams & ep, const _Float16 * Wt = nullptr,
                bool dec = false,
                bool a_q8 = false, const int8_t * qa = nullptr, const float * qd = nullptr);
    DevBuf q8a_, q8d_;
    DevBuf q8h_, q8hd_;  // Q8_0 rows of the GELU output (MLP0 epilogue -> MLP1 operand; decode passes <= 32 rows)
    DevBuf q16a_, q16d_;  // gemm_q16 operands: Q8_0 integers as f16 [M][K], scales [K/32][mpad]
    // Q5_0 models: the Q8_0 activation buffers producers write for the next linear (else null)
    // Q8_0 / Q8_1 rows written by producers (LayerNorm, attention); K-quant models quantize to Q8_K
    // in linear() from the f32 rows instead
    int8_t * q8a() { return m->q5 && !m->kq ? q8a_.as<int8_t>() : nullptr; }
    float * q8d() { return m->q5 && !m->kq ? q8d_.as<float>() : nullptr; }
    DevBuf e_xn32_, e_ao32_, d_xn32_, d_ao32_, d_xl32_;

    DevBuf sm_ws_;       // key-split soft_max attention workspace (flash_attn = false passes)
    DevBuf amap_, cap_;  // DTW: head map [L][H], captured probabilities [n_ah][T][cap_rows_]
    int n_ah_ = 0, cap_rows_ = 0;

    DevBuf mel_jobs_, pcm_tmp_;
    DevBuf gws_part_;  // split-K workspace of the decode-row GEMMs
    GemmWs gws_;
};

} // namespace owk
