// Internal definitions of whisper_context / whisper_state for the MI355X engine.
#pragma once

#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "engine.h"
#include "grammar.h"
#include "kv_cells.h"
#include "model.h"
#include "owk.h"
#include "whisper.h"

namespace owk {

struct Segment {
    int64_t t0 = 0, t1 = 0;
    std::string text;
    float no_speech_prob = 0.0f;
    std::vector<whisper_token_data> tokens;
    bool speaker_turn_next = false;
};

// whisper_sequence (ref src/whisper.cpp:783-794)
struct Sequence {
    std::vector<whisper_token_data> tokens;
    int result_len = 0;
    double sum_logprobs_all = 0, sum_logprobs = 0, avg_logprobs = 0, entropy = 0, score = 0;
};

// whisper_decoder (ref 797-820)
struct Decoder {
    Sequence sequence;
    int i_batch = 0;        // logits row of this decoder in the current decode call
    int seek_delta = 0;
    bool failed = false, completed = false, has_ts = false;
    std::vector<float> probs, logits, logprobs;  // host copies (sampling / beam / callback paths)
    TokenOut gtok{};        // device-side greedy pick for the current logits
    std::mt19937 rng;
    Grammar grammar;        // GBNF parse state (whisper_full_params.grammar_rules)
};

constexpr int MAX_DECODERS = 8;  // WHISPER_MAX_DECODERS (ref 142)

} // namespace owk

struct whisper_state {
    std::unique_ptr<owk::Engine> eng;
    int64_t t_sample_us = 0, t_encode_us = 0, t_decode_us = 0, t_batchd_us = 0, t_prompt_us = 0, t_mel_us = 0;
    int32_t n_sample = 0, n_encode = 0, n_decode = 0, n_batchd = 0, n_prompt = 0, n_fail_p = 0, n_fail_h = 0;
    int32_t kv_self_n_dec = 1;
    owk::KvCells kv;  // cell map of slot 0 (staged API) / of this clip in batch mode
    int mel_n_len = 0, mel_n_len_org = 0, mel_n_mel = 0;
    std::vector<float> logits;  // whisper_get_logits
    // emulated reference state->logits buffer (only what the no-speech probability reads):
    // its row count, per-row maxima and row 0; live on the device during a call, host
    // copies persist with the state between calls
    int logits_rows = 0;
    std::vector<float> logits_rowmax;
    std::vector<float> logits_row0;
    std::vector<owk::Segment> result_all;
    std::vector<whisper_token> prompt_past0, prompt_past1;
    int lang_id = 0;
    // whisper_full_params.audio_ctx of the last whisper_full (ref exp_n_audio_ctx, whisper.cpp:921):
    // the staged whisper_encode / whisper_decode calls keep using it, as in the reference
    int exp_n_audio_ctx = 0;
    owk::Decoder decoders[owk::MAX_DECODERS];
    float no_speech_prob = 0.0f;
    std::vector<float> energy;
    int64_t t_beg = 0, t_last = 0;
    whisper_token tid_last = 0;
    // context_params.flash_attn of the owning context (selects the attention numerics)
    bool flash_attn = true;
    // DTW alignment heads (dtw_token_timestamps): [layer][head] -> global index or -1
    std::vector<int> dtw_amap;
    int dtw_n_ah = 0;
    // whisper_full's VAD pre-pass (ref whisper.cpp:923-932, 6643-6826): the state's own VAD
    // context and the processed -> original centisecond table the segment getters apply
    whisper_vad_context * vad_context = nullptr;
    bool has_vad_segments = false;
    std::vector<std::pair<int64_t, int64_t>> vad_map;
    // held by a whisper_full / owk_full_batch call that uses this state (its engine and results):
    // calls on different states of one context run concurrently, as the reference allows
    std::mutex mu;
};

struct whisper_context {
    int64_t t_load_us = 0, t_start_us = 0;
    whisper_context_params params{};
    std::unique_ptr<owk::Model> model;
    whisper_state * state = nullptr;
    std::string path_model;
    owk::Prof prof;
    std::mutex mu;  // whisper_full calls while the per-kernel recorder (prof, shared) is on
    whisper_timings timings{};
};

namespace owk {
int64_t time_us();
owk::VocabInfo vocab_info(const whisper_context * ctx, const whisper_full_params & p, std::vector<int> & suppress);
struct CallToken {  // one token of a reference decode call (whisper_batch entry)
    int token, pos, seq;
    bool logits;
};
// allocate KV cells for one reference decode call of one clip and emit engine rows
int prepare_decode_call(whisper_state * st, int slot, const std::vector<CallToken> & toks,
                        std::vector<DecodeRow> & rows, std::vector<int> & keys, int & n_logit);
// alignment heads of a context (ref get_alignment_heads_by_layer 8688-8707 / aheads_masks_init
// 1160-1273): amap[layer * n_head + head] = index in layer-major preset order, or -1.
// Returns false (with a logged error) on an invalid preset, like aheads_masks_init.
bool alignment_heads(const whisper_context * ctx, std::vector<int> & amap, int & n_ah);
// DTW time index of each text token placed by the path (timestamps.cpp)
std::vector<int32_t> dtw_time_indices(const float * cap, int n_ah, int n_audio_ctx, int n_tok, int sot_len, int n_frames,
                                      int medfilt);
// DTW token timestamps of segments [i_segment, i_segment + n_segments) (timestamps.cpp)
void dtw_timestamps(whisper_context * ctx, whisper_state * st, int i_segment, int n_segments, int seek, int n_frames,
                    int medfilt, const std::vector<float> & cap, int n_ah, int n_audio_ctx, int n_tok, int sot_len);
// configure a state's engine for its context (attention mode, alignment heads)
void configure_engine(const whisper_context * ctx, whisper_state * st);
// Silero VAD (vad.cpp)
bool vad_filter(whisper_context * ctx, whisper_state * state, const whisper_full_params & params, const float * samples,
                int n_samples, std::vector<float> & filtered);
int64_t vad_map_time(int64_t t, const std::vector<std::pair<int64_t, int64_t>> & map);
int full_batch(whisper_context * ctx, whisper_state ** states, const whisper_full_params * params,
               const owk_full_ext * ext, const float * const * samples, const int * n_samples, int n_clips);
} // namespace owk
