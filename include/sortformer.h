/*
 * sortformer.h -- drop-in C ABI of the MI355X streaming-SortFormer diarizer
 * (libsortformer.so).
 *
 * Every declaration replaces the identically named one of the reference header
 * /root/reference streaming-sortformer/src/sortformer.h (cited "ref:<line>"): same
 * names, struct layouts, enum values, return conventions and ownership, so
 * sortformer-cli, test-streaming-api, the Swift SDK bridge and the node addon link
 * unchanged. Plain C, no export macro (ref:1-8).
 *
 * Ownership: buffers returned through `float **` are malloc'd and released by the
 * caller with free() (ref:38-121). A context is NOT re-entrant (ref sortformer.cpp:
 * 140-142); one HIP stream per context. A stream state holds a non-owning context
 * pointer (ref sortformer.cpp:2677).
 */
#ifndef SORTFORMER_H
#define SORTFORMER_H

#ifdef __cplusplus
extern "C" {
#endif

struct sortformer_context;

/* ref:11-21 */
struct sortformer_params {
    int   chunk_len;              /* 188 */
    int   right_context;          /* 1 */
    int   fifo_len;               /* 0 */
    int   spkcache_len;           /* 188 */
    int   spkcache_update_period; /* 188 */
    float threshold;              /* 0.5 */
    int   median_filter;          /* 11 */
    int   n_threads;              /* 4 (host threads; the model runs on the GPU) */
    int   chunk_left_context;     /* 1 */
};

struct sortformer_params sortformer_default_params(void);                                        /* ref:23 */

/* GGUF model -> device-resident weights; NULL on error (ref:25) */
struct sortformer_context * sortformer_init(const char * model_path, struct sortformer_params params);

void sortformer_free(struct sortformer_context * ctx);                                           /* ref:27 */

/* 16 kHz mono PCM16 WAV -> malloc'd float samples; sample count or -1 (ref:29-32) */
int sortformer_load_wav(const char * path, float ** samples_out);

/* log-mel [n_mels][T] (T padded to a multiple of 16); returns T or -1 (ref:34-47) */
int sortformer_compute_mel(struct sortformer_context * ctx, const float * samples, int n_samples,
                           float ** mel_out, int * n_mels_out, int * seq_len_out);

/* conv2d subsampling (x8) + linear -> [T_out][d_model]; returns T_out or -1 (ref:49-63) */
int sortformer_compute_preenc(struct sortformer_context * ctx, const float * mel_data, int n_mels,
                              int n_mel_frames, int seq_len, float ** preenc_out, int * d_model_out);

/* conformer layers 0..target_layer -> [T][d_model]; returns T or -1 (ref:65-77) */
int sortformer_compute_conformer(struct sortformer_context * ctx, const float * preenc_data, int T,
                                 int d_model, int target_layer, float ** conf_out);

/* 512 -> 192 projection; returns T or -1 (ref:79-89) */
int sortformer_compute_projection(struct sortformer_context * ctx, const float * conf_data, int T,
                                  int d_model_in, float ** proj_out, int * d_model_out_ptr);

/* transformer layers 0..target_layer -> [T][192]; returns T or -1 (ref:91-103) */
int sortformer_compute_transformer(struct sortformer_context * ctx, const float * proj_data, int T,
                                   int d_model, int target_layer, float ** trans_out);

/* prediction head -> sigmoid probabilities [T][4]; returns T or -1 (ref:105-114) */
int sortformer_compute_prediction(struct sortformer_context * ctx, const float * trans_data, int T,
                                  int d_model, float ** pred_out);

/* streaming (AOSC speaker-cache) diarization of a whole clip; frames written or -1 (ref:116-124) */
int sortformer_diarize(struct sortformer_context * ctx, const float * audio_samples, int n_samples,
                       float * probs_out, int n_frames_max);

/* probabilities -> RTTM text; bytes written or -1 (buffer too small) (ref:126-136) */
int sortformer_to_rttm(const float * probs, int n_frames, float threshold, int median_filter,
                       const char * filename, char * rttm_out, int rttm_out_size);

/* ---- streaming API (ref:138-206) ---- */
struct sortformer_stream_state;

enum sortformer_stream_preset {
    SORTFORMER_PRESET_LOW_LATENCY = 0,
    SORTFORMER_PRESET_2S          = 1,
    SORTFORMER_PRESET_3S          = 2,
    SORTFORMER_PRESET_5S          = 3,
};

struct sortformer_stream_params {
    int chunk_len;
    int right_context;
    int left_context;
    int fifo_len;
    int spkcache_len;
    int spkcache_update_period;
};

struct sortformer_stream_params sortformer_stream_preset_params(enum sortformer_stream_preset preset);

struct sortformer_stream_state * sortformer_stream_init(struct sortformer_context * ctx,
                                                        enum sortformer_stream_preset preset);

struct sortformer_stream_state * sortformer_stream_init_with_params(struct sortformer_context * ctx,
                                                                    struct sortformer_stream_params params);

/* new frames written (probs_out_max counts frames) or -1 (ref:184-191, sortformer.cpp:3105) */
int sortformer_stream_feed(struct sortformer_stream_state * st, const float * audio_samples, int n_samples,
                           float * probs_out, int probs_out_max);

int sortformer_stream_flush(struct sortformer_stream_state * st, float * probs_out, int probs_out_max);

void sortformer_stream_reset(struct sortformer_stream_state * st);

void sortformer_stream_free(struct sortformer_stream_state * st);

#ifdef __cplusplus
}
#endif

#endif /* SORTFORMER_H */
