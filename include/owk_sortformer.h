/* MI355X extensions of the streaming-SortFormer C ABI (libsortformer.so).
 * include/sortformer.h stays the reference's interface (ref/streaming-sortformer/src/sortformer.h);
 * this header adds what the GPU engine can do beyond it. Plain C. */
#ifndef OWK_SORTFORMER_H
#define OWK_SORTFORMER_H

#include "sortformer.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Feed n_streams live streams of ONE context at once (many streams per
 * GPU). Stream i gets samples[i][0 .. n_samples[i]) exactly as sortformer_stream_feed(ssts[i],
 * ...) would, and n_out[i] frames of 4 speaker probabilities are written to probs_out[i]
 * (at most probs_out_max[i] frames). The pending chunks of all streams are processed in
 * rounds, each round one GPU head pass over the stacked inputs of its streams. Each state
 * may appear once per call. Returns 0, or -1 on invalid arguments / device errors. */
int owk_sortformer_stream_feed_batch(struct sortformer_stream_state ** states, const float * const * samples,
                                     const int * n_samples, int n_streams, float * const * probs_out,
                                     const int * probs_out_max, int * n_out);

/* test hook (host only, no device): the streaming state's AOSC speaker-cache bookkeeping as
 * sortformer_stream_feed runs it (ref streaming-sortformer/src/sortformer.cpp:1729-1752 update of the
 * silence profile from n_pop popped FIFO frames, then 1783-1920 compression of an n_frames cache to
 * spkcache_len frames). embs [n_frames][d], preds [n_frames][4], mean_sil [d] after n_sil silent
 * frames; outputs out_embs [spkcache_len][d], out_preds [spkcache_len][4], out_mean_sil [d]. Returns
 * spkcache_len, -1 when n_frames <= spkcache_len (no compression; out_mean_sil still written), -2 on
 * invalid arguments. */
int owk_sortformer_debug_aosc(int d, int n_frames, const float * embs, const float * preds, const float * mean_sil,
                              int n_sil, int n_pop, const float * pop_embs, const float * pop_preds, int spkcache_len,
                              int sil_frames_per_spk, float * out_embs, float * out_preds, float * out_mean_sil);

#ifdef __cplusplus
}
#endif

#endif /* OWK_SORTFORMER_H */
