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

#ifdef __cplusplus
}
#endif

#endif /* OWK_SORTFORMER_H */
