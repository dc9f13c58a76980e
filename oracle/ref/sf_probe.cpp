// TEST INFRASTRUCTURE — SortFormer parity oracle probe, never part of the product.
//
// Compiles the reference streaming-sortformer in place (#include of
// /root/reference/streaming-sortformer/src/sortformer.cpp; nothing is copied into this repo)
// into oracle/_ref/libsortformer_ref.so with one extern "C" accessor more: the AOSC speaker-cache
// bookkeeping of the streaming state (update_silence_profile, sortformer.cpp:1729-1752, then
// compress_spkcache, 1783-1920), which the library keeps static. tests/test_sanitize_host.py drives
// it beside the product's restatement (libsortformer.so owk_sortformer_debug_aosc).
#include "sortformer.cpp"

extern "C" {

// spkcache of n_frames frames (embeddings [n][d], predictions [n][4]) and the running silence profile
// (mean_sil [d], n_sil frames so far); n_pop popped FIFO frames (pop_embs [n_pop][d], pop_preds
// [n_pop][4]) update the silence profile first; then the cache is compressed to spkcache_len frames.
// Outputs: out_embs [spkcache_len][d], out_preds [spkcache_len][4], out_mean_sil [d]; returns the new
// length (or -1 when the cache does not exceed spkcache_len, where the reference does not compress).
int ref_sf_aosc(int d, int n_frames, const float * embs, const float * preds, const float * mean_sil, int n_sil,
                int n_pop, const float * pop_embs, const float * pop_preds, int spkcache_len, int sil_frames_per_spk,
                float * out_embs, float * out_preds, float * out_mean_sil) {
    stream_config cfg = default_stream_config();
    cfg.spkcache_len = spkcache_len;
    cfg.spkcache_sil_frames_per_spk = sil_frames_per_spk;
    const int n_spk = 4;
    stream_state st = init_stream_state(d);
    st.spkcache.assign(embs, embs + (size_t) n_frames * d);
    st.spkcache_preds.assign(preds, preds + (size_t) n_frames * n_spk);
    st.spkcache_len = n_frames;
    st.spkcache_preds_valid = true;
    st.mean_sil_emb.assign(mean_sil, mean_sil + d);
    st.n_sil_frames = n_sil;
    if (n_pop > 0) update_silence_profile(st, cfg, pop_embs, pop_preds, n_pop, d, n_spk);
    std::copy(st.mean_sil_emb.begin(), st.mean_sil_emb.end(), out_mean_sil);
    if (n_frames <= spkcache_len) return -1;
    compress_spkcache(st, cfg, d, n_spk);
    std::copy(st.spkcache.begin(), st.spkcache.end(), out_embs);
    std::copy(st.spkcache_preds.begin(), st.spkcache_preds.end(), out_preds);
    return st.spkcache_len;
}

}  // extern "C"
