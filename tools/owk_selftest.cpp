// Stand-alone smoke driver of libwhisper.so through the public C ABI (no Python).
//   owk_selftest <model.bin> [wav-less: synthetic 11 s tone]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "owk.h"
#include "whisper.h"

int main(int argc, char ** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s model.bin\n", argv[0]);
        return 1;
    }
    setvbuf(stdout, nullptr, _IONBF, 0);
    printf("device_ok=%d\n", owk_device_ok(0));
    auto cp = whisper_context_default_params();
    whisper_context * ctx = whisper_init_from_file_with_params(argv[1], cp);
    printf("ctx=%p\n", (void *) ctx);
    if (!ctx) return 2;
    whisper_state * st = whisper_init_state(ctx);
    printf("state=%p\n", (void *) st);
    std::vector<float> pcm(176000);
    for (size_t i = 0; i < pcm.size(); ++i) pcm[i] = 0.3f * sinf(0.05f * i) * sinf(0.0007f * i);
    int r = whisper_pcm_to_mel_with_state(ctx, st, pcm.data(), (int) pcm.size(), 1);
    printf("mel=%d n_len=%d\n", r, whisper_n_len_from_state(st));
    r = whisper_encode_with_state(ctx, st, 0, 1);
    printf("encode=%d\n", r);
    whisper_token sot = whisper_token_sot(ctx);
    r = whisper_decode_with_state(ctx, st, &sot, 1, 0, 1);
    const float * lg = whisper_get_logits_from_state(st);
    int am = 0;
    for (int i = 1; i < whisper_n_vocab(ctx); ++i)
        if (lg[i] > lg[am]) am = i;
    printf("decode=%d argmax=%d logit=%f\n", r, am, lg[am]);
    auto p = whisper_full_default_params(WHISPER_SAMPLING_GREEDY);
    p.print_progress = false;
    p.temperature_inc = 0.0f;
    r = whisper_full_with_state(ctx, st, p, pcm.data(), (int) pcm.size());
    printf("full=%d segments=%d\n", r, whisper_full_n_segments_from_state(st));
    for (int i = 0; i < whisper_full_n_segments_from_state(st); ++i)
        printf("  [%lld %lld] %s\n", (long long) whisper_full_get_segment_t0_from_state(st, i),
               (long long) whisper_full_get_segment_t1_from_state(st, i), whisper_full_get_segment_text_from_state(st, i));
    whisper_free_state(st);
    whisper_free(ctx);
    printf("ok\n");
    return 0;
}
