// Silero VAD behind the reference's whisper_vad_* C API (include/whisper.h:678-732) and
// whisper_full's VAD pre-pass, on the MI355X.
//
//   loader                 ref/src/whisper.cpp:4717-5084 (ggml-bin "silero-16k" file)
//   detect_speech(_stateful), reset_state, probs
//                          ref/src/whisper.cpp:5086-5208 -> k_vad.hip (all chunks of a call
//                          encoded in parallel, one LSTM workgroup per stream)
//   segments_from_probs    ref/src/whisper.cpp:5210-5444 (host; integer sample arithmetic)
//   whisper_vad filter     ref/src/whisper.cpp:6643-6826 (host)
//   time mapping           ref/src/whisper.cpp:7947-8025 (host)
// The reference forces the VAD onto the CPU (whisper_vad_init_context, 4655-4661); here it
// runs on the context's GPU (whisper_vad_context_params.gpu_device), so use_gpu is ignored.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstring>
#include <fstream>
#include <map>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "model.h"
#include "state.h"
#include "whisper.h"
#include "owk.h"

using namespace owk;

struct whisper_vad_context {
    int device = 0;
    int n_window = 512, n_context = 64;
    std::string type, version;
    int64_t t_vad_us = 0;
    hipStream_t stream = nullptr;
    DevBuf weights;      // every tensor in kernel layout
    VadWeights w{};
    DevBuf state;        // LSTM h | c (zero = reference buffer clear)
    DevBuf pcm, ig, hist, probs_dev, meta;
    std::vector<float> probs;
    ~whisper_vad_context() {
        if (stream) (void) hipStreamDestroy(stream);
    }
};

struct whisper_vad_segment {
    int64_t start, end;  // centiseconds
};
struct whisper_vad_segments {
    std::vector<whisper_vad_segment> data;
};

struct whisper_vad_context_params whisper_vad_default_context_params(void) {
    whisper_vad_context_params r{};
    r.n_threads = 4;
    r.use_gpu = false;
    r.gpu_device = 0;
    return r;
}

struct whisper_vad_params whisper_vad_default_params(void) {
    whisper_vad_params r{};
    r.threshold = 0.5f;
    r.min_speech_duration_ms = 250;
    r.min_silence_duration_ms = 100;
    r.max_speech_duration_s = FLT_MAX;
    r.speech_pad_ms = 30;
    r.samples_overlap = 0.1f;
    return r;
}

namespace {

int cs_to_samples(int64_t cs) { return (int) ((cs / 100.0) * WHISPER_SAMPLE_RATE + 0.5); }
int64_t samples_to_cs(int samples) { return (int64_t) ((samples / (double) WHISPER_SAMPLE_RATE) * 100.0 + 0.5); }

struct RawTensor {
    int type;  // 0 f32, 1 f16
    std::vector<int> ne;
    std::vector<uint8_t> data;
    size_t count() const {
        size_t n = 1;
        for (int v : ne) n *= (size_t) v;
        return n;
    }
    float at(size_t i) const {
        if (type == 1) {
            uint16_t u;
            memcpy(&u, data.data() + 2 * i, 2);
            return f16_to_f32_host(u);
        }
        float f;
        memcpy(&f, data.data() + 4 * i, 4);
        return f;
    }
};

template <typename T> bool rd(whisper_model_loader * l, T & v) { return l->read(l->context, &v, sizeof(T)) == sizeof(T); }

// Parse the file (ref 4761-5076). Expected shapes are the reference's create_tensor list.
bool parse_vad(whisper_model_loader * l, whisper_vad_context & v, std::map<std::string, RawTensor> & t, std::string & err) {
    uint32_t magic = 0;
    if (!rd(l, magic) || magic != 0x67676d6c) {
        err = "invalid model data (bad magic)";
        return false;
    }
    int32_t n = 0;
    if (!rd(l, n) || n < 0 || n > 4096) { err = "bad model type"; return false; }
    std::vector<char> buf(n);
    l->read(l->context, buf.data(), n);
    v.type.assign(buf.data(), n);
    int32_t ver[3], nl = 0;
    for (auto & x : ver) rd(l, x);
    v.version = std::to_string(ver[0]) + "." + std::to_string(ver[1]) + "." + std::to_string(ver[2]);
    rd(l, v.n_window);
    rd(l, v.n_context);
    rd(l, nl);
    const int want[4][3] = {{129, 128, 3}, {128, 64, 3}, {64, 64, 3}, {64, 128, 3}};
    if (nl != 4) { err = "unsupported VAD encoder layer count " + std::to_string(nl); return false; }
    for (int i = 0; i < nl; ++i)
        for (int j = 0; j < 3; ++j) {
            int32_t x = 0;
            rd(l, x);
            if (x != want[i][j]) { err = "unsupported VAD encoder geometry"; return false; }
        }
    int32_t hp[4];
    for (auto & x : hp) rd(l, x);
    if (hp[0] != 128 || hp[1] != 128 || hp[2] != 128 || hp[3] != 1 || v.n_window != 512) {
        err = "unsupported VAD geometry (this engine implements Silero v5/v6 16 kHz)";
        return false;
    }
    while (true) {
        int32_t nd = 0, len = 0, tt = 0;
        rd(l, nd);
        rd(l, len);
        rd(l, tt);
        if (l->eof(l->context)) break;
        if (nd < 0 || nd > 4 || len <= 0 || len > 512 || (tt != 0 && tt != 1)) { err = "bad tensor header"; return false; }
        RawTensor r;
        r.type = tt;
        r.ne.resize(nd);
        for (auto & x : r.ne) rd(l, x);
        std::string name(len, '\0');
        l->read(l->context, &name[0], len);
        r.data.resize(r.count() * (tt == 1 ? 2 : 4));
        if (l->read(l->context, r.data.data(), r.data.size()) != r.data.size()) { err = "truncated tensor " + name; return false; }
        t[name] = std::move(r);
    }
    return true;
}

} // namespace

struct whisper_vad_context * whisper_vad_init_with_params(struct whisper_model_loader * loader,
                                                          struct whisper_vad_context_params params) {
    auto * v = new whisper_vad_context;
    std::map<std::string, RawTensor> t;
    std::string err;
    const bool ok = parse_vad(loader, *v, t, err);
    if (loader->close) loader->close(loader->context);
    if (!ok) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_init_with_params: %s\n", err.c_str());
        delete v;
        return nullptr;
    }
    // expected tensors: name -> (type, element count) (ref 4894-4985)
    const std::pair<const char *, std::pair<int, size_t>> spec[] = {
        {"_model.stft.forward_basis_buffer", {1, 256 * 258}},
        {"_model.encoder.0.reparam_conv.weight", {1, 3 * 129 * 128}}, {"_model.encoder.0.reparam_conv.bias", {0, 128}},
        {"_model.encoder.1.reparam_conv.weight", {1, 3 * 128 * 64}}, {"_model.encoder.1.reparam_conv.bias", {0, 64}},
        {"_model.encoder.2.reparam_conv.weight", {1, 3 * 64 * 64}}, {"_model.encoder.2.reparam_conv.bias", {0, 64}},
        {"_model.encoder.3.reparam_conv.weight", {1, 3 * 64 * 128}}, {"_model.encoder.3.reparam_conv.bias", {0, 128}},
        {"_model.decoder.rnn.weight_ih", {0, 128 * 512}}, {"_model.decoder.rnn.bias_ih", {0, 512}},
        {"_model.decoder.rnn.weight_hh", {0, 128 * 512}}, {"_model.decoder.rnn.bias_hh", {0, 512}},
        {"_model.decoder.decoder.2.weight", {1, 128}}, {"_model.decoder.decoder.2.bias", {0, 1}},
    };
    for (const auto & s : spec) {
        auto it = t.find(s.first);
        if (it == t.end() || it->second.type != s.second.first || it->second.count() != s.second.second) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_init_with_params: tensor '%s' missing or of wrong type/shape\n", s.first);
            delete v;
            return nullptr;
        }
    }
    if (t.size() != sizeof(spec) / sizeof(spec[0])) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_init_with_params: unexpected tensors in the model file\n");
        delete v;
        return nullptr;
    }
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev <= 0) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_init_with_params: no MI355X (gfx950) device available\n");
        delete v;
        return nullptr;
    }
    v->device = std::max(0, std::min(params.gpu_device, n_dev - 1));
    try {
        OWK_HIP_CHECK(hipSetDevice(v->device));
        OWK_HIP_CHECK(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking));
        // one host image of every tensor in kernel layout, then one upload
        std::vector<uint8_t> img;
        auto put_f16 = [&](const std::vector<float> & x) {
            size_t off = (img.size() + 255) & ~size_t(255);
            img.resize(off + x.size() * 2);
            for (size_t i = 0; i < x.size(); ++i) {
                uint16_t u = f32_to_f16_host(x[i]);
                memcpy(img.data() + off + 2 * i, &u, 2);
            }
            return off;
        };
        auto put_f32 = [&](const std::vector<float> & x) {
            size_t off = (img.size() + 255) & ~size_t(255);
            img.resize(off + x.size() * 4);
            memcpy(img.data() + off, x.data(), x.size() * 4);
            return off;
        };
        auto get = [&](const char * name) {
            const RawTensor & r = t.at(name);
            std::vector<float> x(r.count());
            for (size_t i = 0; i < x.size(); ++i) x[i] = r.at(i);
            return x;
        };
        // conv weight [OC][IC][K] -> [(ic*K + k)][OC] (values are exact F16)
        auto transpose = [](const std::vector<float> & x, int oc, int ick) {
            std::vector<float> y(x.size());
            for (int o = 0; o < oc; ++o)
                for (int j = 0; j < ick; ++j) y[(size_t) j * oc + o] = x[(size_t) o * ick + j];
            return y;
        };
        const size_t o_stft = put_f16(transpose(get("_model.stft.forward_basis_buffer"), 258, 256));
        const int enc_oc[4] = {128, 64, 64, 128}, enc_ic[4] = {129, 128, 64, 64};
        size_t o_enc[4], o_encb[4];
        for (int i = 0; i < 4; ++i) {
            const std::string p = "_model.encoder." + std::to_string(i) + ".reparam_conv.";
            o_enc[i] = put_f16(transpose(get((p + "weight").c_str()), enc_oc[i], enc_ic[i] * 3));
            o_encb[i] = put_f32(get((p + "bias").c_str()));
        }
        const size_t o_ih = put_f32(transpose(get("_model.decoder.rnn.weight_ih"), 512, 128));
        const size_t o_bih = put_f32(get("_model.decoder.rnn.bias_ih"));
        const size_t o_hh = put_f32(get("_model.decoder.rnn.weight_hh"));
        const size_t o_bhh = put_f32(get("_model.decoder.rnn.bias_hh"));
        const size_t o_wf = put_f16(get("_model.decoder.decoder.2.weight"));
        const size_t o_bf = put_f32(get("_model.decoder.decoder.2.bias"));
        v->weights.alloc(img.size());
        OWK_HIP_CHECK(hipMemcpy(v->weights.ptr, img.data(), img.size(), hipMemcpyHostToDevice));
        uint8_t * base = v->weights.as<uint8_t>();
        v->w.stft_T = (const _Float16 *) (base + o_stft);
        for (int i = 0; i < 4; ++i) {
            v->w.enc_T[i] = (const _Float16 *) (base + o_enc[i]);
            v->w.enc_b[i] = (const float *) (base + o_encb[i]);
        }
        v->w.ih_T = (const float *) (base + o_ih);
        v->w.b_ih = (const float *) (base + o_bih);
        v->w.w_hh = (const float *) (base + o_hh);
        v->w.b_hh = (const float *) (base + o_bhh);
        v->w.wf = (const _Float16 *) (base + o_wf);
        v->w.bf = (const float *) (base + o_bf);
        v->state.alloc(2 * 128 * sizeof(float));
        OWK_HIP_CHECK(hipMemset(v->state.ptr, 0, v->state.bytes));
    } catch (const std::exception & e) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_init_with_params: %s\n", e.what());
        delete v;
        return nullptr;
    }
    return v;
}

struct whisper_vad_context * whisper_vad_init_from_file_with_params(const char * path_model,
                                                                    struct whisper_vad_context_params params) {
    auto * fin = new std::ifstream(path_model, std::ios::binary);
    if (!*fin) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_init_from_file_with_params: failed to open VAD model '%s'\n", path_model);
        delete fin;
        return nullptr;
    }
    whisper_model_loader loader = {};
    loader.context = fin;
    loader.read = [](void * c, void * out, size_t n) {
        auto * f = (std::ifstream *) c;
        f->read((char *) out, n);
        return (size_t) f->gcount();
    };
    loader.eof = [](void * c) { return ((std::ifstream *) c)->eof(); };
    loader.close = [](void * c) {
        auto * f = (std::ifstream *) c;
        f->close();
        delete f;
    };
    return whisper_vad_init_with_params(&loader, params);
}

namespace owk {

// Run the VAD over n_streams independent streams in one pass: every stream's chunks are
// encoded together, one LSTM workgroup per stream. states: device [n_streams][256] h|c
// (nullptr: the context's own state, n_streams must be 1). probs[s] receives
// ceil(n[s] / 512) floats.
bool vad_run(whisper_vad_context * v, const float * const * pcm, const int * n, int n_streams, float * state_dev,
             float * const * probs_out) {
    std::vector<int64_t> off(n_streams);
    std::vector<int> len(n_streams), first(n_streams), cnt(n_streams);
    int64_t tot = 0;
    int n_chunks = 0;
    for (int s = 0; s < n_streams; ++s) {
        if (n[s] < 0) return false;
        off[s] = tot;
        len[s] = n[s];
        tot += n[s];
        first[s] = n_chunks;
        cnt[s] = (n[s] + v->n_window - 1) / v->n_window;
        n_chunks += cnt[s];
    }
    if (n_chunks == 0) return true;
    std::vector<int> cs(n_chunks), ci(n_chunks);
    for (int s = 0; s < n_streams; ++s)
        for (int i = 0; i < cnt[s]; ++i) {
            cs[first[s] + i] = s;
            ci[first[s] + i] = i;
        }
    OWK_HIP_CHECK(hipSetDevice(v->device));
    v->pcm.alloc(std::max<int64_t>(tot, 1) * sizeof(float));
    v->ig.alloc((size_t) n_chunks * 512 * sizeof(float));
    v->hist.alloc((size_t) n_chunks * 128 * sizeof(float));
    v->probs_dev.alloc((size_t) n_chunks * sizeof(float));
    // metadata: off (i64) | len | first | cnt | cs | ci
    std::vector<uint8_t> meta(n_streams * 8 + (3 * n_streams + 2 * n_chunks) * 4);
    uint8_t * m = meta.data();
    memcpy(m, off.data(), n_streams * 8);
    memcpy(m + n_streams * 8, len.data(), n_streams * 4);
    memcpy(m + n_streams * 12, first.data(), n_streams * 4);
    memcpy(m + n_streams * 16, cnt.data(), n_streams * 4);
    memcpy(m + n_streams * 20, cs.data(), n_chunks * 4);
    memcpy(m + n_streams * 20 + n_chunks * 4, ci.data(), n_chunks * 4);
    v->meta.alloc(meta.size());
    for (int s = 0; s < n_streams; ++s)
        if (n[s] > 0)
            OWK_HIP_CHECK(hipMemcpyAsync(v->pcm.as<float>() + off[s], pcm[s], (size_t) n[s] * sizeof(float),
                                         hipMemcpyHostToDevice, v->stream));
    OWK_HIP_CHECK(hipMemcpyAsync(v->meta.ptr, meta.data(), meta.size(), hipMemcpyHostToDevice, v->stream));
    uint8_t * md = v->meta.as<uint8_t>();
    launch_vad(v->w, v->pcm.as<float>(), (const int64_t *) md, (const int *) (md + n_streams * 8),
               (const int *) (md + n_streams * 20), (const int *) (md + n_streams * 20 + n_chunks * 4), n_chunks,
               (const int *) (md + n_streams * 12), (const int *) (md + n_streams * 16), n_streams, v->ig.as<float>(),
               v->hist.as<float>(), state_dev ? state_dev : v->state.as<float>(), v->probs_dev.as<float>(), v->stream);
    std::vector<float> all(n_chunks);
    OWK_HIP_CHECK(hipMemcpyAsync(all.data(), v->probs_dev.ptr, (size_t) n_chunks * sizeof(float), hipMemcpyDeviceToHost,
                                 v->stream));
    OWK_HIP_CHECK(hipStreamSynchronize(v->stream));
    for (int s = 0; s < n_streams; ++s) std::copy(all.begin() + first[s], all.begin() + first[s] + cnt[s], probs_out[s]);
    return true;
}

// ref 5210-5444; returns the segments in centiseconds
std::vector<whisper_vad_segment> vad_segments(const float * probs, int n_probs, int n_window, const whisper_vad_params & params) {
    const float threshold = params.threshold;
    const int min_speech_duration_ms = params.min_speech_duration_ms;
    const int min_silence_duration_ms = params.min_silence_duration_ms;
    const float max_speech_duration_s = params.max_speech_duration_s;
    const int speech_pad_ms = params.speech_pad_ms;
    const int sr = WHISPER_SAMPLE_RATE;
    const int min_silence_samples = sr * min_silence_duration_ms / 1000;
    const int audio_length_samples = n_probs * n_window;
    const int min_speech_samples = sr * min_speech_duration_ms / 1000;
    const int speech_pad_samples = sr * speech_pad_ms / 1000;
    int max_speech_samples;
    if (max_speech_duration_s > 100000.0f) {
        max_speech_samples = INT_MAX / 2;
    } else {
        const int64_t tmp = (int64_t) sr * (int64_t) (max_speech_duration_s) - n_window - 2 * speech_pad_samples;
        max_speech_samples = (tmp > INT_MAX) ? INT_MAX / 2 : (int) tmp;
        if (max_speech_samples < 0) max_speech_samples = INT_MAX / 2;
    }
    const int min_silence_samples_at_max_speech = sr * 98 / 1000;
    float neg_threshold = threshold - 0.15f;
    if (neg_threshold < 0.01f) neg_threshold = 0.01f;

    struct Sp {
        int start, end;
    };
    std::vector<Sp> sp;
    bool in_speech = false, has_cur = false;
    int temp_end = 0, prev_end = 0, next_start = 0, cur_start = 0;
    for (int i = 0; i < n_probs; ++i) {
        const float p = probs[i];
        const int cs = n_window * i;
        if (p >= threshold && temp_end) {
            temp_end = 0;
            if (next_start < prev_end) next_start = cs;
        }
        if (p >= threshold && !in_speech) {
            in_speech = has_cur = true;
            cur_start = cs;
            continue;
        }
        if (in_speech && (cs - cur_start) > max_speech_samples) {
            if (prev_end) {
                sp.push_back({cur_start, prev_end});
                has_cur = true;
                if (next_start < prev_end) {
                    in_speech = has_cur = false;
                } else {
                    cur_start = next_start;
                }
                prev_end = next_start = temp_end = 0;
            } else {
                sp.push_back({cur_start, cs});
                prev_end = next_start = temp_end = 0;
                in_speech = has_cur = false;
                continue;
            }
        }
        if (p < neg_threshold && in_speech) {
            if (!temp_end) temp_end = cs;
            if ((cs - temp_end) > min_silence_samples_at_max_speech) prev_end = temp_end;
            if ((cs - temp_end) < min_silence_samples) continue;
            if ((temp_end - cur_start) > min_speech_samples) sp.push_back({cur_start, temp_end});
            prev_end = next_start = temp_end = 0;
            in_speech = has_cur = false;
            continue;
        }
    }
    if (has_cur && (audio_length_samples - cur_start) > min_speech_samples) sp.push_back({cur_start, audio_length_samples});
    // merge gaps under 200 ms, then drop segments shorter than min_speech
    const int max_merge_gap_samples = sr * 200 / 1000;
    for (size_t i = 0; sp.size() > 1 && i + 1 < sp.size();) {
        if (sp[i + 1].start - sp[i].end < max_merge_gap_samples) {
            sp[i].end = sp[i + 1].end;
            sp.erase(sp.begin() + i + 1);
        } else {
            ++i;
        }
    }
    sp.erase(std::remove_if(sp.begin(), sp.end(), [&](const Sp & s) { return s.end - s.start < min_speech_samples; }),
             sp.end());
    std::vector<whisper_vad_segment> out(sp.size());
    for (size_t i = 0; i < sp.size(); ++i) {
        if (i == 0) sp[i].start = sp[i].start > speech_pad_samples ? sp[i].start - speech_pad_samples : 0;
        if (i + 1 < sp.size()) {
            const int silence = sp[i + 1].start - sp[i].end;
            if (silence < 2 * speech_pad_samples) {
                sp[i].end += silence / 2;
                sp[i + 1].start = sp[i + 1].start > silence / 2 ? sp[i + 1].start - silence / 2 : 0;
            } else {
                sp[i].end = sp[i].end + speech_pad_samples < audio_length_samples ? sp[i].end + speech_pad_samples
                                                                                  : audio_length_samples;
                sp[i + 1].start = sp[i + 1].start > speech_pad_samples ? sp[i + 1].start - speech_pad_samples : 0;
            }
        } else {
            sp[i].end = sp[i].end + speech_pad_samples < audio_length_samples ? sp[i].end + speech_pad_samples
                                                                              : audio_length_samples;
        }
        out[i].start = samples_to_cs(sp[i].start);
        out[i].end = samples_to_cs(sp[i].end);
    }
    return out;
}

// whisper_full's pre-pass (ref 6643-6826): speech segments + 0.1 s silences, and the
// processed -> original time table of the state
bool vad_filter(whisper_context * ctx, whisper_state * state, const whisper_full_params & params, const float * samples,
                int n_samples, std::vector<float> & filtered) {
    state->vad_map.clear();
    state->has_vad_segments = false;
    if (!state->vad_context) {
        // the pre-pass runs on the whisper context's GPU (one process per GPU: never device 0 by default)
        whisper_vad_context_params vp = whisper_vad_default_context_params();
        vp.gpu_device = ctx->model->device;
        state->vad_context = whisper_vad_init_from_file_with_params(params.vad_model_path, vp);
        if (!state->vad_context) {
            log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad: failed to initialize VAD context\n");
            return false;
        }
    }
    whisper_vad_segments * segs = whisper_vad_segments_from_samples(state->vad_context, params.vad_params, samples, n_samples);
    if (!segs) return false;
    const auto & d = segs->data;
    if (!d.empty()) {
        state->has_vad_segments = true;
        const int overlap_samples = params.vad_params.samples_overlap * WHISPER_SAMPLE_RATE;
        int filtered_n = 0;
        for (size_t i = 0; i < d.size(); ++i) {
            int s0 = cs_to_samples(d[i].start), s1 = cs_to_samples(d[i].end);
            if (i + 1 < d.size()) s1 += overlap_samples;
            s1 = std::min(s1, n_samples - 1);
            filtered_n += s1 - s0;
        }
        const int silence_samples = 0.1 * WHISPER_SAMPLE_RATE;
        const int total_silence = d.size() > 1 ? (int) (d.size() - 1) * silence_samples : 0;
        filtered.assign(filtered_n + total_silence, 0.0f);
        auto & map = state->vad_map;
        int offset = 0;
        for (size_t i = 0; i < d.size(); ++i) {
            int s0 = cs_to_samples(d[i].start), s1 = cs_to_samples(d[i].end);
            if (i + 1 < d.size()) s1 += overlap_samples;
            s0 = std::min(s0, n_samples - 1);
            s1 = std::min(s1, n_samples - 1);
            const int seg_len = s1 - s0;
            if (seg_len <= 0) continue;
            const int64_t orig_start = d[i].start, orig_end = d[i].end;
            const int64_t vad_start = samples_to_cs(offset), vad_end = samples_to_cs(offset + seg_len);
            map.push_back({vad_start, orig_start});
            map.push_back({vad_end, orig_end});
            if (vad_end - vad_start > 100) {  // a point every 200 ms in segments over 1 s
                const int64_t dur = vad_end - vad_start;
                const int num_points = (int) (dur / 20) - 1;
                for (int j = 1; j <= num_points; ++j) {
                    const int64_t vt = vad_start + j * 20;
                    if (vt >= vad_end) continue;
                    map.push_back({vt, orig_start + ((vt - vad_start) * (orig_end - orig_start)) / (vad_end - vad_start)});
                }
            }
            memcpy(filtered.data() + offset, samples + s0, (size_t) seg_len * sizeof(float));
            offset += seg_len;
            if (i + 1 < d.size()) {
                map.push_back({samples_to_cs(offset), orig_end});
                map.push_back({samples_to_cs(offset + silence_samples), d[i + 1].start});
                memset(filtered.data() + offset, 0, (size_t) silence_samples * sizeof(float));
                offset += silence_samples;
            }
        }
        std::sort(map.begin(), map.end(), [](const std::pair<int64_t, int64_t> & a, const std::pair<int64_t, int64_t> & b) {
            return a.first < b.first;
        });
        map.erase(std::unique(map.begin(), map.end(),
                              [](const std::pair<int64_t, int64_t> & a, const std::pair<int64_t, int64_t> & b) {
                                  return a.first == b.first;
                              }),
                  map.end());
    }
    whisper_vad_free_segments(segs);
    return true;
}

// ref 7947-7984
int64_t vad_map_time(int64_t t, const std::vector<std::pair<int64_t, int64_t>> & map) {
    if (map.empty()) return t;
    if (t <= map.front().first) return map.front().second;
    if (t >= map.back().first) return map.back().second;
    auto up = std::lower_bound(map.begin(), map.end(), t,
                               [](const std::pair<int64_t, int64_t> & e, int64_t x) { return e.first < x; });
    if (up->first == t) return up->second;
    auto lo = up - 1;
    const int64_t pd = up->first - lo->first, od = up->second - lo->second;
    if (pd == 0) return lo->second;
    return lo->second + ((t - lo->first) * od) / pd;
}

} // namespace owk

static bool detect(whisper_vad_context * v, const float * samples, int n_samples, bool reset) {
    if (!v || n_samples < 0 || (n_samples > 0 && !samples)) return false;
    const int64_t t0 = time_us();
    try {
        OWK_HIP_CHECK(hipSetDevice(v->device));
        if (reset) OWK_HIP_CHECK(hipMemsetAsync(v->state.ptr, 0, v->state.bytes, v->stream));
        v->probs.assign((n_samples + v->n_window - 1) / v->n_window, 0.0f);
        float * out = v->probs.data();
        if (!vad_run(v, &samples, &n_samples, 1, nullptr, &out)) return false;
    } catch (const std::exception & e) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_detect_speech: %s\n", e.what());
        return false;
    }
    v->t_vad_us += time_us() - t0;
    return true;
}

bool whisper_vad_detect_speech(struct whisper_vad_context * vctx, const float * samples, int n_samples) {
    return detect(vctx, samples, n_samples, true);
}
bool whisper_vad_detect_speech_stateful(struct whisper_vad_context * vctx, const float * samples, int n_samples) {
    return detect(vctx, samples, n_samples, false);
}
void whisper_vad_reset_state(struct whisper_vad_context * vctx) {
    if (!vctx || !vctx->state.ptr) return;
    (void) hipSetDevice(vctx->device);
    (void) hipMemsetAsync(vctx->state.ptr, 0, vctx->state.bytes, vctx->stream);
    (void) hipStreamSynchronize(vctx->stream);
}
int whisper_vad_n_probs(struct whisper_vad_context * vctx) { return (int) vctx->probs.size(); }
float * whisper_vad_probs(struct whisper_vad_context * vctx) { return vctx->probs.data(); }

struct whisper_vad_segments * whisper_vad_segments_from_probs(struct whisper_vad_context * vctx,
                                                              struct whisper_vad_params params) {
    auto * s = new whisper_vad_segments;
    s->data = vad_segments(vctx->probs.data(), (int) vctx->probs.size(), vctx->n_window, params);
    return s;
}
struct whisper_vad_segments * whisper_vad_segments_from_samples(struct whisper_vad_context * vctx,
                                                                struct whisper_vad_params params, const float * samples,
                                                                int n_samples) {
    if (!whisper_vad_detect_speech(vctx, samples, n_samples)) {
        log_msg(GGML_LOG_LEVEL_ERROR, "whisper_vad_segments_from_samples: failed to detect speech\n");
        return nullptr;
    }
    return whisper_vad_segments_from_probs(vctx, params);
}
int whisper_vad_segments_n_segments(struct whisper_vad_segments * segments) { return (int) segments->data.size(); }
float whisper_vad_segments_get_segment_t0(struct whisper_vad_segments * segments, int i) { return segments->data[i].start; }
float whisper_vad_segments_get_segment_t1(struct whisper_vad_segments * segments, int i) { return segments->data[i].end; }
void whisper_vad_free_segments(struct whisper_vad_segments * segments) { delete segments; }
void whisper_vad_free(struct whisper_vad_context * ctx) { delete ctx; }

// ---------------------------------------------------------------------------------
// owk extensions (include/owk.h)
// ---------------------------------------------------------------------------------
int owk_vad_detect_batch(struct whisper_vad_context * vctx, const float * const * samples, const int * n_samples,
                         int n_streams, float * const * probs_out) {
    if (!vctx || n_streams <= 0) return -1;
    try {
        OWK_HIP_CHECK(hipSetDevice(vctx->device));
        DevBuf st;
        st.alloc((size_t) n_streams * 256 * sizeof(float));
        OWK_HIP_CHECK(hipMemsetAsync(st.ptr, 0, st.bytes, vctx->stream));
        if (!vad_run(vctx, samples, n_samples, n_streams, st.as<float>(), probs_out)) return -1;
    } catch (const std::exception & e) {
        log_msg(GGML_LOG_LEVEL_ERROR, "owk_vad_detect_batch: %s\n", e.what());
        return -1;
    }
    return 0;
}

int owk_vad_segments_raw(const float * probs, int n_probs, int n_window, struct whisper_vad_params params,
                         int64_t * out_cs, int cap) {
    const auto segs = vad_segments(probs, n_probs, n_window, params);
    if (out_cs)
        for (int i = 0; i < (int) segs.size() && i < cap; ++i) {
            out_cs[2 * i] = segs[i].start;
            out_cs[2 * i + 1] = segs[i].end;
        }
    return (int) segs.size();
}
