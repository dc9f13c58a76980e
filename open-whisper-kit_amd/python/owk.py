"""ctypes binding of the drop-in C ABI (include/whisper.h + include/owk.h).

This is how tests/, bench.py and __graft_entry__.py drive the MI355X engine: through
the exact exported symbols a reference caller would bind (the same calls the Swift
SDK / examples/cli make). Struct layouts mirror the reference header
(ref include/whisper.h:116-151, 487-591) field for field.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(HERE, "..", "lib", "libwhisper.so"))

WHISPER_SAMPLING_GREEDY = 0
WHISPER_SAMPLING_BEAM_SEARCH = 1


class Aheads(C.Structure):
    _fields_ = [("n_heads", C.c_size_t), ("heads", C.c_void_p)]


class ContextParams(C.Structure):
    _fields_ = [("use_gpu", C.c_bool), ("flash_attn", C.c_bool), ("gpu_device", C.c_int),
                ("dtw_token_timestamps", C.c_bool), ("dtw_aheads_preset", C.c_int), ("dtw_n_top", C.c_int),
                ("dtw_aheads", Aheads), ("dtw_mem_size", C.c_size_t)]


class TokenData(C.Structure):
    _fields_ = [("id", C.c_int32), ("tid", C.c_int32), ("p", C.c_float), ("plog", C.c_float), ("pt", C.c_float),
                ("ptsum", C.c_float), ("t0", C.c_int64), ("t1", C.c_int64), ("t_dtw", C.c_int64),
                ("vlen", C.c_float)]


class VadParams(C.Structure):
    _fields_ = [("threshold", C.c_float), ("min_speech_duration_ms", C.c_int), ("min_silence_duration_ms", C.c_int),
                ("max_speech_duration_s", C.c_float), ("speech_pad_ms", C.c_int), ("samples_overlap", C.c_float)]


class VadContextParams(C.Structure):  # whisper.h:682-686
    _fields_ = [("n_threads", C.c_int), ("use_gpu", C.c_bool), ("gpu_device", C.c_int)]


class _Greedy(C.Structure):
    _fields_ = [("best_of", C.c_int)]


class _Beam(C.Structure):
    _fields_ = [("beam_size", C.c_int), ("patience", C.c_float)]


LOGITS_FILTER_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.POINTER(TokenData), C.c_int, C.POINTER(C.c_float),
                               C.c_void_p)


class FullParams(C.Structure):
    _fields_ = [
        ("strategy", C.c_int),
        ("n_threads", C.c_int), ("n_max_text_ctx", C.c_int), ("offset_ms", C.c_int), ("duration_ms", C.c_int),
        ("translate", C.c_bool), ("no_context", C.c_bool), ("no_timestamps", C.c_bool), ("single_segment", C.c_bool),
        ("print_special", C.c_bool), ("print_progress", C.c_bool), ("print_realtime", C.c_bool),
        ("print_timestamps", C.c_bool),
        ("token_timestamps", C.c_bool), ("thold_pt", C.c_float), ("thold_ptsum", C.c_float), ("max_len", C.c_int),
        ("split_on_word", C.c_bool), ("max_tokens", C.c_int),
        ("debug_mode", C.c_bool), ("audio_ctx", C.c_int),
        ("tdrz_enable", C.c_bool),
        ("suppress_regex", C.c_char_p),
        ("initial_prompt", C.c_char_p), ("carry_initial_prompt", C.c_bool), ("prompt_tokens", C.c_void_p),
        ("prompt_n_tokens", C.c_int),
        ("language", C.c_char_p), ("detect_language", C.c_bool),
        ("suppress_blank", C.c_bool), ("suppress_nst", C.c_bool),
        ("temperature", C.c_float), ("max_initial_ts", C.c_float), ("length_penalty", C.c_float),
        ("temperature_inc", C.c_float), ("entropy_thold", C.c_float), ("logprob_thold", C.c_float),
        ("no_speech_thold", C.c_float),
        ("greedy", _Greedy), ("beam_search", _Beam),
        ("new_segment_callback", C.c_void_p), ("new_segment_callback_user_data", C.c_void_p),
        ("progress_callback", C.c_void_p), ("progress_callback_user_data", C.c_void_p),
        ("encoder_begin_callback", C.c_void_p), ("encoder_begin_callback_user_data", C.c_void_p),
        ("abort_callback", C.c_void_p), ("abort_callback_user_data", C.c_void_p),
        ("logits_filter_callback", C.c_void_p), ("logits_filter_callback_user_data", C.c_void_p),
        ("grammar_rules", C.c_void_p), ("n_grammar_rules", C.c_size_t), ("i_start_rule", C.c_size_t),
        ("grammar_penalty", C.c_float),
        ("vad", C.c_bool), ("vad_model_path", C.c_char_p), ("vad_params", VadParams),
    ]


class FullExt(C.Structure):
    _fields_ = [("suppress_eot", C.c_int), ("samples_on_device", C.c_int), ("reserved", C.c_int * 6)]


# every symbol include/whisper.h + include/owk.h declare (checked by tests/test_abi.py)
def header_symbols(include_dir=None):
    import re
    include_dir = include_dir or os.path.normpath(os.path.join(HERE, "..", "..", "include"))
    syms = []
    for h in ("whisper.h", "owk.h", "owk_diarize.h", "ggml-backend.h"):
        txt = open(os.path.join(include_dir, h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"\b((?:whisper|owk|ggml_backend)_[a-z0-9_]+)\s*\(", txt):
            name = m.group(1)
            if name.endswith("_callback"):
                continue
            syms.append(name)
    return sorted(set(syms))


_lib = None


def load(path: str | None = None) -> C.CDLL:
    """Load libwhisper.so; raises if the HIP build is missing (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("OWK_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise FileNotFoundError(f"libwhisper.so not built at {path} (run `make` / __graft_entry__.build())")
    L = C.CDLL(path)
    vp, ip, fp = C.c_void_p, C.c_int, C.POINTER(C.c_float)
    L.whisper_context_default_params.restype = ContextParams
    L.whisper_full_default_params.restype = FullParams
    L.whisper_full_default_params.argtypes = [ip]
    L.whisper_init_from_file_with_params.restype = vp
    L.whisper_init_from_file_with_params.argtypes = [C.c_char_p, ContextParams]
    L.whisper_init_state.restype = vp
    L.whisper_init_state.argtypes = [vp]
    L.whisper_free.argtypes = [vp]
    L.whisper_free_state.argtypes = [vp]
    L.whisper_full.argtypes = [vp, FullParams, fp, ip]
    L.whisper_full_with_state.argtypes = [vp, vp, FullParams, fp, ip]
    L.whisper_full_parallel.argtypes = [vp, FullParams, fp, ip, ip]
    L.owk_full_batch.argtypes = [vp, C.POINTER(vp), FullParams, C.POINTER(FullExt), C.POINTER(fp), C.POINTER(ip), ip]
    # int f(ctx-or-state) getters: without argtypes ctypes would truncate the pointer to 32 bits
    for n in ("whisper_full_n_segments_from_state", "whisper_n_len_from_state", "whisper_n_len",
              "whisper_full_lang_id_from_state", "whisper_full_lang_id", "whisper_n_text_ctx",
              "whisper_n_audio_ctx", "whisper_model_n_vocab", "whisper_model_n_audio_ctx",
              "whisper_model_n_audio_head", "whisper_model_n_audio_layer", "whisper_model_n_text_ctx",
              "whisper_model_n_text_state", "whisper_model_n_text_head", "whisper_model_ftype",
              "whisper_model_type", "whisper_token_solm", "whisper_token_prev", "whisper_token_nosp",
              "whisper_token_translate", "whisper_token_transcribe"):
        getattr(L, n).argtypes = [vp]
    L.whisper_token_lang.argtypes = [vp, ip]
    L.whisper_lang_id.argtypes = [C.c_char_p]
    L.whisper_lang_str.restype = C.c_char_p
    L.whisper_lang_str.argtypes = [ip]
    L.whisper_tokenize.argtypes = [vp, C.c_char_p, C.POINTER(C.c_int32), ip]
    L.whisper_get_logits.restype = fp
    L.whisper_get_logits.argtypes = [vp]
    L.whisper_full_get_segment_speaker_turn_next_from_state.restype = C.c_bool
    L.whisper_full_get_segment_speaker_turn_next_from_state.argtypes = [vp, ip]
    L.whisper_print_system_info.restype = C.c_char_p
    L.whisper_full_n_segments.argtypes = [vp]
    # context-level (default state) result getters, as whisper-cli uses them
    L.whisper_full_get_segment_t0.restype = C.c_int64
    L.whisper_full_get_segment_t0.argtypes = [vp, ip]
    L.whisper_full_get_segment_t1.restype = C.c_int64
    L.whisper_full_get_segment_t1.argtypes = [vp, ip]
    L.whisper_full_get_segment_text.restype = C.c_char_p
    L.whisper_full_get_segment_text.argtypes = [vp, ip]
    L.whisper_full_n_tokens.argtypes = [vp, ip]
    L.whisper_full_get_segment_t0_from_state.restype = C.c_int64
    L.whisper_full_get_segment_t0_from_state.argtypes = [vp, ip]
    L.whisper_full_get_segment_t1_from_state.restype = C.c_int64
    L.whisper_full_get_segment_t1_from_state.argtypes = [vp, ip]
    L.whisper_full_get_segment_text_from_state.restype = C.c_char_p
    L.whisper_full_get_segment_text_from_state.argtypes = [vp, ip]
    L.whisper_full_get_segment_no_speech_prob_from_state.restype = C.c_float
    L.whisper_full_get_segment_no_speech_prob_from_state.argtypes = [vp, ip]
    L.whisper_full_n_tokens_from_state.argtypes = [vp, ip]
    L.whisper_full_get_token_data_from_state.restype = TokenData
    L.whisper_full_get_token_data_from_state.argtypes = [vp, ip, ip]
    L.whisper_full_get_token_data.restype = TokenData
    L.whisper_full_get_token_data.argtypes = [vp, ip, ip]
    L.whisper_pcm_to_mel_with_state.argtypes = [vp, vp, fp, ip, ip]
    L.whisper_encode_with_state.argtypes = [vp, vp, ip, ip]
    L.whisper_decode_with_state.argtypes = [vp, vp, C.POINTER(C.c_int32), ip, ip, ip]
    L.whisper_get_logits_from_state.restype = fp
    L.whisper_get_logits_from_state.argtypes = [vp]
    L.whisper_n_vocab.argtypes = [vp]
    L.whisper_token_sot.argtypes = [vp]
    L.whisper_token_eot.argtypes = [vp]
    L.whisper_token_beg.argtypes = [vp]
    L.whisper_token_not.argtypes = [vp]
    L.whisper_token_to_str.restype = C.c_char_p
    L.whisper_token_to_str.argtypes = [vp, ip]
    L.whisper_model_n_mels.argtypes = [vp]
    L.whisper_model_n_audio_state.argtypes = [vp]
    L.whisper_model_n_text_layer.argtypes = [vp]
    L.whisper_is_multilingual.argtypes = [vp]
    L.whisper_lang_auto_detect_with_state.argtypes = [vp, vp, ip, ip, fp]
    L.whisper_lang_max_id.restype = ip
    L.whisper_log_set.argtypes = [vp, vp]
    L.owk_prof_enable.argtypes = [vp, ip]
    L.owk_prof_select.argtypes = [vp, C.c_char_p]
    L.owk_prof_reset.argtypes = [vp]
    L.owk_prof_read.argtypes = [vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_long)]
    L.owk_prof_work.argtypes = [vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.owk_prof_classes.restype = C.c_char_p
    L.owk_prof_classes.argtypes = [vp]
    L.owk_device_ok.argtypes = [ip]
    L.owk_debug_mel.argtypes = [vp, fp, ip]
    L.owk_debug_enc.argtypes = [vp, vp, ip, fp, ip]
    L.owk_debug_cross.argtypes = [vp, vp, ip, ip, C.POINTER(C.c_uint16), C.POINTER(C.c_uint16)]
    L.owk_debug_gelu_table.restype = C.POINTER(C.c_uint16)
    u16p = C.POINTER(C.c_uint16)
    L.owk_debug_gemm.argtypes = [ip, ip, ip, ip, u16p, u16p, fp]
    # Silero VAD (whisper.h:678-732, owk.h)
    L.whisper_vad_default_params.restype = VadParams
    L.whisper_vad_default_context_params.restype = VadContextParams
    L.whisper_vad_init_from_file_with_params.restype = vp
    L.whisper_vad_init_from_file_with_params.argtypes = [C.c_char_p, VadContextParams]
    for n in ("whisper_vad_detect_speech", "whisper_vad_detect_speech_stateful"):
        getattr(L, n).restype = C.c_bool
        getattr(L, n).argtypes = [vp, fp, ip]
    L.whisper_vad_reset_state.argtypes = [vp]
    L.whisper_vad_n_probs.argtypes = [vp]
    L.whisper_vad_probs.restype = fp
    L.whisper_vad_probs.argtypes = [vp]
    L.whisper_vad_segments_from_probs.restype = vp
    L.whisper_vad_segments_from_probs.argtypes = [vp, VadParams]
    L.whisper_vad_segments_from_samples.restype = vp
    L.whisper_vad_segments_from_samples.argtypes = [vp, VadParams, fp, ip]
    L.whisper_vad_segments_n_segments.argtypes = [vp]
    for n in ("whisper_vad_segments_get_segment_t0", "whisper_vad_segments_get_segment_t1"):
        getattr(L, n).restype = C.c_float
        getattr(L, n).argtypes = [vp, ip]
    L.whisper_vad_free_segments.argtypes = [vp]
    L.whisper_vad_free.argtypes = [vp]
    L.owk_vad_detect_batch.argtypes = [vp, C.POINTER(fp), C.POINTER(ip), ip, C.POINTER(fp)]
    L.owk_vad_segments_raw.argtypes = [fp, ip, ip, VadParams, C.POINTER(C.c_int64), ip]
    _lib = L
    return L


_LOG_CB = C.CFUNCTYPE(None, C.c_int, C.c_char_p, C.c_void_p)
# quiet(): nothing is printed, but warnings and errors (ggml_log_level >= WARN = 3) are kept in
# `errors` (the last 64) so a failing test can show what the library reported
errors = []


def _keep(lvl, txt, ud):
    if lvl >= 3 and txt:
        errors.append(txt.decode("utf-8", "replace").rstrip())
        del errors[:-64]


_quiet_cb = _LOG_CB(_keep)


def quiet():
    load().whisper_log_set(C.cast(_quiet_cb, C.c_void_p), None)


def fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Whisper:
    """Thin owner of a whisper_context (and its default state)."""

    def __init__(self, model_path: str, device: int = 0, flash_attn: bool = True, dtw_preset: int = 0,
                 dtw_n_top: int = -1):
        self.L = load()
        cp = self.L.whisper_context_default_params()
        cp.gpu_device = device
        cp.flash_attn = flash_attn
        if dtw_preset > 0:
            cp.dtw_token_timestamps = True
            cp.dtw_aheads_preset = dtw_preset
            cp.dtw_n_top = dtw_n_top
        self.dtw = dtw_preset > 0
        self.ctx = self.L.whisper_init_from_file_with_params(model_path.encode(), cp)
        if not self.ctx:
            raise RuntimeError(f"whisper_init_from_file_with_params failed for {model_path}")
        self.n_vocab = self.L.whisper_n_vocab(self.ctx)
        self._states = []

    def close(self):
        for s in self._states:
            self.L.whisper_free_state(s)
        self._states = []
        if self.ctx:
            self.L.whisper_free(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def new_state(self):
        s = self.L.whisper_init_state(self.ctx)
        if not s:
            raise RuntimeError("whisper_init_state failed")
        self._states.append(s)
        return s

    def free_state(self, s):
        if s in self._states:
            self._states.remove(s)
            self.L.whisper_free_state(s)

    def params(self, strategy=WHISPER_SAMPLING_GREEDY, **kw) -> FullParams:
        p = self.L.whisper_full_default_params(strategy)
        p.print_progress = False
        p.print_timestamps = False
        for k, v in kw.items():
            if k == "best_of":
                p.greedy.best_of = v
            elif k == "beam_size":
                p.beam_search.beam_size = v
            elif k == "language":
                p.language = v.encode() if isinstance(v, str) else v
            else:
                setattr(p, k, v)
        return p

    def full(self, state, pcm: np.ndarray, params: FullParams) -> int:
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        return self.L.whisper_full_with_state(self.ctx, state, params, fptr(pcm), len(pcm))

    def full_batch(self, states, pcms, params: FullParams, suppress_eot=False) -> int:
        n = len(pcms)
        arrs = [np.ascontiguousarray(p, dtype=np.float32) for p in pcms]
        ptrs = (C.POINTER(C.c_float) * n)(*[fptr(a) for a in arrs])
        ns = (C.c_int * n)(*[len(a) for a in arrs])
        sts = (C.c_void_p * n)(*states)
        ext = FullExt()
        ext.suppress_eot = 1 if suppress_eot else 0
        return self.L.owk_full_batch(self.ctx, sts, params, C.byref(ext), ptrs, ns, n)

    def full_batch_device(self, states, dev_ptrs, n_samples, params: FullParams, suppress_eot=False) -> int:
        """owk_full_batch over audio already resident in HBM (dev_ptrs: device addresses)."""
        n = len(dev_ptrs)
        ptrs = (C.POINTER(C.c_float) * n)(*[C.cast(C.c_void_p(p), C.POINTER(C.c_float)) for p in dev_ptrs])
        ns = (C.c_int * n)(*n_samples)
        sts = (C.c_void_p * n)(*states)
        ext = FullExt()
        ext.suppress_eot = 1 if suppress_eot else 0
        ext.samples_on_device = 1
        return self.L.owk_full_batch(self.ctx, sts, params, C.byref(ext), ptrs, ns, n)

    def prof_classes(self):
        s = self.L.owk_prof_classes(self.ctx)
        return [c for c in (s.decode() if s else "").split(",") if c]

    def prof(self, cls):
        ms, n, fl, by = C.c_double(), C.c_long(), C.c_double(), C.c_double()
        self.L.owk_prof_read(self.ctx, cls.encode(), C.byref(ms), C.byref(n))
        self.L.owk_prof_work(self.ctx, cls.encode(), C.byref(fl), C.byref(by))
        return dict(ms=ms.value, launches=n.value, flops=fl.value, bytes=by.value)

    def segments(self, state):
        L = self.L
        out = []
        for i in range(L.whisper_full_n_segments_from_state(state)):
            toks = []
            for j in range(L.whisper_full_n_tokens_from_state(state, i)):
                t = L.whisper_full_get_token_data_from_state(state, i, j)
                toks.append((t.id, t.tid, t.p, t.plog, t.pt, t.ptsum, t.t0, t.t1) + ((t.t_dtw,) if self.dtw else ()))
            out.append(dict(t0=L.whisper_full_get_segment_t0_from_state(state, i),
                            t1=L.whisper_full_get_segment_t1_from_state(state, i),
                            text=L.whisper_full_get_segment_text_from_state(state, i).decode("utf-8", "replace"),
                            no_speech_prob=L.whisper_full_get_segment_no_speech_prob_from_state(state, i),
                            tokens=toks))
        return out


# ---------------------------------------------------------------------------------
# speaker attribution (include/owk_diarize.h): the reference SDK's Swift
# DiarizationAligner / RTTMParser, implemented in C++ inside libwhisper.so
# ---------------------------------------------------------------------------------
class OwkWord(C.Structure):
    _fields_ = [("word", C.c_char_p), ("start", C.c_float), ("end", C.c_float), ("probability", C.c_float)]


class OwkDseg(C.Structure):
    _fields_ = [("speaker", C.c_char_p), ("start", C.c_float), ("end", C.c_float)]


class OwkAlignOptions(C.Structure):
    _fields_ = [("fill_nearest", C.c_int), ("sentence_smoothing", C.c_int), ("max_words_in_sentence", C.c_int)]


class AlignmentFailed(ValueError):
    """DiarizationError.alignmentFailed of the reference SDK."""


def _diarize_protos(L):
    vp, ip, fp, cp = C.c_void_p, C.c_int, C.POINTER(C.c_float), C.c_char_p
    L.owk_align_default_options.restype = OwkAlignOptions
    L.owk_align.restype = vp
    L.owk_align.argtypes = [C.POINTER(OwkWord), ip, C.POINTER(OwkDseg), ip, OwkAlignOptions]
    L.owk_alignment_free.argtypes = [vp]
    L.owk_alignment_n_words.argtypes = [vp]
    L.owk_alignment_word_speaker.argtypes = [vp, ip]
    L.owk_alignment_word_speaker.restype = cp
    L.owk_alignment_n_utterances.argtypes = [vp]
    L.owk_alignment_utterance.argtypes = [vp, ip, C.POINTER(cp), C.POINTER(cp), fp, fp, C.POINTER(ip), C.POINTER(ip)]
    L.owk_alignment_text.argtypes = [vp]
    L.owk_alignment_text.restype = cp
    L.owk_rttm_parse.restype = vp
    L.owk_rttm_parse.argtypes = [cp]
    L.owk_rttm_n_segments.argtypes = [vp]
    L.owk_rttm_segment.argtypes = [vp, ip, C.POINTER(cp), fp, fp]
    L.owk_rttm_free.argtypes = [vp]
    L.owk_rttm_generate.argtypes = [C.POINTER(OwkDseg), ip, cp, C.c_char_p, ip]


def _dec(b):
    return None if b is None else b.decode("utf-8")


def align(words, segments, fill_nearest=False, sentence_smoothing=True, max_words_in_sentence=50):
    """DiarizationAligner.align: words = [(text, start, end, prob)], segments = [(speaker, start, end)].
    Returns {"words": [(text, start, end, speaker)], "segments": [{speaker, text, start, end, words}], "text"}."""
    L = load()
    _diarize_protos(L)
    W = (OwkWord * max(1, len(words)))(*[OwkWord(w[0].encode(), w[1], w[2], w[3] if len(w) > 3 else 0.0) for w in words])
    S = (OwkDseg * max(1, len(segments)))(*[OwkDseg(s[0].encode(), s[1], s[2]) for s in segments])
    opt = OwkAlignOptions(int(fill_nearest), int(sentence_smoothing), int(max_words_in_sentence))
    h = L.owk_align(W, len(words), S, len(segments), opt)
    if not h:
        raise AlignmentFailed("maxWordsInSentence must be greater than 0")
    try:
        out_words = [(w[0], w[1], w[2], _dec(L.owk_alignment_word_speaker(h, i))) for i, w in enumerate(words)]
        utts = []
        for i in range(L.owk_alignment_n_utterances(h)):
            spk, txt = C.c_char_p(), C.c_char_p()
            t0, t1 = C.c_float(), C.c_float()
            first, n = C.c_int(), C.c_int()
            L.owk_alignment_utterance(h, i, C.byref(spk), C.byref(txt), C.byref(t0), C.byref(t1), C.byref(first),
                                      C.byref(n))
            utts.append({"speaker": _dec(spk.value), "text": _dec(txt.value), "start": t0.value, "end": t1.value,
                         "words": list(range(first.value, first.value + n.value))})
        return {"words": out_words, "segments": utts, "text": _dec(L.owk_alignment_text(h))}
    finally:
        L.owk_alignment_free(h)


def rttm_parse(text):
    """RTTMParser.parse -> [(speaker, start, end)] sorted by start."""
    L = load()
    _diarize_protos(L)
    h = L.owk_rttm_parse(text.encode())
    try:
        out = []
        for i in range(L.owk_rttm_n_segments(h)):
            spk = C.c_char_p()
            t0, t1 = C.c_float(), C.c_float()
            L.owk_rttm_segment(h, i, C.byref(spk), C.byref(t0), C.byref(t1))
            out.append((_dec(spk.value), t0.value, t1.value))
        return out
    finally:
        L.owk_rttm_free(h)


def rttm_generate(segments, filename):
    """RTTMParser.generate for [(speaker, start, end)]."""
    L = load()
    _diarize_protos(L)
    S = (OwkDseg * max(1, len(segments)))(*[OwkDseg(s[0].encode(), s[1], s[2]) for s in segments])
    n = L.owk_rttm_generate(S, len(segments), filename.encode(), None, 0)
    buf = C.create_string_buffer(n + 1)
    L.owk_rttm_generate(S, len(segments), filename.encode(), buf, n + 1)
    return buf.value.decode()
