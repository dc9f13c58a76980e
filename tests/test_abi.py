"""CPU: the drop-in library loads without a GPU, exports every symbol include/*.h declares,
and the public structs have the reference layout (whisper.h by value ABI)."""
import ctypes as C
import os
import shutil
import subprocess

import pytest

import owk

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "whisper.h"
#define P(x) printf("%s %zu\n", #x, (size_t)(x));
int main(void) {
    P(sizeof(struct whisper_context_params));
    P(sizeof(struct whisper_token_data));
    P(sizeof(struct whisper_full_params));
    P(sizeof(struct whisper_vad_params));
    P(offsetof(struct whisper_full_params, n_threads));
    P(offsetof(struct whisper_full_params, token_timestamps));
    P(offsetof(struct whisper_full_params, max_tokens));
    P(offsetof(struct whisper_full_params, suppress_regex));
    P(offsetof(struct whisper_full_params, language));
    P(offsetof(struct whisper_full_params, temperature));
    P(offsetof(struct whisper_full_params, greedy));
    P(offsetof(struct whisper_full_params, beam_search));
    P(offsetof(struct whisper_full_params, new_segment_callback));
    P(offsetof(struct whisper_full_params, logits_filter_callback));
    P(offsetof(struct whisper_full_params, grammar_rules));
    P(offsetof(struct whisper_full_params, vad));
    P(offsetof(struct whisper_full_params, vad_params));
    P(offsetof(struct whisper_context_params, dtw_aheads));
    P(offsetof(struct whisper_token_data, t_dtw));
    return 0;
}
"""


def _probe(tmp_path, includes):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not available")
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run([gcc, "-std=c11", *[f"-I{i}" for i in includes], str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return dict((ln.rsplit(" ", 1)[0], int(ln.rsplit(" ", 1)[1])) for ln in out.strip().splitlines())


def test_library_exports_every_header_symbol():
    lib = owk.load()
    syms = owk.header_symbols()
    assert len(syms) > 100
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_binding_matches_header(tmp_path):
    got = _probe(tmp_path, [os.path.join(ROOT, "include")])
    assert got["sizeof(struct whisper_full_params)"] == C.sizeof(owk.FullParams)
    assert got["sizeof(struct whisper_context_params)"] == C.sizeof(owk.ContextParams)
    assert got["sizeof(struct whisper_token_data)"] == C.sizeof(owk.TokenData)
    assert got["offsetof(struct whisper_full_params, logits_filter_callback)"] == owk.FullParams.logits_filter_callback.offset
    assert got["offsetof(struct whisper_full_params, vad_params)"] == owk.FullParams.vad_params.offset


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="reference sources not present")
def test_header_layout_identical_to_reference(tmp_path):
    ours = _probe(tmp_path, [os.path.join(ROOT, "include")])
    (tmp_path / "r").mkdir()
    ref = _probe(tmp_path / "r", ["/root/reference/include", "/root/reference/ggml/include"])
    assert ours == ref


def test_library_reports_gfx950_build():
    lib = owk.load()
    lib.owk_build_info.restype = C.c_char_p
    info = lib.owk_build_info().decode()
    assert "gfx950" in info
