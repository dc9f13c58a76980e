"""Extract the DATA sections (mel filterbank + tokenizer vocab) of the reference's own
weightless test models (models/for-tests-ggml-*.bin, used by tests/CMakeLists.txt:18-89)
into open-whisper-kit_amd/assets/ so synthetic-weight models can be written on machines
without /root/reference. Runs only where /root/reference exists; outputs are committed.

File layout read here: whisper_model_load, src/whisper.cpp:1496-1675
(magic, 11 x i32 hparams, filters {n_mel, n_fft, f32[n_mel*n_fft]}, vocab {n, (len u32, bytes)*}).
"""
import gzip, os, struct, sys
import numpy as np

REF = "/root/reference/models"
OUT = os.path.join(os.path.dirname(__file__), "..", "open-whisper-kit_amd", "assets")

def split(path):
    b = open(path, "rb").read()
    off = 4 + 11 * 4
    n_mel, n_fft = struct.unpack_from("<ii", b, off); off += 8
    filt = np.frombuffer(b, dtype="<f4", count=n_mel * n_fft, offset=off).reshape(n_mel, n_fft)
    off += n_mel * n_fft * 4
    vstart = off
    n_vocab, = struct.unpack_from("<i", b, off); off += 4
    for _ in range(n_vocab):
        ln, = struct.unpack_from("<I", b, off); off += 4 + ln
    assert off == len(b), (off, len(b))  # weightless: nothing after the vocab
    return filt, b[vstart:off]

if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    f_en, v_en = split(os.path.join(REF, "for-tests-ggml-tiny.en.bin"))
    f_ml, v_ml = split(os.path.join(REF, "for-tests-ggml-tiny.bin"))
    assert np.array_equal(f_en, f_ml)
    np.save(os.path.join(OUT, "mel_filters_80.npy"), np.ascontiguousarray(f_en))
    for name, v in (("vocab_en.bin.gz", v_en), ("vocab_multilingual.bin.gz", v_ml)):
        with gzip.GzipFile(os.path.join(OUT, name), "wb", mtime=0) as f:
            f.write(v)
    print("ok", f_en.shape, len(v_en), len(v_ml))
