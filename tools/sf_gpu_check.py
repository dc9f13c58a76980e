"""Quick GPU-vs-golden report for the SortFormer path (diagnostic; the tests are tests/test_sortformer.py)."""
import json, os, sys, time
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S, sortformer as SF, sortformer_synth as SS
G = os.path.join(ROOT, "tests", "golden")
meta = json.load(open(os.path.join(G, "sf_golden.json"))); A = np.load(os.path.join(G, "sf_golden.npz"))
cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models"); os.makedirs(cache, exist_ok=True)
path = os.path.join(cache, f"synth-sortformer-s{meta['seed']}.gguf")
assert SS.write_model(path, meta["seed"]) == meta["sha256"]
sf = SF.Sortformer(path)
def rep(name, got, want):
    d = np.abs(got.astype(np.float64) - want); print(f"{name:28s} shape {got.shape} max|d| {d.max():.3e} mean|d| {d.mean():.3e} max|want| {np.abs(want).max():.3e}", flush=True)
test60 = S.read_wav_16k_mono(os.path.join(G, "sf_test60.wav"))
mel, seq = sf.mel(test60[:16000 * 15]); rep("mel", mel, A["stage/mel"])
rep("preenc", sf.preenc(A["stage/mel"], meta["results"]["stage/seq_len"]), A["stage/preenc"])
for L in (0, 16): rep(f"conf{L}", sf.conformer(A["stage/preenc"], L), A[f"stage/conf{L}"])
rep("proj", sf.projection(A["stage/conf16"]), A["stage/proj"])
for L in (0, 17): rep(f"trans{L}", sf.transformer(A["stage/proj"], L), A[f"stage/trans{L}"])
rep("pred", sf.prediction(A["stage/trans17"]), A["stage/pred"])
t = time.time(); p = sf.diarize(test60); el = time.time() - t
rep("diarize/test60", p, A["diarize/test60"]); print("  diarize 60 s:", el, "s")
r = SF.to_rttm(p, 0.5, 11, "/x/test60.wav"); print("  rttm identical:", r == meta["results"]["rttm/test60"])
p2 = sf.diarize(S.synth_audio(16000 * 45, 11)); rep("diarize/synth45", p2, A["diarize/synth45"])
sf2 = SF.Sortformer(path, chunk_len=48, fifo_len=40, spkcache_update_period=64, right_context=2, chunk_left_context=2)
rep("diarize_fifo", sf2.diarize(test60), A["diarize_fifo/test60"])
for name, (preset, blocks) in {"2s_blocks8000": ("2s", [8000]), "low_ragged": ("low", [3200, 7000, 160, 12345, 999]), "5s_blocks16000": ("5s", [16000])}.items():
    st = sf.stream(preset); outs=[]; counts=[]; pos=0; i=0
    while pos < len(test60):
        n = min(blocks[i % len(blocks)], len(test60)-pos); o = st.feed(test60[pos:pos+n]); outs.append(o); counts.append(o.shape[0]); pos += n; i += 1
    fl = st.flush(); outs.append(fl); counts.append(fl.shape[0])
    print("  counts equal:", counts == meta["results"][f"stream_counts/{name}"])
    rep("stream/" + name, np.concatenate(outs), A["stream/" + name])
# timing: 10 min synthetic
x = S.synth_audio(16000 * 600, 3)
sf.diarize(x[:16000*30]); t = time.time(); p = sf.diarize(x); el = time.time() - t
print(f"diarize 600 s: {el:.3f} s  RTF {600/el:.1f}")
