import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "open-whisper-kit_amd", "python"))
import owk, owk_synth as S
owk.quiet()
pcm = S.synth_audio(480000, 7)
path = S.ensure_model("tiny.en", 1234)
for fa, preset in ((True, 0), (False, 0), (False, 3)):
    w = owk.Whisper(path, flash_attn=fa, dtw_preset=preset)
    st = w.new_state()
    p = w.params(0, language="en", temperature_inc=0.0)
    ret = w.full(st, pcm, p)
    print(fa, preset, ret, [(s['t0'], s['t1'], [t[0] for t in s['tokens']], [t[3] for t in s['tokens']][:2]) for s in w.segments(st)], flush=True)
    w.close()
