set -o pipefail
mkdir -p gpurun_out/diag
export OWK_MODEL_CACHE=/tmp/owk_models
for lib in new old; do
  L=open-whisper-kit_amd/lib/libwhisper.so; [ $lib = old ] && L=open-whisper-kit_amd/lib_old/libwhisper.so
  OWK_LIB=$L timeout -k 10 120 python tools/diag_tokens.py base.en test60 gpurun_out/diag/$lib.json temperature_inc=0.0 no_context=False || exit 1
done
python - <<'PY'
import json
a=json.load(open('gpurun_out/diag/new.json')); b=json.load(open('gpurun_out/diag/old.json'))
fa=[(i,t) for i,s in enumerate(a['segments']) for t in s['tokens']]; fb=[(i,t) for i,s in enumerate(b['segments']) for t in s['tokens']]
for k,(x,y) in enumerate(zip(fa,fb)):
    if x[1][0]!=y[1][0] or x[1][1]!=y[1][1]:
        print('first diff at', k, 'seg', x[0], y[0], 'new', x[1][:4], 'old', y[1][:4]); break
else: print('identical', len(fa), len(fb))
import numpy as np
pa=np.array([t[1][2] for t in zip(fa,fb)]) if False else None
n=min(len(fa),len(fb)); d=[abs(fa[i][1][2]-fb[i][1][2]) for i in range(min(n,k if 'k' in dir() else n))]
print('max |dp| before diff', max(d) if d else 0)
print([ (s['t0'],s['t1'],len(s['tokens'])) for s in a['segments']][:8]); print([ (s['t0'],s['t1'],len(s['tokens'])) for s in b['segments']][:8])
PY
