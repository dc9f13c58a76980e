# A/B: k_sm_split_pv's last-arriver reduction (one memory round trip through LDS) against HEAD's
#   tools/ab_smpv.sh LIB_A LIB_B   (outputs gpurun_out/r06v/)
set -o pipefail
export OWK_MODEL_CACHE=/tmp/owk_models
O=gpurun_out/r06v
mkdir -p $O
for v in a b a b; do
  if [ $v = a ]; then export OWK_LIB=$1; else export OWK_LIB=$2; fi
  OWK_LIB=$OWK_LIB timeout -k 10 120 python3 -u -c "
import ctypes as C, os
L = C.CDLL(os.environ['OWK_LIB'])
L.owk_debug_attn_softmax.restype = C.c_double
L.owk_debug_attn_softmax.argtypes = [C.c_int] * 5 + [C.c_void_p, C.c_void_p, C.c_int]
for R in (1, 2):
    for T in (448, 1500):
        us = min(L.owk_debug_attn_softmax(0, 1, R, 20, T, None, None, 50) for _ in range(5))
        print('$v', {'rows': R, 'keys': T, 'keysplit_us': round(us, 2)}, flush=True)
" >> $O/split.txt || exit 1
  timeout -k 10 400 python3 -u tools/seq_asr.py --minutes 2 > $O/seq_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $O/seq_$v.txt)" >> $O/seq.txt
done
unset OWK_LIB
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -k "softmax or split" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/kernels.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_c4.py -v -rP --timeout 400 --timeout-method thread -p no:cacheprovider > $O/c4.txt 2>&1
