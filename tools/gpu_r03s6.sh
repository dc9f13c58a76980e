#!/bin/bash
set -o pipefail
T=gpurun_out/r03s6; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k "epilogue" --timeout 120 --timeout-method thread > $T/epi.log 2>&1; rc=$?
tail -3 $T/epi.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $T/epi.log | head; exit $rc; }
OWK_GEMM256=8 timeout -k 10 120 python -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools')
import gemm_big_check as G, numpy as np, ctypes as C, json
L=G.owk.load(); L.owk_debug_gemm.argtypes=[C.c_int]*4+[C.POINTER(C.c_uint16)]*2+[C.POINTER(C.c_float)]
rng=np.random.default_rng(0)
for M,N,K in [(4100,1280,1280),(3000,2560,640),(6000,1536,5120),(2048,1024,64)]:
    a=rng.uniform(-1,1,(M,K)).astype(np.float16); w=rng.uniform(-1,1,(N,K)).astype(np.float16); out=np.zeros((M,N),np.float32)
    P=lambda x: x.view(np.uint16).ctypes.data_as(C.POINTER(C.c_uint16))
    rc=L.owk_debug_gemm(0,M,N,K,P(a),P(w),out.ctypes.data_as(C.POINTER(C.c_float)))
    ref=a.astype(np.float64)@w.astype(np.float64).T
    print(json.dumps({'8p_check':[M,N,K],'rc':rc,'err':float(np.abs(out-ref).max())}),flush=True)
" > $T/check.txt 2>&1 || { cat $T/check.txt; exit 1; }
cat $T/check.txt
timeout -k 10 600 python tools/gemm_big_check.py > $T/bench.txt 2>&1 || { tail $T/bench.txt; exit 1; }
grep gemm $T/bench.txt
