"""GPU kernel numerics vs a plain fp32 reference of the same op (numpy on the f16 inputs).

The GEMM dispatch covers the decode-row kernel (M <= 32, incl. split-K), the skinny
kernel (M <= 64) and the 128x128 tile kernel; f32 accumulation of exact f16 products,
so the only difference to the fp32 reference is summation order."""
import ctypes as C

import numpy as np
import pytest

import owk

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 5, 16, 17, 32, 33, 64, 65, 130])
@pytest.mark.parametrize("NK", [(384, 384), (1280, 5120), (5120, 1280), (51866, 384)])
def test_gemm_dispatch(M, NK):
    N, K = NK
    if N * K > 2e7 and M > 64:
        pytest.skip("large big-tile case covered by the parity tests")
    L = owk.load()
    rng = np.random.default_rng(M * 7 + N)
    a = (rng.standard_normal((M, K)) * 0.5).astype(np.float16)
    w = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    out = np.zeros((M, N), np.float32)
    u16 = C.POINTER(C.c_uint16)
    rc = L.owk_debug_gemm(0, M, N, K, a.view(np.uint16).ctypes.data_as(u16), w.view(np.uint16).ctypes.data_as(u16),
                          out.ctypes.data_as(C.POINTER(C.c_float)))
    assert rc == 0
    ref = a.astype(np.float32) @ w.astype(np.float32).T
    assert np.isfinite(out).all()
    np.testing.assert_allclose(out, ref, atol=2e-4 * np.sqrt(K), rtol=1e-4)
