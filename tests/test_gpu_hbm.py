"""The on-box HBM reference kernel bench.py reports beside the roofline (orbx_debug_hbm_copy)."""
import ctypes as C

import pytest


@pytest.mark.gpu
def test_gpu_hbm_copy_reference(gpu):
    import torch
    from orb_slam2_commit_amd import _lib
    n = 64 << 20
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros_like(src)
    ms = C.c_float(0)
    assert _lib.lib().orbx_debug_hbm_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), n, 3,
                                          C.byref(ms)) == 0
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    assert ms.value > 0
    assert _lib.lib().orbx_debug_hbm_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), 17, 1,
                                          C.byref(ms)) != 0  # not a multiple of 16
