"""On-box HBM stream-copy reference (orbx_debug_hbm_copy): GB/s of read + write per copy."""
import ctypes as C
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import _lib  # noqa: E402

n = 2 << 30
src = torch.ones(n, dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)
ms = C.c_float()
for _ in range(3):
    assert _lib.lib().orbx_debug_hbm_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), n, 10,
                                          C.byref(ms)) == 0
    print("%.1f GB/s" % (2 * n / (ms.value / 1e3) / 1e9))
