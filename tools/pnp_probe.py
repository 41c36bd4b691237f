"""Phase timing of one Refine() EPnP (s_memtime stamps of a probe build, build_ab/probe)."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import PnPsolver, _lib, synth  # noqa: E402
from orb_slam2_commit_amd.glibc_rand import GlibcRand  # noqa: E402

P = synth.pnp_problem(seed=3, n=1200, outlier_frac=0.25, noise_px=0.5)
s = PnPsolver(P["p3d"], P["p2d"], P["sigma2"], P["fx"], P["fy"], P["cx"], P["cy"])
s.SetRansacParameters(0.99, 10, 300, 4, 0.5, 5.991)
T, nm, inl, ni = s.iterate(5, GlibcRand(1))
buf = (C.c_ulonglong * 64)()
_lib.lib().orbx_debug_pnp_probe(buf)
v = np.array(buf[:], np.int64)
names = ["start", "cws+pw0tpw0+svd", "alphas", "MtM", "jacobi12", "L,rho", "pw0", "betas+GN(w0)", "pcs/abt/svd/err",
         "rep", "end"]
print("found", T is not None, "inliers", ni)
for w in range(4):
    row = v[16 * w:16 * w + 11]
    print("wave", w, [int(x - v[0]) if x else None for x in row])
