"""Per-phase cycles of the k_ba_lin_schur blocks in the last launch of a config-4 LocalBA call
(probe build: tools/build_variant.sh lsprobe -DORBX_LS_PROBE; ORBX_LIB_OVERRIDE=build_ab/lsprobe/liborbx.so).
Stamps (thread 0 of each block): 0 entry, 1 edge linearised, 2 pose terms stored, 3 point sums and
D^-1 done, 4 after the barrier, 5 B D^-1 / cf stored.  Prints median / max over blocks of each phase
and of the block start skew and end, in shader cycles."""
import ctypes as C
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import Optimizer, _lib, synth  # noqa: E402


def main():
    L = _lib.lib()
    if not hasattr(L, "orbx_debug_ls_probe"):
        raise SystemExit("not a probe build (ORBX_LIB_OVERRIDE=build_ab/lsprobe/liborbx.so)")
    P = synth.localba_problem(seed=7)
    o = Optimizer(0)
    o.LocalBundleAdjustment(P)
    o.LocalBundleAdjustment(P)
    buf = (C.c_ulonglong * (1024 * 8))()
    if L.orbx_debug_ls_probe(buf) != 0:
        raise SystemExit("probe read failed")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)
    a = a[a[:, 0] > 0]
    nb = len(a)
    t0 = a[:, 0].min()
    out = dict(blocks=nb)
    names = ["lin_edge", "pose_terms", "point_sums", "barrier", "bd_cf"]
    for i, n in enumerate(names):
        d = a[:, i + 1] - a[:, i]
        out[n] = dict(median=int(np.median(d)), max=int(d.max()))
    out["start_skew"] = dict(median=int(np.median(a[:, 0] - t0)), max=int((a[:, 0] - t0).max()))
    out["end"] = dict(median=int(np.median(a[:, 5] - t0)), max=int((a[:, 5] - t0).max()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
