"""Per-level FAST survivor counts (k_octree's T) on bench-like KITTI frames, beside the LDS slots
the plan gives k_octree (Geometry::oct_kcap): candidates past kcap live in global scratch and are
re-read every split round."""
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import ORBextractor, _lib, synth  # noqa: E402


def dbg(ex, what, image=0, arg=0, dtype=np.int32):
    L = _lib.lib()
    n = L.orbx_debug_copy(ex._h, what, image, arg, None, 0)
    buf = np.zeros(n, np.uint8)
    L.orbx_debug_copy(ex._h, what, image, arg, _lib.ptr(buf), n)
    return buf.view(dtype)


def main(n=4):
    imgs = synth.stereo_batch(0, n)
    ex = ORBextractor(2000, 1.2, 8, 20, 7)
    per = []
    for i in range(2 * n):
        ex(imgs[i])
        cells = dbg(ex, 3).reshape(-1, 8)
        counts = dbg(ex, 2)
        T = np.bincount(cells[:, 0], weights=counts, minlength=8).astype(int)
        ncell = np.bincount(cells[:, 0], minlength=8)
        per.append(T)
    per = np.array(per)
    print(json.dumps(dict(T_mean=per.mean(0).round(1).tolist(), T_max=per.max(0).tolist(),
                          cells_per_level=ncell.tolist())))


if __name__ == "__main__":
    main()
