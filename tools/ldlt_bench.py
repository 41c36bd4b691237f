"""Correctness + timing of the LocalBA reduced-system LDLT kernel alone."""
import ctypes as C
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import _lib  # noqa: E402


def run(N, reps=20, seed=0):
    rng = np.random.default_rng(seed)
    M = rng.normal(size=(N, N))
    S = np.ascontiguousarray(M @ M.T + N * np.eye(N))
    b = rng.normal(size=N)
    x = np.zeros(N)
    ms = C.c_float(0)
    rc = _lib.lib().orbx_debug_ldlt(_lib.ptr(S), _lib.ptr(b), N, _lib.ptr(x), reps, C.byref(ms))
    ref = np.linalg.solve(S, b)
    return dict(N=N, rc=rc, ms=ms.value, err=float(np.abs(x - ref).max() / np.abs(ref).max()))


if __name__ == "__main__":
    for N in [int(a) for a in sys.argv[1:]] or [60, 120, 138, 180, 240]:
        print(json.dumps(run(N)))
