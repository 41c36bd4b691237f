"""Per-phase s_memtime stamps of the reduced-system LDLT kernel (orbx_debug_ldlt_ex).

For the 8-wide panel kernel: stamp 0 = entry, 1 = tiles loaded and panel 0 published,
2 + 2M = panel M's look-ahead tiles updated (after the barrier), 3 + 2M = panel M+1's rows and the
rest of panel M's update done, 32 + M = panel M+1's rows done (thread 0's chain), 48 = back solve's
first block loaded, 49 + j = its j-th two-block step starts, 63 = back solve done.  Prints cycles per phase as JSON.
usage: python tools/ldlt_stamps.py [N ...]
"""
import ctypes as C
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import _lib  # noqa: E402


def stamps(N, kind=0, reps=5, seed=0):
    rng = np.random.default_rng(seed)
    M = rng.normal(size=(N, N))
    S = np.ascontiguousarray(M @ M.T + N * np.eye(N))
    b = rng.normal(size=N)
    x = np.zeros(N)
    ms = C.c_float(0)
    st = (C.c_ulonglong * 64)()
    rc = _lib.lib().orbx_debug_ldlt_ex(_lib.ptr(S), _lib.ptr(b), N, _lib.ptr(x), reps, C.byref(ms), kind,
                                       C.cast(st, C.c_void_p))
    ref = np.linalg.solve(S, b)
    t = [int(v) for v in st]
    t0 = t[0]
    marks = {i: t[i] - t0 for i in range(64) if t[i] >= t0 and t[i] != 0}
    npan = (N + 7) // 8
    out = dict(N=N, kind=kind, rc=rc, ms=ms.value, err=float(np.abs(x - ref).max() / np.abs(ref).max()),
               load=marks.get(1), total=marks.get(63))
    per = []
    prev = marks.get(1)
    for M in range(npan):
        a, c = marks.get(2 + 2 * M), marks.get(3 + 2 * M)
        if a is None or c is None or prev is None:
            break
        r = marks.get(32 + M)
        per.append(dict(M=M, lookahead=a - prev, rows_and_update=c - a, rows_chain=(r - a) if r is not None else None))
        prev = c
    out["panels"] = per
    if prev is not None and marks.get(63) is not None:
        out["back_solve"] = marks[63] - prev
        bs = [marks.get(48)] + [marks.get(49 + j) for j in range(8)] + [marks[63]]
        bs = [v for v in bs if v is not None]
        out["back_solve_head"] = bs[0] - prev if bs else None
        out["back_solve_steps"] = [b - a for a, b in zip(bs, bs[1:])]
    return out


if __name__ == "__main__":
    for N in [int(a) for a in sys.argv[1:]] or [120]:
        print(json.dumps(stamps(N)))
