"""Single-call latency of the projection-family matchers through the host C-ABI (DESIGN rows F1-F3,
F8-F8e): the problem struct is built once over host arrays, then only the C call is timed (host
arrays in and out, PCIe included), median of `reps` calls after warm-up.  The per-frame members
(SearchByProjection(F, MPs) / (F, LastF) / (F, KF)) at 2,000 features / 3,000 points, the KeyFrame
ones (Fuse, the Sim3 projections, SearchBySim3, SearchForInitialization) at the sizes of
tools/matcher_time.py.  Usage: python tools/matcher_latency.py [reps] > profiles/r05_matcher_time.json"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from test_projection import _init_case, _kw, _sim3, _sim3_pair_case  # noqa: E402
from orb_slam2_commit_amd import ORBmatcher, _lib, orb, synth  # noqa: E402
from orb_slam2_commit_amd._lib import check  # noqa: E402


def med_ms(fn, reps):
    for _ in range(3):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(float(np.median(t)) * 1e3, 4), round(float(np.percentile(t, 90)) * 1e3, 4)


def main(reps=50):
    L = _lib.lib()
    out = {"note": "median / p90 ms of one C-ABI call (host arrays in and out, PCIe included); the problem "
                   "struct is built once outside the timed call", "calls": {}}
    names = {0: "SearchByProjection(F, MPs) local map", 1: "SearchByProjection(F, LastF)",
             2: "SearchByProjection(F, KF, sAlreadyFound)", 3: "Fuse(KF, MPs) matching half",
             4: "SearchByProjection(KF, Scw)", 5: "Fuse(KF, Scw) matching half"}
    for kind in range(6):
        fr = synth.projection_frame(100, n=2000)
        pts = synth.projection_points(200, fr, min(kind, 3), n_points=3000)
        if kind >= 4:
            fr = _sim3(fr, 0)
        kw = _kw(kind, fr, 0)
        kw.pop("nnratio", None)
        frh, ptsh = orb._host_frame(fr), orb._host_points(pts)
        p, o = orb.proj_problem(frh, ptsh, kind, **kw)
        call = lambda: check(L.orbx_search_by_projection(C.byref(p), 0), "orbx_search_by_projection")
        md, p90 = med_ms(call, reps)
        out["calls"]["%s (2000 features, 3000 points)" % names[kind]] = dict(median_ms=md, p90_ms=p90,
                                                                            nmatches=int(o["nmatches"][0]))
    m = ORBmatcher(0.9, True)
    f1, f2, prev = _init_case(1200, n=2000)
    md, p90 = med_ms(lambda: m.SearchForInitialization(f1, f2, prev, 100), reps)
    out["calls"]["SearchForInitialization (N1=2000, N2=2600, window 100), Python mirror"] = dict(median_ms=md, p90_ms=p90)
    kf1, kf2, p1, p2, s, R12, t12 = _sim3_pair_case(950, n=2000, s12=1.1)
    md, p90 = med_ms(lambda: m.SearchBySim3(kf1, kf2, p1, p2, s, R12, t12, 7.5), reps)
    out["calls"]["SearchBySim3 (2000 + 2000 features, th 7.5), Python mirror"] = dict(median_ms=md, p90_ms=p90)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
