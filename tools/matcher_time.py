"""Per-call time of the loop-closing / initialisation matchers (DESIGN rows F8b-F8e) on the GPU through
the host C-ABI (host arrays in and out, one problem per call), beside the oracle's single-thread time.
Usage: python tools/matcher_time.py > profiles/r04_matcher_time.json"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from test_projection import _init_case, _sim3, _sim3_pair_case  # noqa: E402
from orb_slam2_commit_amd import ORBmatcher, synth  # noqa: E402


def timeit(fn, reps):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return float(np.median(t)) * 1e3


m = ORBmatcher(0.9, True)
out = {"note": "median ms per call, host arrays in/out through the C-ABI (PCIe-inclusive); oracle = "
               "oracle/ C++ restatement, one thread", "calls": {}}
f1, f2, prev = _init_case(1200, n=2000)
out["calls"]["SearchForInitialization (N1=2000, N2=2600, window 100)"] = dict(
    gpu_ms=timeit(lambda: m.SearchForInitialization(f1, f2, prev, 100), 20),
    oracle_ms=timeit(lambda: oracle.search_for_initialization(f1, f2, prev, 100, 0.9, True), 5),
    nmatches=int(m.SearchForInitialization(f1, f2, prev, 100)[0]))
fr = synth.projection_frame(100, n=2000)
pts = synth.projection_points(200, fr, 3, n_points=3000)
f4 = _sim3(fr, 0)
out["calls"]["SearchByProjection(KF, Scw) (2000 features, 3000 points, th 10)"] = dict(
    gpu_ms=timeit(lambda: m.SearchByProjectionSim3(f4, f4["Tcw"], pts, 10), 20),
    oracle_ms=timeit(lambda: oracle.search_by_projection(f4, pts, 4, th=10.0), 5))
out["calls"]["Fuse(KF, Scw) matching half (2000 features, 3000 points, th 4)"] = dict(
    gpu_ms=timeit(lambda: m.FuseSim3(f4, f4["Tcw"], pts, 4.0), 20),
    oracle_ms=timeit(lambda: oracle.search_by_projection(f4, pts, 5, th=4.0), 5))
kf1, kf2, p1, p2, s, R12, t12 = _sim3_pair_case(950, n=2000, s12=1.1)
out["calls"]["SearchBySim3 (2000 + 2000 features, th 7.5)"] = dict(
    gpu_ms=timeit(lambda: m.SearchBySim3(kf1, kf2, p1, p2, s, R12, t12, 7.5), 20),
    oracle_ms=timeit(lambda: oracle.search_by_sim3(kf1, kf2, p1, p2, s, R12, t12, 7.5), 5))
print(json.dumps(out, indent=1))
