"""Time PnPsolver.iterate on the config-3 shaped problems (GPU) beside the oracle."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/oracle")
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402

from orb_slam2_commit_amd import PnPsolver, _lib, synth  # noqa: E402
from orb_slam2_commit_amd.glibc_rand import GlibcRand  # noqa: E402

PARAMS = (0.99, 10, 300, 4, 0.5, 5.991)


def run(name, n, of, noise, seed, reps=10, cpu=True):
    P = synth.pnp_problem(seed=seed, n=n, outlier_frac=of, noise_px=noise)
    args = (P["p3d"], P["p2d"], P["sigma2"], P["fx"], P["fy"], P["cx"], P["cy"])
    t_create = t_iter = t_close = 0.0
    for rep in range(reps + 1):  # rep 0 warms up (first-use init, pool growth)
        t0 = time.perf_counter()
        s = PnPsolver(*args)
        s.SetRansacParameters(*PARAMS)
        st = _lib.RandState()
        _lib.lib().orbx_rand_seed(C.byref(st), 1)
        nm_, ni_, found_ = C.c_int(), C.c_int(), C.c_int()
        Tb = np.zeros(16, np.float32)
        inl = np.zeros(max(n, 1), np.uint8)
        t1 = time.perf_counter()
        rc = _lib.lib().orbx_pnp_iterate_stream(s._h, 5, C.byref(st), C.byref(nm_), _lib.ptr(Tb), _lib.ptr(inl),
                                                C.byref(ni_), C.byref(found_))
        t2 = time.perf_counter()
        assert rc == 0
        T, ni = (Tb if found_.value else None), ni_.value
        s.close()
        t3 = time.perf_counter()
        if rep:
            t_create += t1 - t0
            t_iter += t2 - t1
            t_close += t3 - t2
    gpu_ms = (t_create + t_iter + t_close) / reps * 1e3
    out = dict(case=name, n=n, found=T is not None, inliers=ni, gpu_ms_per_solve=round(gpu_ms, 3),
               create_ms=round(t_create / reps * 1e3, 3), iterate_ms=round(t_iter / reps * 1e3, 3),
               close_ms=round(t_close / reps * 1e3, 3))
    if cpu:
        import oracle
        t0 = time.perf_counter()
        for _ in range(reps):
            o = oracle.PnPsolver(*args, *PARAMS)
            o.iterate(5, GlibcRand(1))
        out["oracle_ms_per_solve"] = round((time.perf_counter() - t0) / reps * 1e3, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    run("config3", 1200, 0.4, 1.0, 3)
    run("refine_1200", 1200, 0.3, 0.5, 5)
    run("reloc_150", 150, 0.5, 0.5, 21)
