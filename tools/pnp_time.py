"""Time PnPsolver.iterate on the config-3 shaped problems (GPU) beside the oracle."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/oracle")
from orb_slam2_commit_amd import PnPsolver, synth  # noqa: E402
from orb_slam2_commit_amd.glibc_rand import GlibcRand  # noqa: E402

PARAMS = (0.99, 10, 300, 4, 0.5, 5.991)


def run(name, n, of, noise, seed, reps=10, cpu=True):
    P = synth.pnp_problem(seed=seed, n=n, outlier_frac=of, noise_px=noise)
    args = (P["p3d"], P["p2d"], P["sigma2"], P["fx"], P["fy"], P["cx"], P["cy"])
    t0 = time.perf_counter()
    for _ in range(reps):
        s = PnPsolver(*args)
        s.SetRansacParameters(*PARAMS)
        T, nm, inl, ni = s.iterate(5, GlibcRand(1))
        s.close()
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    out = dict(case=name, n=n, found=T is not None, inliers=ni, gpu_ms_per_solve=round(gpu_ms, 3))
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
