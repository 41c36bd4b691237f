"""Time orbx_pnp_iterate_many on a config-3 frame batch (B solvers, 1200 matches, 40 % outliers)."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import PnPsolver, synth  # noqa: E402
from orb_slam2_commit_amd.glibc_rand import GlibcRand  # noqa: E402
from orb_slam2_commit_amd.orb import pnp_iterate_many  # noqa: E402

PRM = (0.99, 10, 300, 4, 0.5, 5.991)


def main(B=128, reps=5):
    probs = [synth.pnp_problem(seed=3000 + f, n=1200, outlier_frac=0.4) for f in range(B)]
    rngs = [GlibcRand(1 + f) for f in range(B)]
    ts = []
    for r in range(reps + 1):
        sv = PnPsolver.create_many(probs, *PRM)
        t0 = time.perf_counter()
        res = pnp_iterate_many(sv, 5, rngs)
        t1 = time.perf_counter()
        for s in sv:
            s.close()
        if r:
            ts.append(t1 - t0)
    found = sum(1 for x in res if x[0] is not None)
    print(json.dumps(dict(B=B, ms=[round(t * 1e3, 3) for t in ts], found=found)))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
