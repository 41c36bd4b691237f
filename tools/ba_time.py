"""Time Optimizer::LocalBundleAdjustment on the config-4 problem (GPU handle, repeated calls)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import Optimizer, synth  # noqa: E402


def main(reps=10):
    P = synth.localba_problem(seed=7)
    o = Optimizer(0)
    # A/B hook (tools only): ORBX_TOOL_BA_OPTS="split_ctl=1,..." -> orbx_ba_debug_options of the handle
    import os
    opts = os.environ.get("ORBX_TOOL_BA_OPTS")
    if opts:
        o.set_debug_options(**{k: int(v) for k, v in (kv.split("=") for kv in opts.split(","))})
    r = o.LocalBundleAdjustment(P)  # warm-up (allocations, code load)
    ts = []
    t0 = time.perf_counter()
    for _ in range(reps):
        t1 = time.perf_counter()
        r = o.LocalBundleAdjustment(P)
        ts.append(time.perf_counter() - t1)
    dt = (time.perf_counter() - t0) / reps
    its = sum(r["iterations"])
    print(json.dumps(dict(ms_per_call=dt * 1e3, median_ms=float(np.median(ts)) * 1e3, iterations=r["iterations"], trials=r["trials"],
                          iters_per_s=its / dt, trials_per_s=r["trials"] / dt,
                          edges=int(len(P["edge_point"])))))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
