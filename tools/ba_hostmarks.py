"""LocalBA config 4 with the trace option: the per-call host marks (intake, structure, phases,
write-back) the library prints on stderr, summarised as medians over the calls, beside the
Python-measured wall per call.  usage: python tools/ba_hostmarks.py [calls]"""
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def child(reps):
    from orb_slam2_commit_amd import Optimizer, synth
    P = synth.localba_problem(seed=7)
    o = Optimizer(0)
    o.LocalBundleAdjustment(P)
    o.set_debug_options(trace=1)
    ts = []
    for _ in range(reps):
        t1 = time.perf_counter()
        o.LocalBundleAdjustment(P)
        ts.append(time.perf_counter() - t1)
    print(json.dumps(dict(wall_median_ms=float(np.median(ts)) * 1e3)))


def main(reps):
    r = subprocess.run([sys.executable, __file__, "--child", str(reps)], capture_output=True, text=True, timeout=300)
    keys = ["total", "intake", "struct1", "phase1", "struct2", "phase2", "writeback"]
    rows = []
    for line in r.stderr.splitlines():
        if not line.startswith("[orbx_ba]"):
            continue
        v = {k: float(m) for k, m in re.findall(r"(\w+) ([0-9.]+)(?: ms)?(?=[,;)]|\s|$)", line)}
        rows.append(v)
    out = {k: round(float(np.median([v[k] for v in rows if k in v])), 4) for k in keys}
    out.update(json.loads(r.stdout.strip().splitlines()[-1]))
    out["calls"] = len(rows)
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(int(sys.argv[2]))
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
