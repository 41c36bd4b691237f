"""LocalBA throughput with K config-4-shaped problems (different seeds) in ONE batched call
(orbx_ba_run_many): every LM trial kernel runs once for all K problems."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import Optimizer, synth  # noqa: E402


def main(K=8, calls=10):
    probs = [synth.localba_problem(seed=7 + 1000 * k) for k in range(K)]
    o = Optimizer(0)
    o.LocalBundleAdjustmentMany(probs)  # warm-up (allocations)
    t0 = time.perf_counter()
    its = 0
    for _ in range(calls):
        rs = o.LocalBundleAdjustmentMany(probs)
        its += sum(sum(r["iterations"]) for r in rs)
    el = time.perf_counter() - t0
    print(json.dumps(dict(K=K, calls=calls, iters_per_s=round(its / el, 1), ms_per_call=round(el / calls * 1e3, 3))))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8, int(sys.argv[2]) if len(sys.argv) > 2 else 10)
