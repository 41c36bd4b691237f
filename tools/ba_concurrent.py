"""LocalBA throughput with K independent problems in flight on one GPU (one solver handle, one HIP
stream and one host thread each; ctypes releases the GIL inside orbx_ba_run)."""
import json
import sys
import threading
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orb_slam2_commit_amd import Optimizer, synth  # noqa: E402


def main(K=4, calls=10):
    probs = [synth.localba_problem(seed=7 + 1000 * k) for k in range(K)]
    opts = [Optimizer(0) for _ in range(K)]
    for o, P in zip(opts, probs):
        o.LocalBundleAdjustment(P)
    its = [0] * K

    def run(k):
        for _ in range(calls):
            r = opts[k].LocalBundleAdjustment(probs[k])
            its[k] += sum(r["iterations"])

    th = [threading.Thread(target=run, args=(k,)) for k in range(K)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    print(json.dumps(dict(K=K, calls=calls, iters_per_s=round(sum(its) / el, 1), ms_per_call=round(el / calls * 1e3, 3))))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
