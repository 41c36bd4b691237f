"""Kernel timeline of the drop-in single stereo frame (shim/build/frame_bench, the bench's
single_frame leg) from a rocprofv3 kernel-trace directory: per frame, the device span from the first
kernel to the last, the kernel-busy time, and the per-kernel durations.
  python tools/single_frame_prof.py make FILE N      # write N KITTI-shaped synthetic stereo pairs
  python tools/single_frame_prof.py parse DIR        # summarise DIR's *kernel_trace.csv"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def make(path, n):
    from orb_slam2_commit_amd import synth
    with open(path, "wb") as f:
        for s in synth.sequence_seeds(0, n):
            L, R = synth.stereo_pair(s, 1241, 376)
            f.write(np.ascontiguousarray(L).tobytes())
            f.write(np.ascontiguousarray(R).tobytes())


def parse(d):
    fs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    ks = []
    for f in fs:
        ks += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):  # rocprofv3's default rocpd output
        import sqlite3
        ks += list(sqlite3.connect(f).execute("select start, end, name from kernels"))
    ks = sorted((a, b, n.split("(")[0].split("<")[0].replace("void ", "")) for a, b, n in ks)
    # frames: a k_stereo_finalize closes each frame
    frames, cur = [], []
    for k in ks:
        cur.append(k)
        if "k_stereo_finalize" in k[2]:
            frames.append(cur)
            cur = []
    frames = frames[20:]  # the warm-up frames
    span, busy, per = [], [], defaultdict(list)
    for fr in frames:
        span.append((fr[-1][1] - fr[0][0]) / 1e3)
        # busy = union of kernel intervals
        t, e0 = 0, None
        s0 = None
        for a, b, _ in sorted(fr):
            if s0 is None or a > e0:
                if s0 is not None:
                    t += e0 - s0
                s0, e0 = a, b
            else:
                e0 = max(e0, b)
        t += e0 - s0
        busy.append(t / 1e3)
        agg = defaultdict(float)
        for a, b, n in fr:
            agg[n] += (b - a) / 1e3
        for n, v in agg.items():
            per[n].append(v)
    out = dict(frames=len(frames), kernels_per_frame=len(frames[0]) if frames else 0,
               span_us_median=float(np.median(span)), busy_us_median=float(np.median(busy)),
               per_kernel_us_median={n: round(float(np.median(v)), 2) for n, v in sorted(per.items(), key=lambda x: -np.median(x[1]))})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "make":
        make(sys.argv[2], int(sys.argv[3]))
    else:
        parse(sys.argv[2])
