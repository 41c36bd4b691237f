"""profiles/<tag>_rocprof_stages.json from a rocprofv3 --kernel-trace --stats summary of bench.py:
per bench stage, the summed duration of its dispatches / the profiled steps (one k_blur dispatch
per step), so bench.py can give every stage's roofline fraction from the profiler beside its live
HIP-event figure.  Usage:
    python tools/rocprof_stages.py <run_kernel_stats.csv> <head> "<bench command>" > profiles/r04_rocprof_stages.json
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_prof import short  # noqa: E402

STEP_KERNEL = "k_blur"  # one dispatch per stereo_frames_device call (step)


def main(path, head, command=""):
    tot, calls = {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            tot[k] = tot.get(k, 0.0) + float(row["TotalDurationNs"])
            calls[k] = calls.get(k, 0) + int(row["Calls"])
    steps = calls.get(STEP_KERNEL) or calls.get("k_fastblur") or 1
    stages = {k: {"total_ns": int(v), "dispatches": calls[k], "ms_per_step": v / steps / 1e6}
              for k, v in sorted(tot.items()) if k.startswith("k_")}
    json.dump(dict(source="rocprofv3 --kernel-trace --stats; tools/rocprof_stages.py", csv=os.path.basename(path),
                   head=head, command=command, steps=steps, stages=stages), sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
