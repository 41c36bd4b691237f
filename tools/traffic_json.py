"""profiles/traffic.json from tools/traffic_now.sh output: HBM bytes per bench stage event
(2*FETCH_SIZE*1024 + WRITE_SIZE*1024, the gfx950 correction of tools/parse_prof.py).

A stage event is what bench.py's per-stage timer brackets: one launch for most stages, one per
level for k_resize, and every launch group of k_fast together (k_fast runs as up to two launches
per step, split by LDS size), so k_fast's bytes are summed over its dispatches of a step (steps are
counted by k_blur's dispatches, one per step).
Usage: python tools/traffic_json.py gpurun_out/tn HEAD [batch] > profiles/traffic.json"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_prof import short  # noqa: E402


def load(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


# bench stages timed as ONE event per step though they run as several launches (k_fast: LDS launch
# groups; k_octree: level groups; k_describe: k_orient + k_rbrief): bytes summed over the step
STEP_STAGES = ("k_fast", "k_octree", "k_describe")


def main(d, head, batch="256"):
    f = load(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = load(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    steps = max(len(f.get("k_blur", [])), 1)
    out, disp = {}, {}
    for k in sorted(set(f) | set(w)):
        n = max(len(f.get(k, [])), len(w.get(k, [])), 1)
        total = 2.0 * sum(f.get(k, [])) * 1024 + sum(w.get(k, [])) * 1024
        per_event = total / steps if k in STEP_STAGES else total / n
        out[k] = int(per_event)
        disp[k] = n
    json.dump(dict(source="tools/traffic_now.sh + tools/traffic_json.py", head=head, batch=int(batch),
                   per_launch_bytes=out, dispatches=disp, steps=steps,
                   note="2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per bench stage event (k_fast, k_octree, "
                        "k_describe: per step, summed over their launches; others: per dispatch)"), sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
