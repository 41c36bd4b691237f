"""profiles/<tag>_localba_traffic.json: HBM bytes per LocalBA LM iteration from two PMC passes over
tools/ba_time.py (FETCH_SIZE pass, WRITE_SIZE pass; gfx950 correction 2*FETCH_SIZE*1024 +
WRITE_SIZE*1024, tools/parse_prof.py).  Every dispatch of the run (warm-up call + `reps` timed calls)
is summed and divided by the LM iterations those calls ran (ba_time.py's JSON line, 'iterations'
per call x (reps + 1)).  Usage:
    python tools/ba_traffic.py <dir with fetch/ and write/> <reps> <head> > profiles/r04_localba_traffic.json
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_prof import short  # noqa: E402


def load(path, counter):
    acc = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                k = short(row["Kernel_Name"])
                acc[k] = acc.get(k, 0.0) + float(row["Counter_Value"])
    return acc


def main(d, reps, head):
    reps = int(reps)
    f = load(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = load(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    line = [ln for ln in open(os.path.join(d, "fetch.log")) if ln.startswith("{")][-1]
    r = json.loads(line)
    its = sum(r["iterations"]) * (reps + 1)
    per_kernel = {k: int(2.0 * f.get(k, 0.0) * 1024 + w.get(k, 0.0) * 1024) for k in sorted(set(f) | set(w))
                  if k.startswith("k_ba")}
    total = sum(per_kernel.values())
    json.dump(dict(source="tools/ba_traffic.py (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of tools/ba_time.py)",
                   head=head, calls=reps + 1, iterations_per_call=r["iterations"], lm_iterations=its,
                   bytes_per_iteration=int(total / its),
                   per_kernel_bytes_per_iteration={k: int(v / its) for k, v in per_kernel.items()}),
              sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
