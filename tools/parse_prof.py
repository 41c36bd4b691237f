"""Summarise tools/profile.sh output into profiles/ (committed evidence).

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-kernel average FETCH_SIZE/WRITE_SIZE per dispatch
  profiles/traffic.json             HBM bytes per launch per kernel, read by bench.py

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE/WRITE_SIZE are in KiB; FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024 and write
bytes = WRITE_SIZE * 1024.  Other access widths are uncalibrated: the values
are upper-bound estimates for byte-granular kernels (noted in DESIGN.md).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    n = n.split("::")[-1]
    return n.split("<")[0] if n.startswith("k_") else n


def pmc(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(prof_dir="gpurun_out/prof", tag="r01", batch="256"):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(prof_dir, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, "%s_kernel_stats.csv" % tag))
    fetch = pmc(os.path.join(prof_dir, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(prof_dir, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    per_launch = {}
    summary = {}
    for k in sorted(set(fetch) | set(write)):
        rb = 2.0 * fetch.get(k, 0.0) * 1024
        wb = write.get(k, 0.0) * 1024
        per_launch[k] = int(rb + wb)
        summary[k] = {"FETCH_SIZE_KiB_avg": fetch.get(k), "WRITE_SIZE_KiB_avg": write.get(k),
                      "read_bytes_corrected": int(rb), "write_bytes": int(wb)}
    for extra in ("localba", "pnp"):
        src = os.path.join(prof_dir, extra, "run_kernel_stats.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(out, "%s_%s_kernel_stats.csv" % (tag, extra)))
    json.dump(summary, open(os.path.join(out, "%s_pmc.json" % tag), "w"), indent=1)
    import subprocess
    head = subprocess.run(["git", "-C", root, "rev-parse", "--short", "HEAD"], capture_output=True,
                          text=True).stdout.strip() or None
    json.dump({"source": "%s_pmc.json" % tag, "head": head, "batch": int(batch), "per_launch_bytes": per_launch,
               "note": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per dispatch, averaged over dispatches"},
              open(os.path.join(out, "traffic.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
