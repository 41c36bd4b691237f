"""Average duration per (kernel, grid) from a rocprofv3 kernel trace (csv): per-level launches of
k_resize / k_resize_blur show up as separate grids.  usage: python tools/kgrid_stats.py DIR [substr ...]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
keys = sys.argv[2:] or ["k_resize", "k_blur"]
acc = collections.defaultdict(list)
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if any(k in n for k in keys):
            g = (r.get("Grid_Size_X") or r.get("Grid_Size", "?"), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))
            acc[(n.split("(")[0].replace("orbx::", ""), g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = 0.0
for (n, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    m = sum(v) / len(v) / 1e3
    print("%-20s grid %-22s n %4d  avg %8.1f us" % (n, "x".join(g), len(v), m))
