"""Per-kernel HBM bytes per dispatch from tools/traffic_now.sh output (gfx950 correction as
tools/parse_prof.py: 2*FETCH_SIZE*1024 + WRITE_SIZE*1024)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_prof import pmc  # noqa: E402

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tn"
f = pmc(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
w = pmc(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
for k in sorted(set(f) | set(w)):
    print("%-22s %14d" % (k, int(2 * f.get(k, 0) * 1024 + w.get(k, 0) * 1024)))
