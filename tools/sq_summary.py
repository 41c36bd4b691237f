"""Per-kernel SQ counter summary from tools/pmc_kernel.sh output (two --pmc passes).

Per dispatch averages, then per wave and issue fractions:
  VALU issue fraction = SQ_INSTS_VALU * 2 cycles (wave64 on a 32-wide CDNA4 SIMD) /
                        (1024 SIMDs * GRBM_GUI_ACTIVE / 8)   [GRBM sums the 8 XCDs]
  SALU issue fraction = SQ_INSTS_SALU * 1 cycle / (256 CUs * GRBM_GUI_ACTIVE / 8)  [one scalar issue per CU per cycle]
  wait/active        = SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY
Usage: python tools/sq_summary.py gpurun_out/pmc > profiles/<tag>_sq_counters.json
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_prof import short  # noqa: E402


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main(d="gpurun_out/pmc"):
    merged = defaultdict(dict)
    for p in ("p1", "p2"):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if os.path.exists(f):
            for k, cs in load(f).items():
                for c, v in cs.items():
                    merged[k][c] = sum(v) / len(v)
    out = {}
    for k, c in sorted(merged.items()):
        if not k.startswith("k_"):
            continue
        r = dict(per_dispatch={n: round(v) for n, v in c.items()})
        waves = c.get("SQ_WAVES")
        cyc = c.get("GRBM_GUI_ACTIVE")
        if waves:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
                if n in c:
                    r["%s_per_wave" % n] = round(c[n] / waves, 1)
        if cyc:
            xcd_cycles = cyc / 8.0
            if "SQ_INSTS_VALU" in c:
                r["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * 2 / (1024 * xcd_cycles), 4)
            if "SQ_INSTS_SALU" in c:
                r["salu_issue_frac"] = round(c["SQ_INSTS_SALU"] / (256 * xcd_cycles), 4)
        if c.get("SQ_ACTIVE_INST_ANY"):
            r["wait_over_active"] = round(c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_ACTIVE_INST_ANY"], 3)
        out[k] = r
    print(json.dumps(dict(note=__doc__.strip().splitlines()[0], kernels=out), indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
