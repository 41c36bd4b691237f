"""libm cosf/sinf vs the shared deterministic sincos (oracle sincos_det) -- census for DESIGN.md §4.

The reference rotates the BRIEF pattern with the host libm's float cos/sin
(src/ORBextractor.cc:117); oracle and GPU share sincos_det instead.  This walks
every float angle in [0, 2*pi]: how many give a different cosf / sinf, and for how
many of those the 512 rotated pattern offsets (src/ORBextractor.cc:119-125)
change.  Writes the pattern-changing angles to tests/golden/trig_pattern_angles.npy
(test fixture: tests/test_oracle_kat.py checks each one still differs).

    python tools/trig_census.py        (~1 min, one core)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402


def main():
    hi = float(np.float32(2 * np.pi))
    dc, ds, n = oracle.trig_census(0.0, hi, 1)
    nt, npat, n2, ang = oracle.trig_pattern_census(0.0, hi, 1)
    ang = np.sort(ang)
    np.save(os.path.join(ROOT, "tests", "golden", "trig_pattern_angles.npy"), ang)
    frac = float(np.spacing(ang).astype(np.float64).sum() / (2 * np.pi))
    print(json.dumps(dict(floats=n, cos_mismatch=dc, sin_mismatch=ds, any_mismatch=nt, pattern_changes=npat,
                          pattern_change_measure=frac)))


if __name__ == "__main__":
    main()
