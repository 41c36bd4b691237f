"""Timeline of the last LocalBA call in a rocprofv3 kernel(+memory-copy) trace of tools/ba_time.py.

Prints every dispatch / copy of the last call (from its k_ba_prep to its k_ba_export) with duration
and the gap before it, then totals: kernel time, copy time, idle gaps, and the call's device span.
usage: python tools/ba_timeline.py <rocprofv3 output dir>
"""
import csv
import glob
import sys


def load(d):
    ev = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
    ev.sort()
    return ev


def main(d):
    ev = load(d)
    starts = [i for i, e in enumerate(ev) if "k_ba_prep" in e[2]]
    ends = [i for i, e in enumerate(ev) if "k_ba_export" in e[2]]
    a = starts[-1]
    while a > 0 and ev[a - 1][2].startswith("COPY") and ev[a][0] - ev[a - 1][1] < 50_000:
        a -= 1
    b = ends[-1]
    while b + 1 < len(ev) and ev[b + 1][2].startswith("COPY"):
        b += 1
    prev = None
    kern = copy = gap = 0.0
    for s, e, n in ev[a:b + 1]:
        g = (s - prev) / 1e3 if prev is not None else 0.0
        dur = (e - s) / 1e3
        print("%-48s %8.2f us  gap %7.2f" % (n.replace("orbx::", "")[:48], dur, g))
        if n.startswith("COPY"):
            copy += dur
        else:
            kern += dur
        gap += max(g, 0.0)
        prev = max(e, prev or e)
    print("kernels %.1f us, copies %.1f us, gaps %.1f us, span %.1f us, dispatches %d"
          % (kern, copy, gap, (ev[b][1] - ev[a][0]) / 1e3, b - a + 1))


if __name__ == "__main__":
    main(sys.argv[1])
