"""Kernel overlap in a rocprofv3 kernel trace: union of kernel intervals vs their sum over the
headline window (the last N k_blur dispatches = N steps).  Usage: python tools/overlap.py TRACE.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", r.get("Stream_Id", "")))
            for r in rows)
blur = [k for k in ks if "k_blur" in k[2]]
t0 = blur[-12][0] - 1  # window: from the 12th-last step's blur (the timed loop) to the end
win = [k for k in ks if k[0] >= t0 and "orbx" in k[2]]
tot = sum(e - s for s, e, _, _ in win)
union, cur_s, cur_e = 0, None, None
for s, e, _, _ in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
span = max(e for _, e, _, _ in win) - min(s for s, _, _, _ in win)
print("kernels %d  sum %.3f ms  union %.3f ms  span %.3f ms  overlap %.1f %%  idle %.1f %%" %
      (len(win), tot / 1e6, union / 1e6, span / 1e6, 100 * (1 - union / tot), 100 * (1 - union / span)))
q = {}
for s, e, n, qq in win:
    q.setdefault(qq, 0)
    q[qq] += 1
print("queues:", q)
