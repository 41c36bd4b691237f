import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# take the last LocalBA call: from the last k_ba_pair_table... simply analyse the last 200 dispatches
rows = rows[-260:]
prev = None
tot_gap = 0; tot_k = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"][:40]
    gap = (s - prev) / 1e3 if prev else 0
    if prev: tot_gap += max(gap, 0)
    tot_k += (e - s) / 1e3
    print("%-40s dur %7.2f us gap %7.2f us" % (name, (e - s) / 1e3, gap))
    prev = e
print("kernel us", tot_k, "gap us", tot_gap)
