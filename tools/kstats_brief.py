"""Mean duration (us) per kernel from a rocprofv3 --stats kernel_stats.csv: python tools/kstats_brief.py CSV [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
print({r["Name"].split("(")[0].replace("orbx::", "").replace("void ", "")[:24]: round(float(r["AverageNs"]) / 1e3, 2)
       for r in rows[:n]})
