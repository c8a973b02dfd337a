"""Summarise a rocprofv3 kernel_stats.csv (and the BA kernel sequence of the last solve)."""
import csv
import re
import sys

d = sys.argv[1]
for r in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
    n = re.sub(r"\(anonymous namespace\)::", "", r["Name"]).split("(")[0].replace("rsvio::", "")
    print(f"{n:36s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1000:8.2f} us  total "
          f"{float(r['TotalDurationNs']) / 1e3:9.1f} us")
rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "ba_reset" in r["Kernel_Name"]]
if len(idx) >= 2:
    seq = [r for r in rows[idx[-2]:idx[-1]] if r["Queue_Id"] == rows[idx[-2]]["Queue_Id"]]
    t0 = int(seq[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seq)
    print(f"last full solve: {len(seq)} dispatches, {(t1 - t0) / 1000:.1f} us first start -> last end")
