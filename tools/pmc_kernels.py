"""Per-kernel average of rocprofv3 --pmc counters (counter_collection.csv) -- diagnostic."""
import collections
import csv
import glob
import re
import sys

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(anonymous namespace\)", "", r["Kernel_Name"]).split("(")[0].split("::")[-1]
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[n].add(r["Dispatch_Id"])
for n, d in sorted(agg.items()):
    k = len(disp[n])
    print(f"{n[:28]:28s} x{k:<4d} " + " ".join(f"{c.replace('SQ_', '')}={v / k:.0f}" for c, v in sorted(d.items())))
