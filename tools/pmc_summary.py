"""Per-kernel HBM traffic per dispatch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

rocprofv3 reports both counters in KiB per dispatch.  MI355X_MICROARCH.md (HBM section): on
gfx950 FETCH_SIZE counts 64 B per 128-B request of wide coalesced 16-B-per-lane reads (x2 needed
for those); other access widths are uncalibrated.  We report the raw counter bytes and, per
kernel, the x2-corrected fetch for the kernels whose loads are 16 B per lane (pyramid copy, BA
record loads); the LK gathers are 1-byte loads and are reported raw.
usage: python tools/pmc_summary.py gpurun_out/pmc_TAG out.json
"""
import collections
import csv
import json
import sys

base, out = sys.argv[1], sys.argv[2]
res = collections.defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{base}_{c}/run_counter_collection.csv")):
        n = r["Kernel_Name"].replace("rsvio::(anonymous namespace)::", "").split("(")[0]
        vals[n].append(float(r["Counter_Value"]) * 1024.0)
    for n, v in vals.items():
        res[n][c.lower() + "_bytes_per_dispatch"] = sum(v) / len(v)
        res[n]["dispatches"] = len(v)
doc = {"source": base, "unit": "bytes per dispatch (rocprofv3 KiB x 1024, raw counters)", "kernels": res}
json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps(res.get("lk_track_kernel", {})))
