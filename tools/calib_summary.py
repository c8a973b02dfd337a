"""FETCH_SIZE calibration summary (tools/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE).

usage: python tools/calib_summary.py <pmc dir> <fetch_calib stdout> out.json
Per calibration kernel: raw FETCH_SIZE bytes, the expected line bytes (distinct 128-B lines x
128) and the multiplier expected / raw that turns the counter into bytes for that access shape.
"""
import csv
import glob
import json
import re
import sys

pmc_dir, stdout, out = sys.argv[1], sys.argv[2], sys.argv[3]
exp = dict((k, int(v)) for k, v in re.findall(r"(\w+) (\d+)", open(stdout).read().split(":", 1)[1]))
rows = []
for f in glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
fetch = {}
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    key = {"wide16": "wide16", "byte1": "byte1", "u8_gath": "u8_gath"}.get(n)
    if n == "u16_stride":
        key = "u16_l128" if "u16_l128" not in fetch else "u16_l64"
    if key:
        fetch[key] = float(r["Counter_Value"]) * 1024.0
doc = {"source": pmc_dir, "unit": "bytes", "kernels": {}}
for k, v in fetch.items():
    doc["kernels"][k] = {"fetch_size_raw": v, "expected_line_bytes": exp[k], "multiplier": exp[k] / v if v else None}
json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps(doc["kernels"], indent=1))
