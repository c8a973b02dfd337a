"""Per-step host + device timeline of bench.py's protocol step from a rocprofv3 trace.

  rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run -- \
      python3 bench.py --steps 20 --warmup 5 --reps 2 --no-cpu --no-rows --pipeline-frames 0
  python tools/step_timeline.py DIR

A step is anchored on its ba_build_layout dispatch (one per rsvio_ba_set_problem).  Its host start
T0 is the image upload: the launch of the step's upload_words_kernel (rsvio_upload_async), or else
the hipMemcpyAsync on the launching thread just before set_problem's own window copy.  Every main-thread HIP call and
every device kernel / copy from T0 to the next step's T0 is labelled (name, occurrence in the step);
the medians over the steps whose host call sequence has the most common signature are printed in
microseconds from T0.
"""
import collections
import csv
import glob
import os
import re
import statistics
import sys


def rows(d, suffix):
    import gzip
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True) + \
            glob.glob(os.path.join(d, "**", f"*{suffix}.gz"), recursive=True):
        out += list(csv.DictReader(gzip.open(p, "rt") if p.endswith(".gz") else open(p)))
    return out


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0].replace("rsvio::", "")
    n = re.sub(r"<.*", "", n).replace("void ", "")
    return n.strip()


def main(d):
    kern = rows(d, "kernel_trace.csv")
    api = rows(d, "hip_api_trace.csv")
    cpy = rows(d, "memory_copy_trace.csv")
    corr_api = {r["Correlation_Id"]: r for r in api}
    anchors = sorted((r for r in kern if "ba_build_layout" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    if len(anchors) < 4:
        print("too few protocol steps in the trace")
        return
    tid = corr_api[anchors[0]["Correlation_Id"]]["Thread_Id"]
    main_api = sorted((r for r in api if r["Thread_Id"] == tid), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in main_api]
    # the image upload's launch: an upload_words_kernel dispatch (rsvio_upload_async) if the step
    # has one, else the hipMemcpyAsync before set_problem's own window copy
    up_launch = sorted(int(corr_api[r["Correlation_Id"]]["Start_Timestamp"]) for r in kern
                       if "upload_words_kernel" in r["Kernel_Name"] and r["Correlation_Id"] in corr_api)
    t0s = []
    for a in anchors:
        la = int(corr_api[a["Correlation_Id"]]["Start_Timestamp"])
        ups = [u for u in up_launch if u < la]
        if ups and (not t0s or ups[-1] > t0s[-1]):
            t0s.append(ups[-1])
            continue
        cp = [i for i, r in enumerate(main_api) if int(r["Start_Timestamp"]) < la and r["Function"] == "hipMemcpyAsync"]
        t0s.append(int(main_api[cp[-2]]["Start_Timestamp"]) if len(cp) >= 2 else la)
    dev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern]
    dev += [("copy_" + r.get("Direction", "?"), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in cpy]
    dev.sort(key=lambda e: e[1])
    steps = []
    for i in range(len(t0s) - 1):
        a, b = t0s[i], t0s[i + 1]
        if b - a > 2_000_000:  # a rep boundary (host work between reps), not one step
            continue
        h = []
        for r in main_api:  # (a run of one call -- the event polls -- is one entry: first start, last end)
            if not a <= int(r["Start_Timestamp"]) < b:
                continue
            s0, e0 = int(r["Start_Timestamp"]) - a, int(r["End_Timestamp"]) - a
            if h and h[-1][0] == r["Function"] and r["Function"] in ("hipEventQuery", "hipStreamQuery"):
                h[-1] = (h[-1][0], h[-1][1], e0)
            else:
                h.append((r["Function"], s0, e0))
        dv = [(n, s - a, e - a) for n, s, e in dev if a <= s < b]
        steps.append((tuple(x[0] for x in h), h, dv, b - a))
    sig = collections.Counter(s[0] for s in steps).most_common(1)[0][0]
    sel = [s for s in steps if s[0] == sig]
    print(f"{len(steps)} steps, {len(sel)} with the common host sequence ({len(sig)} HIP calls); "
          f"median step {statistics.median(s[3] for s in sel) / 1000:.1f} us")
    print("host (main thread), us from T0: start  end")
    for j, f in enumerate(sig):
        print(f"  {j:2d} {f:32s} {statistics.median(s[1][j][1] for s in sel) / 1000:8.1f} "
              f"{statistics.median(s[1][j][2] for s in sel) / 1000:8.1f}")
    lab = collections.defaultdict(list)
    for s in sel:
        seen = collections.Counter()
        for n, st, en in s[2]:
            lab[(n, seen[n])].append((st, en))
            seen[n] += 1
    print("device, us from T0: start  end  (label #occurrence, steps seen)")
    for (n, k), v in sorted(lab.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
        if len(v) < len(sel) // 2:
            continue
        print(f"  {n[:40]:40s} #{k:<2d} {statistics.median(x[0] for x in v) / 1000:8.1f} "
              f"{statistics.median(x[1] for x in v) / 1000:8.1f}  ({len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
