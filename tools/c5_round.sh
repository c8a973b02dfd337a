#!/bin/bash
# GPU box: config-5 camera solve -- the BA parity tests, then tools/c5_probe.py under rocprofv3
# (per-kernel split) with the default solver and with RSVIO_K5=pipe4 (the VALU two-rows-per-lane
# solver past 10 free keyframes), then one SQ counter pass of the default for VALU_MFMA_BUSY_CYCLES.
# usage: tools/c5_round.sh TAG [tests|notests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 180 --timeout-method thread \
    > gpurun_out/c5_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/c5_tests_$TAG.log; exit 1; }
  tail -2 gpurun_out/c5_tests_$TAG.log
fi
for V in default pipe4; do
  if [ $V = default ]; then E=""; else E="RSVIO_K5=$V"; fi
  env $E timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_${TAG}_$V -o run --output-format csv -- \
    python3 tools/c5_probe.py 30 > gpurun_out/c5_${TAG}_$V.txt 2> gpurun_out/c5_${TAG}_$V.err || { tail -20 gpurun_out/c5_${TAG}_$V.err; exit 1; }
  echo "== $V: $(cat gpurun_out/c5_${TAG}_$V.txt)"
  python3 tools/kstats.py gpurun_out/c5prof_${TAG}_$V | head -8
  rm -f gpurun_out/c5prof_${TAG}_$V/run_kernel_trace.csv
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d gpurun_out/c5pmc_$TAG -o run --output-format csv -- \
  python3 tools/c5_probe.py 10 > gpurun_out/c5pmc_$TAG.txt 2> gpurun_out/c5pmc_$TAG.err || { tail -20 gpurun_out/c5pmc_$TAG.err; exit 1; }
python3 - gpurun_out/c5pmc_$TAG <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for row in csv.DictReader(open(f[0])):
    k = row["Kernel_Name"]
    if "camera_solve" not in k:
        continue
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"]); n[(k, row["Counter_Name"])] += 1
for k, d in acc.items():
    print(k[:60], {c: round(v / max(n[(k, c)], 1), 1) for c, v in d.items()})
PY
