#!/bin/bash
# GPU box: parity tests, smoke, 1-GPU bench (all rows), a HEADLINE-ONLY rocprofv3 kernel-trace
# summary (bench.py --no-rows --no-cpu --pipeline-frames 0) so the roofline's LK and per-BA-
# kernel times reproduce from profiles/, two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) of
# that same headline command, and the FETCH_SIZE calibration (tools/fetch_calib.hip).
# Usage: tools/gpu_round.sh TAG [tests|notests] [bench|nobench] [prof|noprof]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
HEAD="bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0"
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
  tail -2 gpurun_out/gpu_tests_$TAG.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
fi
if [ "${3:-bench}" = "bench" ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi
if [ "${4:-prof}" = "prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head_$TAG -o run --output-format csv -- python3 $HEAD > gpurun_out/prof_head_bench_$TAG.json 2> gpurun_out/prof_head_$TAG.err || { tail -30 gpurun_out/prof_head_$TAG.err; exit 1; }
  python tools/kstats.py gpurun_out/prof_head_$TAG > gpurun_out/kstats_head_$TAG.txt
  cp gpurun_out/prof_head_$TAG/run_kernel_stats.csv gpurun_out/headline_kernel_stats_$TAG.csv
  rm -f gpurun_out/prof_head_$TAG/run_kernel_trace.csv
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv -- python3 $HEAD > gpurun_out/pmc_bench_${TAG}_$C.json 2> gpurun_out/pmc_${TAG}_$C.err || { tail -30 gpurun_out/pmc_${TAG}_$C.err; exit 1; }
  done
  python tools/pmc_summary.py gpurun_out/pmc_${TAG} gpurun_out/pmc_traffic_${TAG}.json
  rm -f gpurun_out/pmc_${TAG}_*/run_counter_collection.csv.bak gpurun_out/pmc_${TAG}_*/run_kernel_trace.csv
  if [ -x tools/fetch_calib ]; then
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/calib_$TAG -o run --output-format csv -- ./tools/fetch_calib > gpurun_out/calib_$TAG.out 2> gpurun_out/calib_$TAG.err || { tail -20 gpurun_out/calib_$TAG.err; exit 1; }
    python tools/calib_summary.py gpurun_out/calib_$TAG gpurun_out/calib_$TAG.out gpurun_out/fetch_calib_$TAG.json
  fi
fi
du -sh gpurun_out
