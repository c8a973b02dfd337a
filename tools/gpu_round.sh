#!/bin/bash
# GPU box: parity tests, smoke, 1-GPU bench (all rows), and a HEADLINE-ONLY rocprofv3
# kernel-trace summary (bench.py --no-rows --no-cpu --pipeline-frames 0) so the roofline's LK
# and per-BA-kernel times reproduce from profiles/.  Usage: tools/gpu_round.sh TAG [tests|notests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
  tail -2 gpurun_out/gpu_tests_$TAG.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 > gpurun_out/prof_head_bench_$TAG.json 2> gpurun_out/prof_head_$TAG.err || { tail -30 gpurun_out/prof_head_$TAG.err; exit 1; }
python tools/kstats.py gpurun_out/prof_head_$TAG > gpurun_out/kstats_head_$TAG.txt
find gpurun_out/prof_head_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/headline_kernel_stats_$TAG.csv \;
rm -f gpurun_out/prof_head_$TAG/run_kernel_trace.csv
du -sh gpurun_out
