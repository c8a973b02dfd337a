#!/bin/bash
# GPU box: smoke, 1-GPU bench, rocprofv3 kernel-trace summary of the same command, and two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for roofline.traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
STEPS=${2:-50}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || { tail -30 gpurun_out/prof_$TAG.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-rows --pipeline-frames 0 > gpurun_out/pmc_bench_${TAG}_$C.json 2> gpurun_out/pmc_${TAG}_$C.err || { tail -30 gpurun_out/pmc_${TAG}_$C.err; exit 1; }
done
find gpurun_out/prof_$TAG gpurun_out/pmc_${TAG}_* -name "*.csv" | head -20
python tools/pmc_summary.py gpurun_out/pmc_${TAG} gpurun_out/pmc_traffic_${TAG}.json
python tools/kstats.py gpurun_out/prof_$TAG > gpurun_out/kstats_$TAG.txt
# keep the summaries; the raw per-dispatch traces exceed gpurun's 64 MiB merge limit
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/pmc_${TAG}_*/run_counter_collection.csv gpurun_out/pmc_${TAG}_*/run_kernel_trace.csv
du -sh gpurun_out
