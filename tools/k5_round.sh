#!/bin/bash
# GPU box: K5 factorisation A/B -- BA + estimator parity tests on the in-tree library, then the
# headline step interleaved against a variant library (e.g. the 8-column panel K5), then a
# headline-only rocprofv3 kernel summary of the in-tree library.
# usage: tools/k5_round.sh TAG VARIANT_LIB [reps] [tests|notests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; VAR=$2; REPS=${3:-3}
if [ "${4:-tests}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_estimator_gpu.py tests/test_motion_gpu.py -x -v -m gpu \
    --timeout 180 --timeout-method thread > gpurun_out/k5_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/k5_tests_$TAG.log; exit 1; }
  tail -2 gpurun_out/k5_tests_$TAG.log
fi
bash tools/ab_multi.sh $TAG $REPS new=- old=RSVIO_LIB=$VAR || exit 1
HEAD="bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k5prof_$TAG -o run --output-format csv -- python3 $HEAD \
  > gpurun_out/k5prof_$TAG.json 2> gpurun_out/k5prof_$TAG.err || { tail -30 gpurun_out/k5prof_$TAG.err; exit 1; }
python tools/kstats.py gpurun_out/k5prof_$TAG > gpurun_out/k5_kstats_$TAG.txt
rm -f gpurun_out/k5prof_$TAG/run_kernel_trace.csv
head -20 gpurun_out/k5_kstats_$TAG.txt
if [ -f rs-vio_amd/lib/librsvio_gpu_stamps.so ]; then
  timeout -k 10 120 python3 tools/k5_blk_probe.py > gpurun_out/k5_stamps_$TAG.txt 2>&1 || { tail -20 gpurun_out/k5_stamps_$TAG.txt; exit 1; }
  cat gpurun_out/k5_stamps_$TAG.txt
fi
