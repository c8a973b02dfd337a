#!/bin/bash
# GPU box: K5 camera-solve A/B (RSVIO_K5 = pipe4 | mfma | gj1) on config-3 solves -- per-kernel
# durations (rocprofv3 kernel trace), the ba_loop solve time, and an SQ counter pass per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-k5ab}
shift
for V in ${@:-pipe4 mfma}; do
  RSVIO_K5=$V timeout -k 10 120 python3 tools/ba_loop.py 200 > gpurun_out/${TAG}_$V.txt 2>&1 || { cat gpurun_out/${TAG}_$V.txt; exit 1; }
  RSVIO_K5=$V timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$V -o run --output-format csv -- python3 tools/ba_loop.py 200 >> gpurun_out/${TAG}_$V.txt 2>&1 || { tail -20 gpurun_out/${TAG}_$V.txt; exit 1; }
  RSVIO_K5=$V timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/${TAG}_sq_$V -o run --output-format csv -- python3 tools/ba_loop.py 50 >> gpurun_out/${TAG}_$V.txt 2>&1 || { tail -20 gpurun_out/${TAG}_$V.txt; exit 1; }
  python3 tools/kstats.py gpurun_out/${TAG}_prof_$V > gpurun_out/${TAG}_kstats_$V.txt 2>&1
  rm -f gpurun_out/${TAG}_prof_$V/run_kernel_trace.csv
  grep -h "camera_solve\|schur_chunks\|backsub" gpurun_out/${TAG}_kstats_$V.txt | head -5
  head -1 gpurun_out/${TAG}_$V.txt
done
