#!/bin/bash
# GPU box: SQ counters (one --pmc pass per library, kernel trace only) of the headline command
# (bench.py's protocol step only) for the in-tree library and a reference build (RSVIO_LIB): per
# kernel WAVE_CYCLES, WAIT_ANY (parked), BUSY_CYCLES, INSTS_VALU, INSTS_SALU, INSTS_LDS.
# usage: tools/sq_head_ab.sh TAG REF_LIB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; REF=$2
for v in new ref; do
  if [ $v = ref ]; then export RSVIO_LIB=$REF; else unset RSVIO_LIB; fi
  D=gpurun_out/${TAG}_sqh_$v
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --kernel-trace -d $D -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 > $D.txt 2>&1 || { tail -20 $D.txt; exit 1; }
  echo "== $v"
  python3 tools/pmc_kernels.py $D | grep -v rocclr
  find $D -name '*kernel_trace.csv' -delete
done > gpurun_out/${TAG}_sqh_summary.txt
cat gpurun_out/${TAG}_sqh_summary.txt
