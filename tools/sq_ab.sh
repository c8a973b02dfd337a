#!/bin/bash
# GPU box: SQ counters (one --pmc pass each, kernel trace only) of the BA LM chain (tools/ba_loop.py,
# the config-3 window re-solved) for the in-tree library and a reference build (RSVIO_LIB), per
# kernel: WAVE_CYCLES, WAIT_ANY (parked), BUSY_CYCLES, INSTS_VALU, INSTS_LDS, VALU_MFMA_BUSY_CYCLES.
# usage: tools/sq_ab.sh TAG REF_LIB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; REF=$2
for v in new ref; do
  if [ $v = ref ]; then export RSVIO_LIB=$REF; else unset RSVIO_LIB; fi
  D=gpurun_out/${TAG}_sq_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
    --kernel-trace -d $D -o run --output-format csv -- python3 tools/ba_loop.py 50 > $D.txt 2>&1 || { tail -20 $D.txt; exit 1; }
  echo "== $v"
  python3 tools/pmc_kernels.py $D | grep -v rocclr
  find $D -name '*kernel_trace.csv' -delete
done > gpurun_out/${TAG}_sq_summary.txt
cat gpurun_out/${TAG}_sq_summary.txt
