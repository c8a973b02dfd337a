#!/bin/bash
# GPU box: SQ counters (one --pmc pass per library, kernel trace only) of the 1-rank P2P-sharded
# chain (tools/p2p_probe.py, bench's BA partition) for the in-tree library (its default fold) and
# a reference build (RSVIO_LIB, e.g. the round's starting library with its default fold 1).
# usage: tools/sq_sharded_ab.sh TAG REF_LIB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PROBE_CU_SPLIT=0.25 WORLD_SIZE=1 RANK=0 MASTER_ADDR=127.0.0.1 PROBE_SINGLE=0
TAG=$1; REF=$2
for v in new ref; do
  if [ $v = ref ]; then export RSVIO_LIB=$REF RSVIO_P2P_FOLD=1; else unset RSVIO_LIB RSVIO_P2P_FOLD; fi
  D=gpurun_out/${TAG}_sqs_$v
  MASTER_PORT=$((29600 + RANDOM % 100)) timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
    --kernel-trace -d $D -o run --output-format csv -- python3 tools/p2p_probe.py 1 50 > $D.txt 2>&1 || { tail -20 $D.txt; exit 1; }
  echo "== $v"
  grep "ms/iter" $D.txt
  python3 tools/pmc_kernels.py $D | grep -v rocclr
  find $D -name '*kernel_trace.csv' -delete
done > gpurun_out/${TAG}_sqs_summary.txt
cat gpurun_out/${TAG}_sqs_summary.txt
