#!/bin/bash
# GPU box: instruction-fetch counters of the BA LM chain (tools/ba_loop.py, config-3 window
# re-solved): pass 1 wave cycles / instruction waits / fetches, pass 2 the I-cache's hits and
# misses; per kernel (tools/pmc_kernels.py).  usage: tools/ifetch_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
P=1
for C in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  D=gpurun_out/${TAG}_if$P
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $D -o run --output-format csv -- python3 tools/ba_loop.py 50 > $D.txt 2>&1 || { tail -20 $D.txt; exit 1; }
  echo "== pass $P: $C"
  python3 tools/pmc_kernels.py $D | grep -v rocclr
  find $D -name '*kernel_trace.csv' -delete
  P=$((P + 1))
done > gpurun_out/${TAG}_ifetch.txt
cat gpurun_out/${TAG}_ifetch.txt
