#!/bin/bash
# GPU box: verdict r04 item 1's same-basis A/B -- the unsharded single-rank LM chain against the
# 1-rank P2P-sharded chain, both on bench.py's BA CU partition (PROBE_CU_SPLIT=0.25: 192 CUs), each
# under rocprofv3 (rank process profiled directly); per-kernel summaries + ms/iter.
# usage: tools/same_basis.sh TAG [fold]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; F=${2:-1}
export PROBE_CU_SPLIT=0.25 WORLD_SIZE=1 RANK=0 MASTER_ADDR=127.0.0.1
for mode in single sharded; do
  D=gpurun_out/sb_${TAG}_$mode
  if [ $mode = single ]; then export PROBE_SINGLE=1; else export PROBE_SINGLE=0; fi
  MASTER_PORT=$((29600 + RANDOM % 100)) RSVIO_P2P_FOLD=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D -o run \
    --output-format csv -- python3 tools/p2p_probe.py 1 100 > $D.txt 2> $D.err || { tail -20 $D.err; exit 1; }
  cat $D.txt
  python3 tools/kstats.py $D 2>/dev/null | grep -v "at::native\|elementwise\|rocclr" | head -10
  find $D -name '*kernel_trace.csv' -delete
done > gpurun_out/sb_${TAG}_summary.txt
cat gpurun_out/sb_${TAG}_summary.txt
