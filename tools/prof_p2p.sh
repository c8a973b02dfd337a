#!/bin/bash
# GPU box: rocprofv3 kernel traces of tools/p2p_probe.py (sharded BA alone, R ranks on cuda:0) at
# each exchange fold level.  Each rank is its own process started from this shell (RANK /
# WORLD_SIZE / MASTER_PORT), and only rank 0 runs under rocprofv3 with the rank itself after
# `--` (no launcher or spawner is ever profiled).  usage: tools/prof_p2p.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
# CFGS: "ranks:fold" pairs (default: the single-rank fold-2 reference, then 2 ranks at each level);
# LL=1 in the environment: K5's system exchange flag-in-word (RSVIO_P2P_LL)
CFGS=${CFGS:-"1:2 2:2 2:1 2:0"}
PORT=${PORT:-29571}
for cfg in $CFGS; do
  cfg=${cfg/:/ }
  set -- $cfg
  R=$1; F=$2
  D=gpurun_out/p2pprof_${TAG}_r${R}_f${F}_ll${LL:-0}
  export RSVIO_P2P_LL=${LL:-0} RSVIO_P2P_FOLD=$F RSVIO_P2P_FOLD_SHARED=1 WORLD_SIZE=$R MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT
  PIDS=""
  for r in $(seq 1 $((R - 1))); do
    RANK=$r timeout -k 10 240 python3 tools/p2p_probe.py $R 50 > $D.r$r.txt 2>&1 &
    PIDS="$PIDS $!"
  done
  RANK=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- \
    python3 tools/p2p_probe.py $R 50 > $D.txt 2> $D.err || { tail -20 $D.err; exit 1; }
  for p in $PIDS; do wait $p || { echo "rank process $p failed"; exit 1; }; done
  cat $D.txt $D.r*.txt 2>/dev/null
  for f in $(find $D -name 'run_kernel_stats.csv'); do
    echo "== $D ($(dirname $f))"
    python3 tools/kstats.py "$(dirname $f)" 2>/dev/null | grep -v "at::native\|elementwise\|rocclr" | head -12
  done
  find $D -name '*kernel_trace.csv' -delete
  PORT=$((PORT + 1))
done > gpurun_out/p2pprof_${TAG}_summary.txt
cat gpurun_out/p2pprof_${TAG}_summary.txt
