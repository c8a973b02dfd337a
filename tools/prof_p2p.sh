#!/bin/bash
# GPU box: rocprofv3 kernel traces of tools/p2p_probe.py (sharded BA alone, 2 ranks on cuda:0) at
# each exchange fold level, plus the single-rank reference (1 rank).  usage: tools/prof_p2p.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
# CFGS: "ranks:fold" pairs (default: the single-rank fold-2 reference, then 2 ranks at each level);
# LL=1 in the environment: K5's system exchange flag-in-word (RSVIO_P2P_LL)
CFGS=${CFGS:-"1:2 2:2 2:1 2:0"}
for cfg in $CFGS; do
  cfg=${cfg/:/ }
  set -- $cfg
  R=$1; F=$2
  D=gpurun_out/p2pprof_${TAG}_r${R}_f${F}_ll${LL:-0}
  RSVIO_P2P_LL=${LL:-0} RSVIO_P2P_FOLD=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- \
    python3 tools/p2p_probe.py $R 50 > $D.txt 2> $D.err || { tail -20 $D.err; exit 1; }
  cat $D.txt
  for f in $(find $D -name 'run_kernel_stats.csv'); do
    echo "== $D ($(dirname $f))"
    python3 tools/kstats.py "$(dirname $f)" 2>/dev/null | grep -v "at::native\|elementwise\|rocclr" | head -12
  done
  find $D -name '*kernel_trace.csv' -delete
done > gpurun_out/p2pprof_${TAG}_summary.txt
cat gpurun_out/p2pprof_${TAG}_summary.txt
