#!/bin/bash
# GPU box: the 1-rank P2P-sharded chain (fold F; PROBE_SINGLE=1: the unsharded chain) under rocprofv3 for each library variant given
# (lib/librsvio_gpu_<name>.so; "-" = the product library), bench.py's BA CU partition; per
# variant the probe's ms/iter and the per-kernel averages.
# usage: tools/lib_ab_sharded.sh TAG FOLD name...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PROBE_CU_SPLIT=0.25 WORLD_SIZE=1 RANK=0 MASTER_ADDR=127.0.0.1 PROBE_SINGLE=${PROBE_SINGLE:-0}
TAG=$1; F=$2; shift 2
for name in "$@"; do
  D=gpurun_out/lab_${TAG}_$name
  if [ "$name" = - ]; then unset RSVIO_LIB; else export RSVIO_LIB=$PWD/rs-vio_amd/lib/librsvio_gpu_$name.so; fi
  echo "== $name"
  MASTER_PORT=$((29600 + RANDOM % 100)) RSVIO_P2P_FOLD=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D -o run \
    --output-format csv -- python3 tools/p2p_probe.py 1 100 > $D.txt 2> $D.err || { tail -20 $D.err; exit 1; }
  grep "ms/iter" $D.txt
  python3 tools/kstats.py $D 2>/dev/null | grep -v "at::native\|elementwise\|rocclr" | head -6
  find $D -name '*kernel_trace.csv' -delete
done 2>&1 | tee gpurun_out/lab_${TAG}.txt
