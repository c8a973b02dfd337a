#!/bin/bash
# GPU box: K5's phase stamps (stamps build) on the same basis -- the unsharded single-rank chain
# against the 1-rank P2P-sharded chain at each fold level given, bench.py's BA CU partition.
# usage: tools/k5_sb_stamps.sh TAG [folds...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
export RSVIO_LIB=$PWD/rs-vio_amd/lib/librsvio_gpu_stamps.so PROBE_STAMPS=1 PROBE_CU_SPLIT=0.25
export WORLD_SIZE=1 RANK=0 MASTER_ADDR=127.0.0.1
{
  PROBE_SINGLE=1 MASTER_PORT=$((29600 + RANDOM % 100)) timeout -k 10 120 python3 tools/p2p_probe.py 1 100 || exit 1
  for F in "$@"; do
    PROBE_SINGLE=0 RSVIO_P2P_FOLD=$F MASTER_PORT=$((29600 + RANDOM % 100)) timeout -k 10 120 python3 tools/p2p_probe.py 1 100 || exit 1
  done
} 2>&1 | grep -v Gloo > gpurun_out/k5sb_$TAG.txt
cat gpurun_out/k5sb_$TAG.txt
