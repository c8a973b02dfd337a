#!/bin/bash
# GPU box: the sharded-BA round-5 checks -- P2P / sharding tests, then the same-basis A/B
# (tools/same_basis.sh) for the round-start library (base), fold 1 and fold 3 of this tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05j}
timeout -k 10 900 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu -k "sharded or p2p or attach" --timeout 240 \
  --timeout-method thread > gpurun_out/shard_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/shard_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/shard_tests_$TAG.log
RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_base.so bash tools/same_basis.sh ${TAG}_base 1 || exit 1
bash tools/same_basis.sh ${TAG}_f1 1 || exit 1
bash tools/same_basis.sh ${TAG}_f3 3 || exit 1
