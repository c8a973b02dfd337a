#!/bin/bash
# GPU box (one GPU): N-rank same-device rehearsal of the N>1 bench path (N processes sharing cuda:0,
# P2P exchange with N-rank slots) -- the driver's N=2/4/8 runs launch bench.py the same way.
#   tools/nx_rehearsal.sh N TAG [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-8}
TAG=${2:-r06}
shift 2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29547 bench.py --gpus $N --steps 10 --warmup 3 --reps 3 --no-cpu --no-rows --pipeline-frames 0 \
  --same-device "$@" > gpurun_out/n${N}_$TAG.json 2> gpurun_out/n${N}_$TAG.err || { tail -30 gpurun_out/n${N}_$TAG.err; exit 1; }
grep metric gpurun_out/n${N}_$TAG.json
