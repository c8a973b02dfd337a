#!/bin/bash
# GPU box (one GPU): 4-rank same-device rehearsal of the N>1 bench path (4 processes sharing cuda:0,
# P2P exchange with 4-rank slots) -- the driver's N=4/8 runs launch bench.py the same way.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r04}
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 4 --steps 10 --warmup 3 --reps 3 --no-cpu --no-rows --pipeline-frames 0 \
  --same-device > gpurun_out/n4_$TAG.json 2> gpurun_out/n4_$TAG.err || { tail -30 gpurun_out/n4_$TAG.err; exit 1; }
grep metric gpurun_out/n4_$TAG.json
