#!/bin/bash
# GPU box (one GPU): 2-rank same-device rehearsal of the N>1 bench path (P2P exchange between two
# processes sharing cuda:0) -- the driver's N=2..8 runs launch bench.py the same way.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 \
  --same-device > gpurun_out/n2_$TAG.json 2> gpurun_out/n2_$TAG.err || { tail -30 gpurun_out/n2_$TAG.err; exit 1; }
cat gpurun_out/n2_$TAG.json
