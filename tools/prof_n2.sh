#!/bin/bash
# GPU box (one GPU): rocprofv3 kernel trace of the 2-rank same-device rehearsal of the sharded BA
# (bench.py --same-device, P2P exchange): per-kernel times of the sharded LM iteration (K4c, K5
# with the reduced system's exchange folded in, K6, X2).  Both ranks are bench.py processes started
# from this shell (RANK / WORLD_SIZE / MASTER_*); only rank 0 runs under rocprofv3, with the rank
# itself after `--` (never a launcher).
# usage: tools/prof_n2.sh TAG [extra env, e.g. RSVIO_P2P_FOLD=0]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
shift
for kv in "$@"; do export "$kv"; done
export WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
ARGS="bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 --same-device"
RANK=1 LOCAL_RANK=1 timeout -k 10 300 python3 $ARGS > gpurun_out/n2prof_${TAG}_r1.json 2> gpurun_out/n2prof_${TAG}_r1.err &
P1=$!
RANK=0 LOCAL_RANK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/n2prof_$TAG -o run --output-format csv -- \
  python3 $ARGS > gpurun_out/n2prof_$TAG.json 2> gpurun_out/n2prof_$TAG.err || { tail -30 gpurun_out/n2prof_$TAG.err; exit 1; }
wait $P1 || { tail -30 gpurun_out/n2prof_${TAG}_r1.err; exit 1; }
for f in $(find gpurun_out/n2prof_$TAG -name 'run_kernel_stats.csv'); do
  d=$(dirname "$f")
  echo "== $d"
  python3 tools/kstats.py "$d" | grep -v "at::native\|elementwise" | head -30
done > gpurun_out/n2prof_${TAG}_kstats.txt
cat gpurun_out/n2prof_${TAG}_kstats.txt
find gpurun_out/n2prof_$TAG -name '*kernel_trace.csv' -delete
