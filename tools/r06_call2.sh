#!/bin/bash
# round 6, call 2: set_problem host phases (RSVIO_BA_PROFILE) around the one-rep stall; the 8-rank
# same-device rehearsal with 2 hardware queues per process (8 x 4 = 32 queues oversubscribe the GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  RSVIO_BA_PROFILE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 \
    --trace-steps gpurun_out/r06b_trace$i.json > gpurun_out/r06b_bench$i.json 2> gpurun_out/r06b_bench$i.err || { tail -30 gpurun_out/r06b_bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06b_bench$i.json'));print(d['value'],d['value_reps'])"
done
GPU_MAX_HW_QUEUES=2 tools/nx_rehearsal.sh 8 r06b_q2
