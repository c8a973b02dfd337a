#!/bin/bash
# round 6, call 3: the PnP rewrite (hash join, 2 barriers per pass): motion + estimator parity,
# stamps; the stall A/B (windows pageable vs page-locked); 7-rank same-device rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_motion_gpu.py tests/test_estimator_gpu.py -x -v -m gpu --timeout 300 \
  --timeout-method thread > gpurun_out/r06c_tests.log 2>&1 || { tail -40 gpurun_out/r06c_tests.log; exit 1; }
tail -3 gpurun_out/r06c_tests.log
timeout -k 10 120 python tools/pnp_probe.py > gpurun_out/r06c_pnp_stamps.txt 2>&1 || { cat gpurun_out/r06c_pnp_stamps.txt; exit 1; }
cat gpurun_out/r06c_pnp_stamps.txt
for i in 1 2 3 4 5 6; do
  pin=$((i % 2))
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 --pin-windows $pin \
    --trace-steps gpurun_out/r06c_trace$i.json > gpurun_out/r06c_bench$i.json 2> gpurun_out/r06c_bench$i.err || { tail -30 gpurun_out/r06c_bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06c_bench$i.json'));print('pin',$pin,d['value'],d['value_reps'],d['protocol_minor_faults'],d['host_numa_balancing'])"
done
tools/nx_rehearsal.sh 7 r06c
timeout -k 10 120 python tools/c5_k5_stamps.py > gpurun_out/r06c_c5_k5_stamps.txt 2>&1 || { cat gpurun_out/r06c_c5_k5_stamps.txt; exit 1; }
cat gpurun_out/r06c_c5_k5_stamps.txt
