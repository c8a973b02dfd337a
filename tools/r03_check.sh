#!/bin/bash
# GPU box: BA parity tests, the 500-frame config-4 parity comparison, a headline-only bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/ba_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/ba_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/ba_tests_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --reps 5 --no-cpu --no-rows --pipeline-frames 0 > gpurun_out/head_$TAG.json 2> gpurun_out/head_$TAG.err || { tail -30 gpurun_out/head_$TAG.err; exit 1; }
cat gpurun_out/head_$TAG.json
if [ "${2:-parity}" = "parity" ]; then
  timeout -k 10 560 python -u tools/config4_parity.py 500 gpurun_out/c4_parity_$TAG.json > gpurun_out/c4_parity_$TAG.log 2>&1 || { tail -30 gpurun_out/c4_parity_$TAG.log; exit 1; }
  tail -20 gpurun_out/c4_parity_$TAG.log
fi
