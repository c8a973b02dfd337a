#!/bin/bash
# round 6, call 32: the config-4 row with the BA + PnP stream on a CU subset (the tracker's stream on
# all CUs) -- all / 192 / 128 / 64 BA CUs, twice each, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_estimator_gpu.py \
  > gpurun_out/r06z8_tests.log 2>&1 || { tail -30 gpurun_out/r06z8_tests.log; exit 1; }
tail -1 gpurun_out/r06z8_tests.log
for rep in 1 2 3; do
  for k in 0 192; do
    timeout -k 10 240 python tools/pipeline_row.py 500 2 $k 2>/dev/null | tail -1 || exit 1
  done
done
