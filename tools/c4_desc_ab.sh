#!/bin/bash
# GPU box: BA + estimator tests, the config-4 Estimator row with the descriptor mode on / off, and
# the protocol order A/B (ba-first vs split).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-c4}
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_estimator_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/ba_est_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/ba_est_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/ba_est_tests_$TAG.log
timeout -k 10 300 python tools/pipeline_row.py 500 2 > gpurun_out/c4_${TAG}_on.txt 2> gpurun_out/c4_${TAG}_on.err || { tail -20 gpurun_out/c4_${TAG}_on.err; exit 1; }
RSVIO_BA_DESC=0 timeout -k 10 300 python tools/pipeline_row.py 500 2 > gpurun_out/c4_${TAG}_off.txt 2> gpurun_out/c4_${TAG}_off.err || { tail -20 gpurun_out/c4_${TAG}_off.err; exit 1; }
echo on; cat gpurun_out/c4_${TAG}_on.txt; echo off; cat gpurun_out/c4_${TAG}_off.txt
bash tools/order_ab.sh $TAG
