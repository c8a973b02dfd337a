#!/bin/bash
# GPU box: tracker + estimator parity tests, then an A/B/A of the LK kernel: the current library
# vs lib/librsvio_gpu_lkold.so (the same tree with the previous lk_track.hip, RSVIO_LIB): LK launch
# time over a CU sweep and the config-4 Estimator row (tracker stage).  Build the old library first
# (here): hipcc -c of the previous lk_track.hip, linked with the other build/*.o objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-lk}
timeout -k 10 400 python -u -m pytest tests/test_tracker_gpu.py tests/test_estimator_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/trk_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/trk_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/trk_tests_$TAG.log
for v in new old new old; do
  if [ $v = old ]; then export RSVIO_LIB=$PWD/rs-vio_amd/lib/librsvio_gpu_lkold.so; else unset RSVIO_LIB; fi
  echo "== $v"
  timeout -k 10 200 python tools/lk_cu_sweep.py 40 2>/dev/null | grep CUs || exit 1
  timeout -k 10 300 python tools/pipeline_row.py 500 2 2>/dev/null | tail -1 || exit 1
done
