#!/bin/bash
# GPU box: crate-tracker + tracker parity tests, then the ft_tracker row A/B/A/B against
# lib/librsvio_gpu_ftold.so (the tree with the previous ft_track.hip, through RSVIO_LIB; built by
# hand: hipcc -c of the old ft_track.hip linked with the other build/*.o objects).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ft_gpu.py tests/test_tracker_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/ft_tests.log 2>&1 || { tail -30 gpurun_out/ft_tests.log; exit 1; }
tail -1 gpurun_out/ft_tests.log
for v in new old new old; do
  if [ $v = old ]; then export RSVIO_LIB=$PWD/rs-vio_amd/lib/librsvio_gpu_ftold.so; else unset RSVIO_LIB; fi
  timeout -k 10 200 python -c "
import sys; sys.path[:0]=['.','rs-vio_amd']
import bench
r=bench.measure_ft_row(0, cpu=False)
print('$v', r['value'], r['device_ms_per_frame'])" 2>/dev/null || exit 1
done
