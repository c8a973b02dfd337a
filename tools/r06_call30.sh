#!/bin/bash
# round 6, call 30: the 6x6-block solver's look-ahead L rows by readlane too -- BA tests, config-5
# A/B: both readlane (default) / diagonal only (librsvio_gpu_bkd.so) / both LDS (librsvio_gpu_bkl.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ba_gpu.py \
  > gpurun_out/r06z6_tests.log 2>&1 || { tail -30 gpurun_out/r06z6_tests.log; exit 1; }
tail -1 gpurun_out/r06z6_tests.log
for rep in 1 2 3; do
  echo -n "both-rl  $rep: "; timeout -k 10 120 python tools/c5_probe.py 40 2>/dev/null | tail -1 || exit 1
  echo -n "diag-rl  $rep: "; RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_bkd.so timeout -k 10 120 python tools/c5_probe.py 40 2>/dev/null | tail -1 || exit 1
  echo -n "both-lds $rep: "; RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_bkl.so timeout -k 10 120 python tools/c5_probe.py 40 2>/dev/null | tail -1 || exit 1
done
timeout -k 10 120 python tools/c5_k5_stamps.py > gpurun_out/r06z6_c5_k5_stamps.txt 2>&1 || { cat gpurun_out/r06z6_c5_k5_stamps.txt; exit 1; }
head -12 gpurun_out/r06z6_c5_k5_stamps.txt
