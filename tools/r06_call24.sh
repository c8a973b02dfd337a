#!/bin/bash
# round 6, call 24: K7's state export in 16-B stores -- BA tests, A/B against the 8-B build
# (lib/librsvio_gpu_r06zz.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ba_gpu.py \
  > gpurun_out/r06y_tests.log 2>&1 || { tail -30 gpurun_out/r06y_tests.log; exit 1; }
tail -2 gpurun_out/r06y_tests.log
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
run() {  # name env... -- args
  local n=$1; shift
  local e=()
  while [ "$1" != "--" ]; do e+=("$1"); shift; done; shift
  env "${e[@]}" timeout -k 10 240 $B "$@" --trace-steps gpurun_out/r06y_ph_$n.json > gpurun_out/r06y_$n.json 2> gpurun_out/r06y_$n.err || { tail -20 gpurun_out/r06y_$n.err; return 1; }
  python -c "
import json,sys
d=json.load(open('gpurun_out/r06y_$n.json')); t=json.load(open('gpurun_out/r06y_ph_$n.json'))
print('$n', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'], d['protocol_minor_faults'], 'phases', t['median_us'])"
}
for rep in 1 2 3; do
  run x16_$rep RSVIO_X=0 -- && run x8_$rep RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_r06zz.so -- || exit 1
done
