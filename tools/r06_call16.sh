#!/bin/bash
# round 6, call 16: rsvio_upload_async (the frame's images by a kernel on the tracker stream) --
# its GPU tests, then A/B against --upload sdma with the native driver's phase times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_upload_gpu.py \
  > gpurun_out/r06q_tests.log 2>&1 || { tail -30 gpurun_out/r06q_tests.log; exit 1; }
tail -2 gpurun_out/r06q_tests.log
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
show() { python -c "
import json,sys
d=json.load(open(sys.argv[1])); t=json.load(open(sys.argv[3]))
print(sys.argv[2], d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'], d['protocol_minor_faults'], 'phases', t['median_us'])" "$1" "$2" "$3"; }
run() {  # name args...
  local n=$1; shift
  timeout -k 10 240 $B "$@" --trace-steps gpurun_out/r06q_ph_$n.json > gpurun_out/r06q_$n.json 2> gpurun_out/r06q_$n.err || { tail -20 gpurun_out/r06q_$n.err; return 1; }
  show gpurun_out/r06q_$n.json $n gpurun_out/r06q_ph_$n.json
}
for rep in 1 2 3; do
  run kern_$rep --upload kernel && run sdma_$rep --upload sdma || exit 1
done
run wfirst_1 --order window-first && run wfirst_2 --order window-first || exit 1
