#!/bin/bash
# round 6, call 15: the staging image by a kernel (ba_stage_in) instead of SDMA -- BA + estimator
# parity tests, then A/B against RSVIO_BA_STAGE=sdma with the native driver's phase times; then one
# run with RSVIO_BA_PROFILE=slow (set_problem calls > 1 ms or > 100 faults, with new mappings)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ba_gpu.py tests/test_estimator_gpu.py \
  > gpurun_out/r06p_tests.log 2>&1 || { tail -30 gpurun_out/r06p_tests.log; exit 1; }
tail -3 gpurun_out/r06p_tests.log
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
show() { python -c "
import json,sys
d=json.load(open(sys.argv[1])); t=json.load(open(sys.argv[3]))
print(sys.argv[2], d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'], d['protocol_minor_faults'], 'phases', t['median_us'])" "$1" "$2" "$3"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 240 $B --trace-steps gpurun_out/r06p_ph_$n.json > gpurun_out/r06p_$n.json 2> gpurun_out/r06p_$n.err || { tail -20 gpurun_out/r06p_$n.err; return 1; }
  show gpurun_out/r06p_$n.json $n gpurun_out/r06p_ph_$n.json
}
for rep in 1 2 3; do
  run kern_$rep RSVIO_X=0 && run sdma_$rep RSVIO_BA_STAGE=sdma || exit 1
done
run slow_1 RSVIO_BA_PROFILE=slow && run slow_2 RSVIO_BA_PROFILE=slow || exit 1
grep -h "rsvio" gpurun_out/r06p_slow_*.err | head -60
