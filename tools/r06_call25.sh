#!/bin/bash
# round 6, call 25: the main thread pinned to the CPU it starts on (--pin-cpu current) vs not,
# alternating, 3 pairs (host-side phase variance between runs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 240 $B "$@" --trace-steps gpurun_out/r06z2_ph_$n.json > gpurun_out/r06z2_$n.json 2> gpurun_out/r06z2_$n.err || { tail -20 gpurun_out/r06z2_$n.err; return 1; }
  python -c "
import json,sys
d=json.load(open('gpurun_out/r06z2_$n.json')); t=json.load(open('gpurun_out/r06z2_ph_$n.json'))
print('$n', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['main_thread'], 'phases', t['median_us'])"
}
for rep in 1 2 3; do
  run pin_$rep --pin-cpu current && run free_$rep || exit 1
done
