#!/bin/bash
# round 6, call 27: every thread on the GPU's NUMA node (--numa-local 1) vs unplaced, alternating, 3 pairs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 240 $B "$@" --trace-steps gpurun_out/r06z3_ph_$n.json > gpurun_out/r06z3_$n.json 2> gpurun_out/r06z3_$n.err || { tail -20 gpurun_out/r06z3_$n.err; return 1; }
  python -c "
import json,sys
d=json.load(open('gpurun_out/r06z3_$n.json')); t=json.load(open('gpurun_out/r06z3_ph_$n.json'))
print('$n', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['main_thread'], 'phases', t['median_us'])"
}
for rep in 1 2 3; do
  run numa_$rep --numa-local 1 && run free_$rep || exit 1
done
