#!/bin/bash
# round 6, call 36: the native driver's own event timeline (--trace-steps): the window laid out on
# the device and the solve's end, from the step's start on the tracker stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0 \
    --trace-steps gpurun_out/r06z11_ph_$rep.json > gpurun_out/r06z11_$rep.json 2> gpurun_out/r06z11_$rep.err || { tail -20 gpurun_out/r06z11_$rep.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/r06z11_$rep.json')); t=json.load(open('gpurun_out/r06z11_ph_$rep.json'))
print('run $rep', d['value'], d['value_reps_min'], d['value_reps_max'], 'timeline', t['timeline_median_us'], 'phases', t['median_us'])"
done
