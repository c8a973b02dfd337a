#!/bin/bash
# round 6, call 17: the staging guard without an event per upload -- BA + estimator tests, two
# headline runs with phase times, the headline-only kernel summary, and the traced step timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ba_gpu.py tests/test_estimator_gpu.py \
  > gpurun_out/r06r_tests.log 2>&1 || { tail -30 gpurun_out/r06r_tests.log; exit 1; }
tail -2 gpurun_out/r06r_tests.log
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
for rep in 1 2; do
  timeout -k 10 240 $B --trace-steps gpurun_out/r06r_ph_$rep.json > gpurun_out/r06r_$rep.json 2> gpurun_out/r06r_$rep.err || { tail -20 gpurun_out/r06r_$rep.err; exit 1; }
  python -c "
import json,sys
d=json.load(open('gpurun_out/r06r_$rep.json')); t=json.load(open('gpurun_out/r06r_ph_$rep.json'))
print('run $rep', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'], d['protocol_minor_faults'], 'phases', t['median_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06r_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 \
  > gpurun_out/r06r_prof.json 2> gpurun_out/r06r_prof.err || { tail -20 gpurun_out/r06r_prof.err; exit 1; }
python tools/kstats.py gpurun_out/r06r_prof > gpurun_out/r06r_headline_kstats.txt; head -14 gpurun_out/r06r_headline_kstats.txt
rm -f gpurun_out/r06r_prof/run_kernel_trace.csv
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06r_tl -o run \
  -- python3 bench.py --steps 20 --warmup 5 --reps 2 --no-cpu --no-rows --pipeline-frames 0 > gpurun_out/r06r_tl.json 2> gpurun_out/r06r_tl.err || { tail -20 gpurun_out/r06r_tl.err; exit 1; }
python tools/step_timeline.py gpurun_out/r06r_tl > gpurun_out/r06r_timeline.txt 2>&1; head -50 gpurun_out/r06r_timeline.txt
gzip -f gpurun_out/r06r_tl/*.csv
