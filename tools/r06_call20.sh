#!/bin/bash
# round 6, call 20: the layout kernel reads 4 observations per thread from the pinned image (three
# 16-B loads) -- BA + estimator tests, A/B against the full stage-in (lib/librsvio_gpu_r06s.so), the
# headline kernel summary, then three runs with the slow set_problem report (the fault burst)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ba_gpu.py tests/test_estimator_gpu.py \
  > gpurun_out/r06u_tests.log 2>&1 || { tail -30 gpurun_out/r06u_tests.log; exit 1; }
tail -2 gpurun_out/r06u_tests.log
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 240 $B --trace-steps gpurun_out/r06u_ph_$n.json > gpurun_out/r06u_$n.json 2> gpurun_out/r06u_$n.err || { tail -20 gpurun_out/r06u_$n.err; return 1; }
  python -c "
import json,sys
d=json.load(open('gpurun_out/r06u_$n.json')); t=json.load(open('gpurun_out/r06u_ph_$n.json'))
print('$n', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'], d['protocol_minor_faults'], 'phases', t['median_us'])"
}
for rep in 1 2 3; do
  run obs4_$rep RSVIO_X=0 && run stg_$rep RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_r06s.so || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06u_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 \
  > gpurun_out/r06u_prof.json 2> gpurun_out/r06u_prof.err || { tail -20 gpurun_out/r06u_prof.err; exit 1; }
python tools/kstats.py gpurun_out/r06u_prof > gpurun_out/r06u_headline_kstats.txt; head -16 gpurun_out/r06u_headline_kstats.txt
rm -f gpurun_out/r06u_prof/run_kernel_trace.csv
for rep in 1 2 3; do
  run slow_$rep RSVIO_BA_PROFILE=slow || exit 1
done
grep -h "rsvio" gpurun_out/r06u_slow_*.err | grep -v "amdgpu.ids" | head -80
