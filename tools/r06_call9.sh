#!/bin/bash
# round 6, call 9: K5 parity (readlane multipliers, the reciprocal pinned early); A/B the pinned
# reciprocal (librsvio_gpu_rcplate.so = the compiler's placement); A/B malloc without trimming
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "variants or window_sizes or config3 or golden or descriptor or sharded_p2p_two or fold_equals" > gpurun_out/r06i_ba_tests.log 2>&1 || { tail -40 gpurun_out/r06i_ba_tests.log; exit 1; }
tail -1 gpurun_out/r06i_ba_tests.log
tools/ab_lib.sh r06i_rcp rs-vio_amd/lib/librsvio_gpu_rcplate.so 3 || exit 1
for rep in 1 2 3 4; do
  for tm in 0 1; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 --tame-malloc $tm \
      > gpurun_out/r06i_tm${tm}_$rep.json 2> gpurun_out/r06i_tm${tm}_$rep.err || { tail -20 gpurun_out/r06i_tm${tm}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06i_tm${tm}_$rep.json'));print('tame',$tm,d['value'],d['value_reps_min'],d['protocol_minor_faults'],d['ba_ms_per_iter'])"
  done
done
