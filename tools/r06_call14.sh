#!/bin/bash
# round 6, call 14: the native driver's host phase times (--trace-steps) under runtime settings:
# base; the observation pass on one thread; H2D copies as blit kernels below 1 MB (no SDMA engine
# hand-off before ba_build_layout / the pyramids); graph kernel-node batch sizes 1 and 64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --reps 3 --no-cpu --no-rows --pipeline-frames 0"
show() { python -c "
import json,sys
d=json.load(open(sys.argv[1])); t=json.load(open(sys.argv[3]))
print(sys.argv[2], d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'], 'phases', t['median_us'])" "$1" "$2" "$3"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 240 $B --trace-steps gpurun_out/r06o_ph_$n.json > gpurun_out/r06o_$n.json 2> gpurun_out/r06o_$n.err || { tail -20 gpurun_out/r06o_$n.err; return 1; }
  show gpurun_out/r06o_$n.json $n gpurun_out/r06o_ph_$n.json
}
for rep in 1 2; do
  run base_$rep RSVIO_X=0 && run thr0_$rep RSVIO_BA_HOST_THREADS=0 && run blit_$rep GPU_FORCE_BLIT_COPY_SIZE=1024 \
    && run gb1_$rep DEBUG_HIP_GRAPH_BATCH_SIZE=1 && run gb64_$rep DEBUG_HIP_GRAPH_BATCH_SIZE=64 || exit 1
done
