#!/bin/bash
# round 6, call 6: the one-rep stall (a ~16 MB burst of the main thread's minor faults inside
# set_problem's first hipMemcpyAsync): a long traced run for its period, kernargs in host memory
# (HIP_FORCE_DEV_KERNARG=0) and a 64 MB kernarg pool; then the same-device rehearsal at 4, 5, 6
# ranks (where does the process time-slicing seen at 7 and 8 start?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --reps 20 --no-cpu --no-rows --pipeline-frames 0 \
    --trace-steps gpurun_out/r06f_trace_$tag.json > gpurun_out/r06f_bench_$tag.json 2> gpurun_out/r06f_bench_$tag.err || { tail -30 gpurun_out/r06f_bench_$tag.err; return 1; }
  python - gpurun_out/r06f_trace_$tag.json gpurun_out/r06f_bench_$tag.json $tag <<'PY'
import json, sys
t = json.load(open(sys.argv[1])); b = json.load(open(sys.argv[2]))
f = t["minor_faults_process_thread"]
print(sys.argv[3], b["value"], "reps min/max", b["value_reps_min"], b["value_reps_max"],
      "fault steps", [(i, x) for i, x in enumerate(f) if x[0] > 50])
PY
}
run default || exit 1
run hostkernarg HIP_FORCE_DEV_KERNARG=0 || exit 1
run pool64m HSA_KERNARG_POOL_SIZE=67108864 || exit 1
for N in 4 5 6; do tools/nx_rehearsal.sh $N r06f | python -c "import json,sys;d=json.loads(sys.stdin.read());print($N, d['value'], d['ba_ms_per_iter'], d['ba_exchange'])" || exit 1; done
