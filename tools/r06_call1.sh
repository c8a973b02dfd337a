#!/bin/bash
# round 6, first call: the 8-rank parity tests + fold-3 capacity guard, traced benches (graphs
# captured on first use vs before the timed region), the 8-rank same-device rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "eight_ranks or (fold_equals and 3-8) or fold3_refused" > gpurun_out/r06a_tests8.log 2>&1 || { tail -40 gpurun_out/r06a_tests8.log; exit 1; }
tail -5 gpurun_out/r06a_tests8.log
for i in 0 1 2; do
  pc=1; [ $i = 0 ] && pc=0
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 --precapture-graphs $pc \
    --trace-steps gpurun_out/r06a_trace$i.json > gpurun_out/r06a_bench$i.json 2> gpurun_out/r06a_bench$i.err || { tail -30 gpurun_out/r06a_bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06a_bench$i.json'));print($pc, d['value'],d['value_reps'])"
done
tools/nx_rehearsal.sh 8 r06a
