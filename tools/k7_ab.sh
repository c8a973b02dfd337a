#!/bin/bash
# GPU box: K7 state-export block count A/B (lib/librsvio_gpu_k7_48.so = the tree built with
# -DRSVIO_K7_BLOCKS=48, through RSVIO_LIB) on the headline protocol step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/rs-vio_amd/lib/librsvio_gpu_k7_48.so
RSVIO_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -q -m gpu -k "export or ticket or descriptor or async" --timeout 180 --timeout-method thread > gpurun_out/k7_tests.log 2>&1 || { tail -30 gpurun_out/k7_tests.log; exit 1; }
tail -1 gpurun_out/k7_tests.log
HEAD="bench.py --steps 20 --warmup 10 --reps 5 --no-cpu --no-rows --pipeline-frames 0"
for v in 16 48 16 48; do
  if [ $v = 48 ]; then export RSVIO_LIB=$V; else unset RSVIO_LIB; fi
  timeout -k 10 200 python $HEAD > gpurun_out/k7_$v.json 2>/dev/null || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/k7_$v.json'))
print('k7 blocks $v', d['value'], d['value_reps'], 'solve', d['ba_ms_per_solve'])"
done
