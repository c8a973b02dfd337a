#!/bin/bash
# GPU box: BA + estimator parity tests, then the headline (protocol + resident) with the BA graph in
# descriptor mode (default) and with RSVIO_BA_DESC=0 (by-value kernels captured per window), A/B/A.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-desc}
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_estimator_gpu.py -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/ba_est_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/ba_est_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/ba_est_tests_$TAG.log
HEAD="bench.py --steps 20 --warmup 10 --reps 5 --no-cpu --no-rows --pipeline-frames 0"
timeout -k 10 200 python $HEAD > gpurun_out/head_${TAG}_on1.json 2> gpurun_out/head_${TAG}_on1.err || { tail -30 gpurun_out/head_${TAG}_on1.err; exit 1; }
RSVIO_BA_DESC=0 timeout -k 10 200 python $HEAD > gpurun_out/head_${TAG}_off.json 2> gpurun_out/head_${TAG}_off.err || { tail -30 gpurun_out/head_${TAG}_off.err; exit 1; }
timeout -k 10 200 python $HEAD > gpurun_out/head_${TAG}_on2.json 2> gpurun_out/head_${TAG}_on2.err || { tail -30 gpurun_out/head_${TAG}_on2.err; exit 1; }
for f in on1 off on2; do python -c "
import json,sys;d=json.load(open('gpurun_out/head_${TAG}_$f.json'))
print('$f', d['value'], d['ms_per_step'], d['value_reps'], 'res', d['value_resident'], 'it', d['ba_ms_per_iter'], d['ba_ms_per_iter_resident'])"; done
