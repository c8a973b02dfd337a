#!/bin/bash
# GPU box: parity tests, then the headline with the BA wait on the decision ticket (default)
# against hipStreamSynchronize (RSVIO_BA_WAIT=sync), twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/wait_tests.log 2>&1 || { tail -30 gpurun_out/wait_tests.log; exit 1; }
tail -1 gpurun_out/wait_tests.log
for i in 1 2; do
for v in sync tick; do
RSVIO_BA_WAIT=$v timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 > gpurun_out/wait_$v.json 2>gpurun_out/wait_$v.err || { tail gpurun_out/wait_$v.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/wait_$v.json'));print('$v',d['value'],d['ms_per_step'],d['ba_ms_per_iter'],d['ba_ms_per_solve'],d['value_pcie'])"
done; done
