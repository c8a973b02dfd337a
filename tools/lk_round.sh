#!/bin/bash
# GPU box: tracker/estimator parity tests, LK phase stamps (L=3, L=6), a short headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tracker_gpu.py tests/test_estimator_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/trk_tests.log 2>&1
rc=$?
tail -3 gpurun_out/trk_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/lk_stamps.py 3 > gpurun_out/lks3.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/lk_stamps.py 6 > gpurun_out/lks6.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-rows > gpurun_out/b1.json 2> gpurun_out/b1.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/b1.json'));print(d['value'], d['ms_per_step'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'])"
