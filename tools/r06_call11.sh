#!/bin/bash
# round 6, call 11: the native Estimator (C++ host logic) vs the Python one, bit for bit; the bench
# with its rows (config-4 row on the native Estimator), no CPU legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_estimator_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "native or pipelined" > gpurun_out/r06k_est_tests.log 2>&1 || { tail -40 gpurun_out/r06k_est_tests.log; exit 1; }
tail -3 gpurun_out/r06k_est_tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --batch-streams 0 > gpurun_out/r06k_bench.json 2> gpurun_out/r06k_bench.err || { tail -30 gpurun_out/r06k_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06k_bench.json"))
print(d["value"], d["value_reps"], d["ba_ms_per_iter"], d["driver"])
r = d["rows"]
p = r["pipeline_config4"]
print("config4", p["value"], p["stage_ms_per_frame"], p["host_ms_per_frame"], p["host_logic"])
print("c5", r["ba_config5"].get("ms_per_iter"), "pnp", r["track_motion"].get("kernel_ms"), r["track_motion"].get("value"))
PY
