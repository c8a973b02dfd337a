#!/bin/bash
# round 6, call 34: bench.py's rows (no CPU legs), the unproject row now timed by graph replay
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -c "
import sys, json
sys.path[:0] = ['.', 'rs-vio_amd']
import bench
r = bench.measure_rows(0, False)
print(json.dumps({k: {q: v.get(q) for q in ('value', 'unit', 'launch_ms', 'timed_by')} for k, v in r.items() if isinstance(v, dict)}))
" > gpurun_out/r06z9_rows.json 2> gpurun_out/r06z9_rows.err || { tail -20 gpurun_out/r06z9_rows.err; exit 1; }
cat gpurun_out/r06z9_rows.json
