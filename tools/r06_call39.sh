#!/bin/bash
# round 6, call 39: the driver's exact default command (python bench.py), twice on this box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-a}
for rep in 1 2; do
  timeout -k 10 600 python bench.py > gpurun_out/r06bv_${TAG}_$rep.json 2> gpurun_out/r06bv_${TAG}_$rep.err || { tail -20 gpurun_out/r06bv_${TAG}_$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r06bv_${TAG}_$rep.json'))
print('$TAG $rep', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'], d['main_thread'], 'config4', d['rows']['pipeline_config4']['value'], 'cpu', d['cpu_baseline']['value'])"
done
