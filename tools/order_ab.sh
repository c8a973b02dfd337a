#!/bin/bash
# GPU box: protocol step order x CU split sweep of the headline (bench.py --no-rows --no-cpu).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-order}
HEAD="bench.py --steps 20 --warmup 10 --reps 5 --no-cpu --no-rows --pipeline-frames 0"
for cfg in "ba-first 0.25" "split 0.25" "ba-first 0.25" "split 0.25"; do
  set -- $cfg
  f=gpurun_out/head_${TAG}_$1_$2
  timeout -k 10 200 python $HEAD --order $1 --cu-split $2 > $f.json 2> $f.err || { tail -30 $f.err; exit 1; }
  python -c "
import json;d=json.load(open('$f.json'))
print('$1 $2', d['value'], d['value_reps'], 'res', d['value_resident'], 'lk', d['tracker_lk_ms_per_frame'], 'ba', d['ba_ms_per_solve'])"
done
