#!/bin/bash
# GPU box: A/B of the headline step between the in-tree library and a reference build
# (RSVIO_LIB=<path>), alternating A/B/A/B on one box; prints value, ms_per_step, the LK launch and
# the BA LM iteration per run.
# usage: tools/ab_lib.sh TAG REF_LIB [reps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; REF=$2; REPS=${3:-2}
HEAD="bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0"
for rep in $(seq 1 $REPS); do
  for v in new ref; do
    if [ $v = ref ]; then L="RSVIO_LIB=$REF"; else L=""; fi
    env $L timeout -k 10 240 python $HEAD > gpurun_out/ab_${TAG}_${v}_${rep}.json 2> gpurun_out/ab_${TAG}_${v}_${rep}.err || { tail -20 gpurun_out/ab_${TAG}_${v}_${rep}.err; exit 1; }
    python3 - gpurun_out/ab_${TAG}_${v}_${rep}.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value", d["value"], "resident", d.get("value_resident"), "ms/step", d["ms_per_step"],
      "lk_ms", d.get("tracker_lk_ms_per_frame"), "ba_ms_iter", d.get("ba_ms_per_iter"),
      "ba_ms_iter_res", d.get("ba_ms_per_iter_resident"), flush=True)
PY
  done
done
