#!/bin/bash
# GPU box: interleaved A/B/C... of the headline step between variants, each given as NAME=ENV
# where ENV is a comma-separated list of assignments (e.g. RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_base.so
# or RSVIO_BA_EXPORT_NC=1; "-" = the in-tree defaults); prints value, the resident value, the LK
# launch and the BA LM iteration (protocol and resident) per run.
# usage: tools/ab_multi.sh TAG REPS NAME=ENV [NAME=ENV ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; REPS=$2; shift 2
HEAD="bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0"
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    E=""; A=""
    case "$envs" in
      -) ;;
      args:*) A=$(echo "${envs#args:}" | tr ',' ' ') ;;   # bench.py arguments, e.g. args:--order,lookahead
      *) E=$(echo "$envs" | tr ',' ' ') ;;
    esac
    out=gpurun_out/abm_${TAG}_${name}_${rep}
    env $E timeout -k 10 240 python $HEAD $A > $out.json 2> $out.err || { tail -20 $out.err; exit 1; }
    python3 - $out.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>8} value {d['value']:9.1f} resident {d.get('value_resident'):9.1f} "
      f"lk_ms {d.get('tracker_lk_ms_per_frame')} ba_ms_iter {d.get('ba_ms_per_iter')} "
      f"res {d.get('ba_ms_per_iter_resident')} solve {d.get('ba_ms_per_solve')}", flush=True)
PY
  done
done
