#!/bin/bash
# round 6, call 10: the protocol step's calls from C++ (lib/librsvio_protocol.so) vs the Python loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for drv in native python; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 --driver $drv \
      > gpurun_out/r06j_${drv}_$rep.json 2> gpurun_out/r06j_${drv}_$rep.err || { tail -20 gpurun_out/r06j_${drv}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06j_${drv}_$rep.json'));print('$drv',d['value'],d['value_reps'],d['ba_ms_per_iter'],d['tracker_lk_ms_per_frame'],d['protocol_minor_faults'])"
  done
done
