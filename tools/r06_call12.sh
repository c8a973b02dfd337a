#!/bin/bash
# round 6, call 12: stall diagnostic -- the runtimes' code pages locked (--lock-code 1) vs not,
# alternating, native driver, malloc tamed (defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ulimit -l 2>&1 | sed 's/^/memlock limit (KB): /'
for rep in 1 2 3 4 5; do
  for lc in 0 1; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 --lock-code $lc \
      > gpurun_out/r06l_lc${lc}_$rep.json 2> gpurun_out/r06l_lc${lc}_$rep.err || { tail -20 gpurun_out/r06l_lc${lc}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06l_lc${lc}_$rep.json'));print('lock',$lc,d['value'],d['value_reps_min'],d['protocol_minor_faults'])"
    grep -h "lock-code" gpurun_out/r06l_lc${lc}_$rep.err || true
  done
done
