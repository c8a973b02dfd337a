#!/bin/bash
# round 6, call 31: the final tree's headline-only kernel summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06zzz_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 \
  > gpurun_out/r06zzz_prof.json 2> gpurun_out/r06zzz_prof.err || { tail -20 gpurun_out/r06zzz_prof.err; exit 1; }
python tools/kstats.py gpurun_out/r06zzz_prof > gpurun_out/r06zzz_headline_kstats.txt; head -18 gpurun_out/r06zzz_headline_kstats.txt
rm -f gpurun_out/r06zzz_prof/run_kernel_trace.csv
