#!/bin/bash
# GPU box: rocprofv3 kernel trace of the BA probe workload (diagnostic)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || { tail -30 gpurun_out/prof_$TAG.err; exit 1; }
