#!/bin/bash
# GPU box: rocprofv3 kernel trace of the config-4 Estimator (tools/pipeline_profile.py), per-kernel summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-x}
N=${2:-200}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp_$TAG -o run --output-format csv -- python3 tools/pipeline_profile.py $N > gpurun_out/pp_$TAG.txt 2> gpurun_out/pp_$TAG.err || { tail -30 gpurun_out/pp_$TAG.err; exit 1; }
f=$(find gpurun_out/pp_$TAG -name 'run_kernel_stats.csv' | head -1)
python3 tools/kstats.py "$(dirname "$f")" > gpurun_out/pp_${TAG}_kstats.txt
head -40 gpurun_out/pp_${TAG}_kstats.txt
