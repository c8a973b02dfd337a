#!/bin/bash
# GPU box: rocprofv3 kernel trace of the crate-variant tracker (tools/ft_probe.py), per-kernel summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ft_$TAG -o run --output-format csv -- python3 tools/ft_probe.py > gpurun_out/ft_$TAG.txt 2> gpurun_out/ft_$TAG.err || { tail -30 gpurun_out/ft_$TAG.err; exit 1; }
f=$(find gpurun_out/ft_$TAG -name 'run_kernel_stats.csv' | head -1)
python3 tools/kstats.py "$(dirname "$f")" > gpurun_out/ft_${TAG}_kstats.txt
cat gpurun_out/ft_$TAG.txt | tail -5
grep -v "at::native" gpurun_out/ft_${TAG}_kstats.txt | head -24
