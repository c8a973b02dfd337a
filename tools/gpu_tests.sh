#!/bin/bash
# Run on the GPU box via gpurun: parity tests (one process, bounded time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SEL="${1:-tests}"
timeout -k 10 900 python -u -m pytest $SEL -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
exit $rc
