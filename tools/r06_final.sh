#!/bin/bash
# round 6 validation: the whole GPU suite, then smoke + the default bench + rocprofv3 kernel stats +
# the two PMC passes (tools/gpu_bench.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06z}
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/gpu_tests_$TAG.log
tail -4 gpurun_out/gpu_tests_$TAG.log
[ $rc = 0 ] || exit $rc
bash tools/gpu_bench.sh $TAG 50
