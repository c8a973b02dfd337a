#!/bin/bash
# round 6, call 7: set_problem alone (fault bursts with and without the early observation copy);
# config-5 K5 after the unrolled back substitution; headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/setprob_faults.py 30000 > gpurun_out/r06g_setprob.txt 2>&1 || { tail gpurun_out/r06g_setprob.txt; exit 1; }
RSVIO_BA_EARLY_COPY=0 timeout -k 10 200 python tools/setprob_faults.py 30000 >> gpurun_out/r06g_setprob.txt 2>&1 || { tail gpurun_out/r06g_setprob.txt; exit 1; }
grep calls gpurun_out/r06g_setprob.txt
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "window_sizes or config5 or past_ten or variants or batched or golden" > gpurun_out/r06g_ba_tests.log 2>&1 || { tail -40 gpurun_out/r06g_ba_tests.log; exit 1; }
tail -1 gpurun_out/r06g_ba_tests.log
timeout -k 10 120 python tools/c5_k5_stamps.py > gpurun_out/r06g_c5_k5_stamps.txt 2>&1 || { cat gpurun_out/r06g_c5_k5_stamps.txt; exit 1; }
head -3 gpurun_out/r06g_c5_k5_stamps.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r06g_c5prof -o run --output-format csv -- \
    python3 tools/c5_probe.py 30 > gpurun_out/r06g_c5.txt 2> gpurun_out/r06g_c5.err || { tail -20 gpurun_out/r06g_c5.err; exit 1; }
cat gpurun_out/r06g_c5.txt
python3 tools/kstats.py gpurun_out/r06g_c5prof | head -9 | tee gpurun_out/r06g_c5_kstats.txt
rm -f gpurun_out/r06g_c5prof/run_kernel_trace.csv
