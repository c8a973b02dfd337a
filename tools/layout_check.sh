set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_estimator_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/layout_tests.log 2>&1 || { tail -30 gpurun_out/layout_tests.log; exit 1; }
tail -1 gpurun_out/layout_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_layout -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-rows --pipeline-frames 0 > gpurun_out/prof_layout_bench.json 2> gpurun_out/prof_layout.err || { tail -20 gpurun_out/prof_layout.err; exit 1; }
python tools/kstats.py gpurun_out/prof_layout | grep -E "build_layout|bab_linearize|lk_track"
rm -f gpurun_out/prof_layout/run_kernel_trace.csv
