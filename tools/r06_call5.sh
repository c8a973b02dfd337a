#!/bin/bash
# round 6, call 5: config-5 K5 after batching the pre-summed system's loads; BA parity subset;
# headline (2 plain + 1 traced)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "window_sizes or config5 or past_ten or variants or batched or golden or config3" > gpurun_out/r06e_ba_tests.log 2>&1 || { tail -40 gpurun_out/r06e_ba_tests.log; exit 1; }
tail -2 gpurun_out/r06e_ba_tests.log
timeout -k 10 120 python tools/c5_k5_stamps.py > gpurun_out/r06e_c5_k5_stamps.txt 2>&1 || { cat gpurun_out/r06e_c5_k5_stamps.txt; exit 1; }
head -3 gpurun_out/r06e_c5_k5_stamps.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r06e_c5prof -o run --output-format csv -- \
    python3 tools/c5_probe.py 30 > gpurun_out/r06e_c5.txt 2> gpurun_out/r06e_c5.err || { tail -20 gpurun_out/r06e_c5.err; exit 1; }
cat gpurun_out/r06e_c5.txt
python3 tools/kstats.py gpurun_out/r06e_c5prof | head -9 | tee gpurun_out/r06e_c5_kstats.txt
rm -f gpurun_out/r06e_c5prof/run_kernel_trace.csv
for i in 1 2 3; do
  tr=""; [ $i = 3 ] && tr="--trace-steps gpurun_out/r06e_trace$i.json"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 $tr \
    > gpurun_out/r06e_bench$i.json 2> gpurun_out/r06e_bench$i.err || { tail -30 gpurun_out/r06e_bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06e_bench$i.json'));print(d['value'],d['value_reps'],d['ba_ms_per_iter'],d['ba_ms_per_iter_resident'],d['protocol_minor_faults'])"
done
