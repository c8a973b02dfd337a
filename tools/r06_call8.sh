#!/bin/bash
# round 6, call 8: BA parity after the empty-chunk skip (config 5) and the padding loop; config-5
# probe + stamps; headline A/B: K5's later-column multipliers by readlane (librsvio_gpu_rlq.so);
# A/B: the observation section's early copy on / off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/r06h_ba_tests.log 2>&1 || { tail -40 gpurun_out/r06h_ba_tests.log; exit 1; }
tail -1 gpurun_out/r06h_ba_tests.log
timeout -k 10 120 python tools/c5_k5_stamps.py > gpurun_out/r06h_c5_k5_stamps.txt 2>&1 || { cat gpurun_out/r06h_c5_k5_stamps.txt; exit 1; }
head -3 gpurun_out/r06h_c5_k5_stamps.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r06h_c5prof -o run --output-format csv -- \
    python3 tools/c5_probe.py 30 > gpurun_out/r06h_c5.txt 2> gpurun_out/r06h_c5.err || { tail -20 gpurun_out/r06h_c5.err; exit 1; }
cat gpurun_out/r06h_c5.txt
python3 tools/kstats.py gpurun_out/r06h_c5prof | head -9 | tee gpurun_out/r06h_c5_kstats.txt
rm -f gpurun_out/r06h_c5prof/run_kernel_trace.csv
tools/ab_lib.sh r06h_rlq rs-vio_amd/lib/librsvio_gpu_rlq.so 3 || exit 1
for rep in 1 2; do
  for ec in 1 0; do
    RSVIO_BA_EARLY_COPY=$ec timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 \
      > gpurun_out/r06h_ec${ec}_$rep.json 2> gpurun_out/r06h_ec${ec}_$rep.err || { tail -20 gpurun_out/r06h_ec${ec}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06h_ec${ec}_$rep.json'));print('early_copy',$ec,d['value'],d['value_reps'],d['ba_ms_per_iter'])"
  done
done
