#!/bin/bash
# round 6, call 4: BA parity after the K5 changes (blocked back substitution, banded updates,
# the wide pre-combine past 10 free keyframes); config-5 stamps + kernel summary; PnP A/B; headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_ba_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/r06d_ba_tests.log 2>&1 || { tail -40 gpurun_out/r06d_ba_tests.log; exit 1; }
tail -3 gpurun_out/r06d_ba_tests.log
timeout -k 10 120 python tools/c5_k5_stamps.py > gpurun_out/r06d_c5_k5_stamps.txt 2>&1 || { cat gpurun_out/r06d_c5_k5_stamps.txt; exit 1; }
head -3 gpurun_out/r06d_c5_k5_stamps.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r06d_c5prof -o run --output-format csv -- \
    python3 tools/c5_probe.py 30 > gpurun_out/r06d_c5.txt 2> gpurun_out/r06d_c5.err || { tail -20 gpurun_out/r06d_c5.err; exit 1; }
cat gpurun_out/r06d_c5.txt
python3 tools/kstats.py gpurun_out/r06d_c5prof | head -9 | tee gpurun_out/r06d_c5_kstats.txt
rm -f gpurun_out/r06d_c5prof/run_kernel_trace.csv
RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_base.so timeout -k 10 120 python tools/pnp_kernel_ms.py base_r05 > gpurun_out/r06d_pnp_ab.txt 2>&1 || { cat gpurun_out/r06d_pnp_ab.txt; exit 1; }
timeout -k 10 120 python tools/pnp_kernel_ms.py new >> gpurun_out/r06d_pnp_ab.txt 2>&1 || { cat gpurun_out/r06d_pnp_ab.txt; exit 1; }
RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_base.so timeout -k 10 120 python tools/pnp_kernel_ms.py base_r05 >> gpurun_out/r06d_pnp_ab.txt 2>&1 || { cat gpurun_out/r06d_pnp_ab.txt; exit 1; }
timeout -k 10 120 python tools/pnp_kernel_ms.py new >> gpurun_out/r06d_pnp_ab.txt 2>&1 || { cat gpurun_out/r06d_pnp_ab.txt; exit 1; }
cat gpurun_out/r06d_pnp_ab.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0 \
    --trace-steps gpurun_out/r06d_trace$i.json > gpurun_out/r06d_bench$i.json 2> gpurun_out/r06d_bench$i.err || { tail -30 gpurun_out/r06d_bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06d_bench$i.json'));print(d['value'],d['value_reps'],d['ba_ms_per_iter'],d['ba_ms_per_iter_resident'],d['protocol_minor_faults'])"
done
