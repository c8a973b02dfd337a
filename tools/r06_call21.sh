#!/bin/bash
# round 6, call 21: where the PnP kernel's LM control time goes -- phase stamps of the current
# kernel, then instruction-fetch counters (SQ wave/inst-wait/ifetch, SQC I-cache hits/misses)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RSVIO_LIB=rs-vio_amd/lib/librsvio_gpu_stamps.so timeout -k 10 120 python tools/pnp_probe.py > gpurun_out/r06v_pnp_stamps.txt 2>&1 || { tail -20 gpurun_out/r06v_pnp_stamps.txt; exit 1; }
cat gpurun_out/r06v_pnp_stamps.txt
timeout -k 10 120 python tools/pnp_kernel_ms.py cur || exit 1
P=1
for C in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  D=gpurun_out/r06v_if$P
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $D -o run --output-format csv -- python3 tools/pnp_kernel_ms.py pmc > $D.txt 2>&1 || { tail -20 $D.txt; exit 1; }
  echo "== pass $P: $C"
  python3 tools/pmc_kernels.py $D | grep -v rocclr
  find $D -name '*kernel_trace.csv' -delete
  P=$((P + 1))
done > gpurun_out/r06v_pnp_ifetch.txt
cat gpurun_out/r06v_pnp_ifetch.txt
