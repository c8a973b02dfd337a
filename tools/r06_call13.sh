#!/bin/bash
# round 6, call 13: (a) the observation pass over helper threads, A/B (RSVIO_BA_HOST_THREADS 0 / 3);
# (b) set_problem's host phases both ways; (c) the CU split with the native driver (56 vs 64 tracker
# CUs); (e) window-first order vs split; (d) a host + device timeline of the protocol step (rocprofv3 hip + kernel + copy traces)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --no-cpu --no-rows --pipeline-frames 0"
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['value_reps_min'],d['value_reps_max'],d['ba_ms_per_iter'],d['tracker_lk_ms_per_frame'],d.get('protocol_minor_faults'))" "$1" "$2"; }
for rep in 1 2 3; do
  for t in 0 3; do
    RSVIO_BA_HOST_THREADS=$t timeout -k 10 240 $B > gpurun_out/r06n_t${t}_$rep.json 2> gpurun_out/r06n_t${t}_$rep.err || { tail -20 gpurun_out/r06n_t${t}_$rep.err; exit 1; }
    show gpurun_out/r06n_t${t}_$rep.json "threads $t"
  done
done
for t in 0 3; do
  RSVIO_BA_PROFILE=1 RSVIO_BA_HOST_THREADS=$t timeout -k 10 240 $B --reps 2 > gpurun_out/r06n_prof_t$t.json 2> gpurun_out/r06n_prof_t$t.err || { tail -20 gpurun_out/r06n_prof_t$t.err; exit 1; }
done
for rep in 1 2; do
  for cs in 0.25 0.21875; do
    timeout -k 10 240 $B --cu-split $cs > gpurun_out/r06m_cs${cs}_$rep.json 2> gpurun_out/r06m_cs${cs}_$rep.err || { tail -20 gpurun_out/r06m_cs${cs}_$rep.err; exit 1; }
    show gpurun_out/r06m_cs${cs}_$rep.json "split $cs"
  done
done
for rep in 1 2; do
  for o in split window-first; do
    timeout -k 10 240 $B --order $o > gpurun_out/r06n_o${o}_$rep.json 2> gpurun_out/r06n_o${o}_$rep.err || { tail -20 gpurun_out/r06n_o${o}_$rep.err; exit 1; }
    show gpurun_out/r06n_o${o}_$rep.json "order $o"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06n_tl -o run \
  -- python3 bench.py --steps 20 --warmup 5 --reps 2 --no-cpu --no-rows --pipeline-frames 0 > gpurun_out/r06n_tl.json 2> gpurun_out/r06n_tl.err || { tail -20 gpurun_out/r06n_tl.err; exit 1; }
python tools/step_timeline.py gpurun_out/r06n_tl > gpurun_out/r06n_timeline.txt 2>&1; cat gpurun_out/r06n_timeline.txt | head -80
gzip -f gpurun_out/r06n_tl/*.csv
