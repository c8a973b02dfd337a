# CU-partition sweep of the headline step (bench.py --cu-split/--cu-layout); one line per setting
set -o pipefail
for a in ${CU_SWEEP:-"0 block" "0.25 block" "0.375 block" "0.5 block"}; do
  set -- $a
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-rows --cu-split $1 --cu-layout $2 > gpurun_out/cu_$1_$2.json 2> gpurun_out/cu_$1_$2.err || { tail -5 gpurun_out/cu_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/cu_$1_$2.json'));print('$1 $2', d['value'], d['ms_per_step'], d['ba_ms_per_solve'], d['ba_ms_per_iter'], d['tracker_lk_ms_per_frame'])"
done
