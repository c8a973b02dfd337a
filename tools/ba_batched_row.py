import sys, json
sys.path[:0]=['.', 'rs-vio_amd']
import bench
import rsvio
rsvio.require_device(0)
for B in (16, 64):
    print(json.dumps(bench.measure_ba_batched_row(0, B, reps=5)), flush=True)
