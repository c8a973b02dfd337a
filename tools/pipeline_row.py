"""GPU box: only bench.py's config-4 Estimator row (no CPU leg), printed as JSON.
usage: python tools/pipeline_row.py [frames] [repeats] [ba_cus]   (ba_cus: the BA + PnP stream on the
last ba_cus mask bits -- ba_cus / 8 CUs of every XCD; 0 or absent: all CUs, still CU-masked)"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
k = int(sys.argv[3]) if len(sys.argv) > 3 else 0
cus = list(range(256 - k, 256)) if k else None
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 1):
    r = bench.measure_pipeline_row(0, cpu=False, n_frames=n, ba_cus=cus)
    print(json.dumps({"ba_cus": k or 256, **{q: r[q] for q in ("value", "ms_per_frame", "stage_ms_per_frame", "host_ms_per_frame",
                                         "keyframes", "ba_solves", "max_position_error_m")}}), flush=True)
