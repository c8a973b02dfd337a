"""track_motion's device time (rsvio_motion_result.kernel_ms, the launch's own wall clock) on the
bench's B8 frame (600 observations, 2,000-point map), median of 200 calls; RSVIO_LIB picks the
library (A/B).  usage: [RSVIO_LIB=...] python tools/pnp_kernel_ms.py [label]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

from rsvio import synthetic as S  # noqa: E402
from rsvio.motion import MotionTracker  # noqa: E402

m = S.motion_frame(seed=3)
mt = MotionTracker()
mt.set_map(m.map_ids, m.map_pw)
ks = []
for i in range(220):
    r = mt.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.T_W_B_last_kf, m.T_C_B2)
    if i >= 20:
        ks.append(r.kernel_ms)
print(f"{sys.argv[1] if len(sys.argv) > 1 else 'lib'}: status {r.status} it {r.iterations} obs {r.n_observations} "
      f"kernel {1e3 * np.median(ks):.2f} us (min {1e3 * np.min(ks):.2f})")
