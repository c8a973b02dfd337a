"""Phase stamps of the 6x6-block camera solve (stamps build): cycles of K5's block 0 at config 3
(tools/k5_round.sh runs it on the GPU box).  Slots: 8+K wave 0 at step K's start, 17+K wave 0
released by barrier K, 26..29 wave 1 done with steps 0..3, 30 / 31 wave 0's part A of steps 0 / 4
done; 0/1/2 start / combine / fail check, 3 back substitution, 4..6 finish."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
os.environ["RSVIO_LIB"] = str(ROOT / "rs-vio_amd" / "lib" / "librsvio_gpu_stamps.so")
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

from rsvio import _lib  # noqa: E402
from rsvio import synthetic as S  # noqa: E402
from rsvio.ba import BundleAdjuster  # noqa: E402

lib = _lib.load()
prob = S.ba_problem(n_kf=10, n_lm=2000, kf_per_lm=6, seed=7)
ba = BundleAdjuster(max_keyframes=10, max_landmarks=2000, max_observations=prob.n_obs)
ba.set_problem_from(prob)
rows = []
for rep in range(8):
    ba.camera_step(1e-4)
    buf = (C.c_ulonglong * 32)()
    lib.rsvio_dbg_ba_stamps(buf, 32)
    rows.append(np.array(buf[:32], dtype=np.int64))
st = np.median(np.stack(rows[3:]), axis=0).astype(np.int64)
t0 = st[0]
names = {0: "start", 1: "combine", 2: "fail check"}
names.update({8 + k: f"w0 step {k} start" for k in range(9)})
names.update({17 + k: f"w0 barrier {k} out" for k in range(8)})
names.update({26 + k: f"w1 step {k} update done" for k in range(4)})
names.update({30: "w0 part A step 0 done", 31: "w0 part A step 4 done", 3: "back substitution", 4: "finish sums",
              5: "trial poses", 6: "result"})
ev = sorted((int(st[k]) - t0, k) for k in names if st[k] > 0)
for t, k in ev:
    print(f"{names[k]:26s} t = {t:7d}")
