"""Phase stamps of the MFMA camera solve (stamps build, RSVIO_K5=mfma): cycles of block 0."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
os.environ["RSVIO_LIB"] = str(ROOT / "rs-vio_amd" / "lib" / "librsvio_gpu_stamps.so")
os.environ["RSVIO_K5"] = "mfma"
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

from rsvio import _lib  # noqa: E402
from rsvio import synthetic as S  # noqa: E402
from rsvio.ba import BundleAdjuster  # noqa: E402

lib = _lib.load()
prob = S.ba_problem(n_kf=10, n_lm=2000, kf_per_lm=6, seed=7)
ba = BundleAdjuster(max_keyframes=10, max_landmarks=2000, max_observations=prob.n_obs)
ba.set_problem_from(prob)
for rep in range(5):
    r = ba.camera_step(1e-4) if rep < 4 else None
buf = (C.c_ulonglong * 64)()
lib.rsvio_dbg_ba_stamps(buf, 64)
st = np.array(buf[:32], dtype=np.int64)
names = {0: "start", 1: "combine", 2: "fail check", 9: "panel 0 factored", 13: "panel 0 trailing",
         15: "panel 2 factored", 19: "panel 2 trailing", 30: "panel 4 factored", 31: "panel 4 trailing",
         7: "last panel factored", 3: "back substitution", 4: "finish sums", 5: "trial poses", 6: "result"}
ev = sorted((int(st[k]), k) for k in names if st[k] > 0)
prev = ev[0][0]
for t, k in ev:
    print(f"{names[k]:22s} +{t - prev:6d} cycles (t = {t - ev[0][0]})")
    prev = t
