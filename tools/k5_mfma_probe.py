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
seq = [("prologue", 0), ("combine", 1), ("fill M", 2), ("panel0 factor", 9), ("panel0 trailing", 13),
       ("panel1 factor", 15), ("panel1 trailing", 19), ("panel2 factor", 30), ("panel2 trailing", 31),
       ("panel3 factor", 7), ("back subst", 3), ("finish", 4), ("poses", 5), ("result", 6)]
prev = st[0]
for name, k in seq:
    print(f"{name:18s} {st[k] - prev:7d} cycles (t = {st[k] - st[0]})")
    prev = st[k]
