"""Phase-stamp probe for pnp_track_motion_kernel (diagnostic build lib/librsvio_gpu_stamps.so).
Prints shader-clock cycles between the STAMP points of the last launch."""
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
from rsvio.motion import MotionTracker  # noqa: E402

lib = _lib.load()
lib.rsvio_dbg_pnp_stamps.restype = C.c_int
m = S.motion_frame(seed=3)
mt = MotionTracker()
mt.set_map(m.map_ids, m.map_pw)
for _ in range(5):
    r = mt.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.T_W_B_last_kf, m.T_C_B2)
print("status", r.status, "iterations", r.iterations, "obs", r.n_observations)
buf = (C.c_ulonglong * 32)()
lib.rsvio_dbg_pnp_stamps(buf, 32)
st = np.array(buf[:], dtype=np.int64)
t0 = st[0]
print("stage (map ids) + prologue:", st[1] - st[0])
print("join:", st[2] - st[1])
npass = r.iterations + 1
for p in range(npass):
    a, b = st[3 + 2 * p], st[4 + 2 * p]
    nxt = st[3 + 2 * (p + 1)] if p + 1 < npass else st[28]
    print(f"pass {p}: linearise+reduce {b - a}, control {nxt - b}")
print("finish:", st[29] - st[28], " total", st[29] - st[0])
lastb = st[4 + 2 * (npass - 2)]
print("last control: to chol end", st[30] - lastb, " se3_plus", st[31] - st[30], " rest", st[3 + 2 * (npass - 1)] - st[31])
