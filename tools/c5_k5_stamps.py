"""Phase stamps of the 6x6-block camera solve at config 5 (W=20: 19 free keyframes, 5,000
landmarks with 8 consecutive keyframes each; stamps build).  Cycles of K5's block 0: start,
combine (the 8 partial systems into LDS), fail check, factorisation (per block step: wave 0's
start of step K, wave 1's end of step K - 1's update, wave 0's release by barrier K), back
substitution, finish.  usage: python tools/c5_k5_stamps.py"""
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
prob = S.ba_problem(n_kf=20, n_lm=5000, kf_per_lm=8, seed=55, init_seed=56)
ba = BundleAdjuster(max_keyframes=20, max_landmarks=5000, max_observations=prob.n_obs)
ba.set_problem_from(prob)
rows = []
for rep in range(8):
    ba.camera_step(1e-4)
    buf = (C.c_ulonglong * 192)()
    lib.rsvio_dbg_ba_stamps(buf, 192)
    rows.append(np.array(buf[:192], dtype=np.int64))
st = np.median(np.stack(rows[3:]), axis=0).astype(np.int64)
t0 = st[0]
nf = int((prob.kf_fixed == 0).sum())
print(f"config 5 K5 (ba_camera_solve_blk<20>, {nf} free keyframes): cycles from entry")
print(f"combine done {st[1] - t0}, fail check {st[2] - t0}, factorisation done {st[3] - t0}, "
      f"back substitution {st[4] - t0}, end {st[5] - t0}")
print("step  w0_start  w0_at_barrier  w0_released  w1_prev_update_done  w7_prev_update_done  step_len")
for k in range(nf):
    a, r, u = st[32 + k] - t0, st[96 + k] - t0, st[64 + k] - t0
    b, u7 = st[128 + k] - t0, st[160 + k] - t0
    nxt = st[32 + k + 1] - t0 if k + 1 < nf else st[3] - t0
    print(f"{k:4d} {a:9d} {b:14d} {r:12d} {u:20d} {u7:20d} {nxt - a:9d}")
