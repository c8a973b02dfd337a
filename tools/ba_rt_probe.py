"""Wall-clock timeline of one BA LM iteration (diagnostic build lib/librsvio_gpu_stamps.so).

RTSTAMP slots (s_memrealtime, 100 MHz, the same clock on every CU) of the last launch of each
kernel: K4c ba_schur_chunks 0 entry / 1 inputs loaded / 2 chunk partial stored / 3 block-sum
written (last arriver); K5 4 entry / 5 exit; K6 6 entry / 7 inputs loaded / 8 partials stored /
9 exit (decision taken by the last wave).  Prints each phase's spread over blocks in us relative
to the first K4c entry of the last iteration."""
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
n_kf = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n_lm = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
prob = S.ba_problem(n_kf=n_kf, n_lm=n_lm, kf_per_lm=min(6, n_kf), seed=7)
ba = BundleAdjuster(max_keyframes=n_kf, max_landmarks=n_lm, max_observations=prob.n_obs)
for rep in range(5):
    ba.set_problem_from(prob)
    r = ba.run()
print("status", r.status, "iters", r.iterations, "solve_ms", r.solve_ms)
nb = 4096
buf = (C.c_ulonglong * (nb * 16))()
lib.rsvio_dbg_ba_rt(buf, nb * 16)
T = np.array(buf[:], dtype=np.int64).reshape(nb, 16).astype(np.float64) * 0.01  # us
k4 = T[:, 0] > 0
t0 = T[k4, 0].max() - 30.0  # the last launch: entries within 30 us of the newest
rows4 = k4 & (T[:, 0] >= t0)
base = T[rows4, 0].min()


def spread(name, col, rows):
    v = T[rows, col]
    v = v[v >= base - 1.0]
    if len(v) == 0:
        print(f"  {name:34s} -")
        return
    print(f"  {name:34s} n={len(v):4d}  first {v.min() - base:7.2f}  median {np.median(v) - base:7.2f}  last {v.max() - base:7.2f}")


print("K4c ba_schur_chunks")
spread("entry", 0, rows4)
spread("inputs loaded", 1, rows4)
spread("chunk partial stored", 2, rows4)
spread("block sum written (last arriver)", 3, rows4)
print("K5 ba_camera_solve")
spread("entry", 4, np.arange(nb) == 0)
spread("exit", 5, np.arange(nb) == 0)
print("K6 ba_backsub_relinearize")
k6 = T[:, 6] >= base
spread("entry", 6, k6)
spread("inputs loaded", 7, k6)
spread("partials stored", 8, k6)
spread("exit", 9, k6)
