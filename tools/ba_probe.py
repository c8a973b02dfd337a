"""Phase-stamp probe for the BA kernels (diagnostic build lib/librsvio_gpu_stamps.so).
Prints shader-clock cycles between STAMP points of block 0 of the last launch."""
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
for rep in range(5):
    ba.set_problem_from(prob)
    r = ba.run()
print("status", r.status, "iters", r.iterations, "solve_ms", r.solve_ms)
buf = (C.c_ulonglong * 64)()
lib.rsvio_dbg_ba_stamps(buf, 64)
st = np.array(buf[:32], dtype=np.int64)
print("camera_solve phases (cycles):", np.diff(st[:7]).tolist(), "total", st[6] - st[0])
print("  register path: factor %d, back substitution %d" % (st[7] - st[2], st[3] - st[7]))
print("  pipe waves: own-phase start", (st[28:32] - st[2]).tolist(), "end", (np.array(buf[24:28], dtype=np.int64) - st[2]).tolist())
print("lm_decide phases (cycles):", np.diff(st[8:11]).tolist())

# multi-block kernels: per-block stamps of the last launch (rows = blocks)
nb = 4096
big = (C.c_ulonglong * (nb * 32))()
lib.rsvio_dbg_ba_stamps(big, nb * 32)
T = np.array(big[:], dtype=np.int64).reshape(nb, 32)


def report(name, cols, labels):
    rows = T[:, cols[0]] > 0
    for c in cols[1:]:
        rows &= T[:, c] > 0
    X = T[rows][:, cols]
    if len(X) == 0:
        print(name, "no stamps")
        return
    t0 = X[:, 0].min()
    print(f"{name}: {len(X)} blocks, span {X[:, -1].max() - t0} cycles, start spread {X[:, 0].max() - t0}")
    for i in range(1, len(cols)):
        d = X[:, i] - X[:, i - 1]
        print(f"   {labels[i - 1]:>22s}: median {int(np.median(d)):7d}  max {int(d.max()):7d}")


report("linearize (initial)", [11, 12, 14], ["obs linearize", "store + partials"])
report("schur_chunks", [16, 17, 18], ["pair products", "lane-ordered chunk sum"])
report("backsub_relinearize", [20, 22, 23, 24, 25, 21],
       ["W^T dc", "dp (first lanes)", "trial linearise", "store linearisation", "partials"])

r = T[1]
print("schur_chunks block 1 (cycles): pairs+block ids loaded %d, decision gathers+sums %d, lm_update %d, "
      "records+products %d, reduce+store %d" % (r[27] - r[26], r[29] - r[27], r[28] - r[29], r[17] - r[16], r[18] - r[17]))
