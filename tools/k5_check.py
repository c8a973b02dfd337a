"""K5 diagnostic: the camera step dc of one reduced system vs numpy's solve of the same S, b."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

from rsvio import _lib, synthetic as S  # noqa: E402
from rsvio.ba import BundleAdjuster  # noqa: E402

lib = _lib.load()
lib.rsvio_dbg_ba_camera_step.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_void_p]
for n_kf in [int(a) for a in sys.argv[1:]] or [8, 11, 12, 14, 17, 20, 21]:
    prob = S.ba_problem(n_kf=n_kf, n_lm=40 * n_kf, kf_per_lm=min(n_kf, 4), seed=100 + n_kf, init_seed=200 + n_kf)
    ba = BundleAdjuster(max_keyframes=max(n_kf, 2), max_landmarks=prob.n_lm, max_observations=prob.n_obs)
    ba.set_problem_from(prob)
    Sm, b, cost = ba.build_system(1e-4)
    n = Sm.shape[0]
    dc = np.zeros(n)
    for rep in range(3):
        _lib.check(lib.rsvio_dbg_ba_camera_step(ba._h, 1e-4, 2.0, dc.ctypes.data))
        ref = np.linalg.solve(Sm, b)
        err = np.abs(dc - ref).max() / np.abs(ref).max()
        bad = np.nonzero(np.abs(dc - ref) > 1e-9 * np.abs(ref).max())[0]
        print(f"n_kf {n_kf} n {n}: rel err {err:.3e}  bad rows {bad[:12].tolist()}{'...' if len(bad) > 12 else ''} ({len(bad)})",
              flush=True)
    ba.close()
