"""Host-time breakdown of a keyframe window change: rsvio_ba_set_problem, the solve's start
(graph capture + instantiate + launch, or direct launches with RSVIO_BA_GRAPHS=0), the wait.
  python tools/setprob_probe.py [reps]"""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]


def main(reps=40):
    import rsvio
    from rsvio import synthetic as S
    from rsvio.ba import BundleAdjuster
    rsvio.require_device(0)
    wins = [S.ba_problem(), S.ba_problem(seed=17, init_seed=23)]
    ba = BundleAdjuster(max_keyframes=10, max_landmarks=2000, max_observations=24000)
    t = {"set_problem": [], "start": [], "wait": [], "state": [], "start_same": [], "wait_same": []}
    for k in range(reps + 5):
        t0 = time.perf_counter()
        ba.set_problem_from(wins[k % 2])
        t1 = time.perf_counter()
        ba.run_async()
        t2 = time.perf_counter()
        ba.wait()
        t3 = time.perf_counter()
        ba.state()
        t4 = time.perf_counter()
        ba.run_async()
        t5 = time.perf_counter()
        ba.wait()
        t6 = time.perf_counter()
        if k >= 5:
            for key, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
                t[key].append(1e3 * v)
    t2x = []
    for k in range(20):
        ba.set_problem_from(wins[k % 2])
        t0 = time.perf_counter()
        ba.set_problem_from(wins[(k + 1) % 2])   # no graph to drop, stream settled
        t2x.append(1e3 * (time.perf_counter() - t0))
    print(f"set_problem right after set_problem: {np.median(t2x):.4f} ms", flush=True)
    import ctypes as C
    from rsvio import _lib
    lib = _lib.load()
    p = wins[0]
    arrs = [np.ascontiguousarray(a) for a in (p.pose7, p.kf_fixed, p.p_W, p.obs_lm, p.obs_kf, p.obs_cam, p.obs_uv,
                                              p.T_C_B2)]
    tc = []
    for k in range(20):
        ba.set_problem_from(wins[1])
        t0 = time.perf_counter()
        lib.rsvio_ba_set_problem(ba._h, p.n_kf, arrs[0].ctypes.data, arrs[1].ctypes.data, p.n_lm, arrs[2].ctypes.data,
                                 p.n_obs, arrs[3].ctypes.data, arrs[4].ctypes.data, arrs[5].ctypes.data,
                                 arrs[6].ctypes.data, arrs[7].ctypes.data)
        tc.append(1e3 * (time.perf_counter() - t0))
    print(f"bare C call after set_problem: {np.median(tc):.4f} ms", flush=True)
    print(f"RSVIO_BA_GRAPHS={os.environ.get('RSVIO_BA_GRAPHS', '1')}: " +
          ", ".join(f"{k} {np.median(v):.4f} ms" for k, v in t.items()), flush=True)
    ba.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 40)
