"""set_problem alone, many times (two config-3 windows alternating, no solve): per call the host
time and the calling thread's minor page faults; prints the slowest calls and every call with a
fault burst (diagnostic of the one-rep stall).  usage: python tools/setprob_faults.py [calls]"""
import resource
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

from rsvio import synthetic as S  # noqa: E402
from rsvio.ba import BundleAdjuster  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
wins = [S.ba_problem(n_lm=2000), S.ba_problem(n_lm=2000, seed=17, init_seed=23)]
ba = BundleAdjuster(max_keyframes=10, max_landmarks=2000, max_observations=max(w.n_obs for w in wins))
for i in range(20):
    ba.set_problem_from(wins[i & 1])
us, fl = np.zeros(n), np.zeros(n, np.int64)
for i in range(n):
    f0 = resource.getrusage(1).ru_minflt  # RUSAGE_THREAD
    t0 = time.perf_counter()
    ba.set_problem_from(wins[i & 1])
    us[i] = 1e6 * (time.perf_counter() - t0)
    fl[i] = resource.getrusage(1).ru_minflt - f0
o = np.argsort(us)[::-1][:5]
print(f"{n} calls: median {np.median(us):.1f} us, p99 {np.percentile(us, 99):.1f}, max {us.max():.1f}; "
      f"calls with > 50 faults: {[(int(i), int(fl[i]), round(float(us[i]))) for i in np.nonzero(fl > 50)[0]]}; "
      f"slowest {[(int(i), round(float(us[i])), int(fl[i])) for i in o]}", flush=True)
ba.close()
