"""Host turnaround of back-to-back config-3 BA solves (run_async + wait, no tracker): wall time
per solve against the solve's own HIP-event time, and the split of the host side."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

from rsvio import synthetic as S  # noqa: E402
from rsvio.ba import BundleAdjuster  # noqa: E402

prob = S.ba_problem(n_kf=10, n_lm=2000, kf_per_lm=6, seed=7)
ba = BundleAdjuster(max_keyframes=10, max_landmarks=2000, max_observations=prob.n_obs)
ba.set_problem_from(prob)
for _ in range(20):
    ba.run()
n = 300
ts, tw, sm = [], [], []
t0 = time.perf_counter()
for _ in range(n):
    a = time.perf_counter()
    ba.run_async()
    b = time.perf_counter()
    r = ba.wait()
    c = time.perf_counter()
    ts.append(b - a)
    tw.append(c - b)
    sm.append(r.solve_ms)
el = time.perf_counter() - t0
print(f"per solve: wall {1e3 * el / n:.4f} ms, event solve_ms {np.mean(sm):.4f}, run_async {1e3 * np.mean(ts):.4f} ms, "
      f"wait {1e3 * np.mean(tw):.4f} ms, iterations {r.iterations}")
