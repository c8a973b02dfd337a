"""Config-3 BA solves in a loop on the product library (a short program to profile under
rocprofv3 --pmc / --kernel-trace).  usage: python tools/ba_loop.py [solves]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

from rsvio import synthetic as S  # noqa: E402
from rsvio.ba import BundleAdjuster  # noqa: E402

prob = S.ba_problem(n_kf=10, n_lm=2000, kf_per_lm=6, seed=7)
ba = BundleAdjuster(max_keyframes=10, max_landmarks=2000, max_observations=prob.n_obs)
ba.set_problem_from(prob)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for _ in range(n):
    r = ba.run()
print("status", r.status, "iters", r.iterations, "solve_ms", r.solve_ms)
