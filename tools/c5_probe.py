"""Config-5 BA (W=20 x 5,000 landmarks, 80,000 observations) solved repeatedly -- run under
rocprofv3 --kernel-trace --stats for the per-kernel split (diagnostic)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

from rsvio import synthetic as S  # noqa: E402
from rsvio.ba import BundleAdjuster  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
prob = S.ba_problem(n_kf=20, n_lm=5000, kf_per_lm=8, seed=55, init_seed=56)
ba = BundleAdjuster(max_keyframes=20, max_landmarks=5000, max_observations=prob.n_obs)
ba.set_problem_from(prob)
ms, its = [], []
for _ in range(reps):
    r = ba.run()
    ms.append(r.solve_ms)
    its.append(r.iterations)
print(f"config 5: status {r.status} iterations {np.median(its)} solve {np.median(ms):.3f} ms "
      f"-> {np.median(ms) / np.median(its):.4f} ms/iter", flush=True)
ba.close()
