"""Host-side overhead probe: wall time of the tracker step and the BA solve vs their device time."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

torch.cuda.set_device(0)
trk = bench.TrackerWorkload(0)
ba = bench.BAWorkload(0, 1, 0)
for _ in range(5):
    ba.start()
    trk.step(False)
    ba.finish(False)
torch.cuda.synchronize()
tt, tb, dev = [], [], []
for _ in range(50):
    t0 = time.perf_counter()
    trk.step(False)
    t1 = time.perf_counter()
    r = ba.ba.run()
    t2 = time.perf_counter()
    ba.start(); trk.step(False); ba.finish(False)
    tt.append(t1 - t0)
    tb.append(t2 - t1)
    dev.append(r.solve_ms)
torch.cuda.synchronize()
print("tracker step host %.1f us; BA run wall %.1f us, device %.1f us" %
      (1e6 * np.median(tt), 1e6 * np.median(tb), 1e3 * np.median(dev)))
t0 = time.perf_counter()
for _ in range(50):
    r = ba.ba.run()
print("BA alone: %.1f us per solve" % (1e6 * (time.perf_counter() - t0) / 50))
t0 = time.perf_counter()
for _ in range(50):
    trk.step(False)
torch.cuda.synchronize()
print("tracker alone: %.1f us per frame" % (1e6 * (time.perf_counter() - t0) / 50))
