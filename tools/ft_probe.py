"""Time the feature_tracker/ crate variant on device-resident 752x480 frames (HIP events on the
tracker's stream) -- run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsvio import ft, synthetic as S  # noqa: E402

W, H = 752, 480
n_frames = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
frames = list(S.mono_sequence(n_frames))
d = torch.from_numpy(np.stack(frames)).cuda()
t = ft.FeatureTracker(W, H)
order = list(range(n_frames)) + list(range(n_frames - 2, 0, -1))
for k in range(10):
    t.process_frame_device(d[order[k % len(order)]].data_ptr())
torch.cuda.synchronize()
st = torch.cuda.ExternalStream(t.stream)
ns = []
t0 = time.perf_counter()
for k in range(steps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    n = t.process_frame_device(d[order[k % len(order)]].data_ptr())
    b.record(st)
    ns.append(n)
    b.synchronize()
    ns[-1] = (n, a.elapsed_time(b))
wall = (time.perf_counter() - t0) / steps
dev = np.median([x[1] for x in ns])
print(f"features/frame {np.mean([x[0] for x in ns]):.0f}  device ms/frame {dev:.3f}  wall ms/frame {wall * 1e3:.3f}"
      f"  -> {1 / wall:.0f} frames/s")
