"""Latency probe for the LK kernel and pyramid: times rsvio_track_points_d / rsvio_build_pyramids_d
for several batch sizes and iteration caps (HIP events on torch's stream).  Diagnostic only."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsvio import _lib  # noqa: E402
from rsvio import synthetic as S  # noqa: E402

W, H, L = 752, 480, 3
lib = _lib.load()
frames = list(S.stereo_sequence(2, W, H))
aff = S.track_features(frames[0][0], 300)
dev = torch.device("cuda", 0)
imgs = torch.from_numpy(np.stack([frames[0][0], frames[1][0]])).to(dev)
pb = int(lib.rsvio_pyramid_bytes(W, H, L))
pyr = torch.empty((2, pb), dtype=torch.uint8, device=dev)
ctx = C.c_void_p()
_lib.check(lib.rsvio_track_ctx_create(W, H, L, 0, C.byref(ctx)))
s = torch.cuda.current_stream()


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return np.median(ts), np.min(ts)


print("pyramid x2:", timeit(lambda: lib.rsvio_build_pyramids_d(ctx, imgs.data_ptr(), 2, pyr.data_ptr(), s.cuda_stream)))
a_dev = torch.from_numpy(aff).to(dev)
out = torch.empty_like(a_dev)
val = torch.empty(300, dtype=torch.uint8, device=dev)
for n in (1, 8, 64, 300):
    for it in (1, 3, 20):
        b = (_lib.TrackBatch * 1)()
        b[0] = _lib.TrackBatch(pyr[0].data_ptr(), pyr[1].data_ptr(), a_dev.data_ptr(), out.data_ptr(),
                               val.data_ptr(), n)
        t = timeit(lambda: lib.rsvio_track_points_d(ctx, b, 1, it, C.c_float(0.01), s.cuda_stream))
        print(f"track n={n:4d} max_iter={it:2d}: median {t[0]:8.1f} us  min {t[1]:8.1f} us")
