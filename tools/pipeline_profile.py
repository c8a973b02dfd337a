"""GPU box: cProfile of the config-4 Estimator over the device backend (pipelined), to find the
host-side cost per frame.  usage: python tools/pipeline_profile.py [frames]"""
import cProfile
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import torch  # noqa: E402

from rsvio import synthetic as S  # noqa: E402
from rsvio.camera import Camera  # noqa: E402
from rsvio.estimator import DeviceBackend, Estimator  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
s = S.euroc_scene_stream_device(n, "cuda:0")
torch.cuda.synchronize()
cams = [Camera.opencv5(*p) for p in s.intrinsics]


def run(frames, prof=None):
    be = DeviceBackend(752, 480, cams, 6, 50, 20, 0.01, 10, 0.05, 0.05, 0)
    est = Estimator(752, 480, cams, s.T_B_Cl, s.T_B_Cr, window=10, backend=be, pipelined=True)
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    for _ in est.run(frames):  # the bench's mode: tracker one frame ahead, pipelined BA
        pass
    est.flush()
    if prof:
        prof.disable()
    el = time.perf_counter() - t0
    est.close()
    return el


run(s.frames[:30])
el = run(s.frames)
print(f"unprofiled: {1e3 * el / n:.3f} ms/frame")
pr = cProfile.Profile()
el = run(s.frames, pr)
print(f"profiled: {1e3 * el / n:.3f} ms/frame")
pstats.Stats(pr).sort_stats("tottime").print_stats(35)
