"""Profile the Estimator's host logic (rsvio.estimator / rsvio.ba.SlidingWindow) on CPU: the same
config-4 stream through the oracle backend under cProfile, listing the host functions (the
oracle's own calls stand in for the device calls).  usage: python tools/host_profile.py [frames]"""
import cProfile
import pstats
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

from oracle import oracle as O  # noqa: E402
from oracle.estimator import OracleBackend  # noqa: E402
from rsvio import synthetic as S  # noqa: E402
from rsvio.camera import Camera  # noqa: E402
from rsvio.estimator import Estimator  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
O.load()
s = S.euroc_scene_stream(n)
cams = [Camera.opencv5(*p) for p in s.intrinsics]
est = Estimator(752, 480, cams, s.T_B_Cl, s.T_B_Cr, window=10, backend=OracleBackend(O, 752, 480, cams))
pr = cProfile.Profile()
pr.enable()
for l, r in s.frames:
    est.process_frame(l, r)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
