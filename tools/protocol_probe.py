"""Host-time breakdown of bench.py's protocol step (PCIe-inclusive frame + a new
keyframe window per step): tracker enqueue (image H2D, pyramids, LK, feature D2H), the window
upload (rsvio_ba_set_problem), the solve start (graph capture/instantiate/launch) -- in that
order, as bench.py's protocol_step -- the tracker sync, the solve wait and the state read-back.
  python tools/protocol_probe.py [steps] [cu_split] [resident]
(resident = 1: the device-resident step instead -- the same window re-solved, no PCIe -- for
kernel-trace comparisons of the two steps)"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main(steps=60, split=0.25, resident=False):
    import torch

    import rsvio
    from rsvio._lib import CuStream
    rsvio.require_device(0)
    cu_trk, cu_ba = bench.cu_partition(0, split, "block")
    streams = [CuStream(0, cu_trk), CuStream(0, cu_ba)]
    trk = bench.TrackerWorkload(0, streams[0].ptr)
    ba = bench.BAWorkload(0, 1, 0, streams[1].ptr)
    trk.enable_pcie()
    names = ("set_problem", "start", "trk_enqueue", "trk_sync", "finish", "state", "total")
    t = {k: [] for k in names}
    if resident:
        for k in range(steps + 10):
            ba.start()
            trk.step(False)
            ba.finish(False)
        torch.cuda.synchronize()
        ba.ba.close()
        trk.close()
        for st in streams:
            st.close()
        return
    for k in range(steps + 10):
        t0 = time.perf_counter()
        ba.next_window()
        t1 = time.perf_counter()
        ba.start()
        t2 = time.perf_counter()
        trk.step(False, pcie=True, wait=False)
        t3 = time.perf_counter()
        trk.sync()
        t4 = time.perf_counter()
        r = ba.finish(False)
        t5 = time.perf_counter()
        ba.ba.state()
        t6 = time.perf_counter()
        if k >= 10:
            for key, v in zip(names, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t6 - t0)):
                t[key].append(1e3 * v)
    print(f"iterations {r.iterations}, device solve {r.solve_ms:.4f} ms")
    print("protocol step ms (median): " + ", ".join(f"{k} {np.median(v):.4f}" for k, v in t.items()), flush=True)
    torch.cuda.synchronize()
    ba.ba.close()
    trk.close()
    for st in streams:
        st.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 60, float(sys.argv[2]) if len(sys.argv) > 2 else 0.25,
         len(sys.argv) > 3 and sys.argv[3] == "1")
