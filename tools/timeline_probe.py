"""Device timeline of bench.py's protocol step in its default (split) order: HIP events on the
tracker and BA streams, all relative to the step's first event (the image upload's start), plus
the host phases.  Medians over the steps, in microseconds.
  python tools/timeline_probe.py [steps] [order] [graphs]   (order: split | ba-first | frame-first;
                                                            graphs 0: the tracker enqueued directly)
Tracker stream: img_up (the images up: rsvio_upload_async, bench.py's default), down (the frame done: pyramids, LK and the feature
lists' D2H; the kernels' own times come from a rocprofv3 kernel trace).  BA stream: win_up (the window's upload + ba_build_layout done: an event recorded after
set_problem), solve_end (an event after the solve's last kernel: recorded after ba.finish, so it
is the stream's position, not a host wait).  Host: when each call returned."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main(steps=80, order="split", graphs=True):
    import torch

    import rsvio
    from rsvio._lib import CuStream
    rsvio.require_device(0)
    cu_trk, cu_ba = bench.cu_partition(0, 0.25, "block")
    streams = [CuStream(0, cu_trk), CuStream(0, cu_ba)]
    trk = bench.TrackerWorkload(0, streams[0].ptr)
    trk.graphs = graphs
    trk.upload_kernel = True  # bench.py's default (--upload kernel: rsvio_upload_async)
    ba = bench.BAWorkload(0, 1, 0, streams[1].ptr)
    trk.enable_pcie()
    dev = torch.device("cuda", 0)
    ts = torch.cuda.ExternalStream(streams[0].ptr, device=dev)
    bs = torch.cuda.ExternalStream(streams[1].ptr, device=dev)
    E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    rows = []
    state_out = (np.empty((ba.prob.n_kf, 7)), np.empty((ba.prob.n_lm, 3)))
    for k in range(steps + 10):
        ev = {n: E() for n in ("t0", "img_up", "down", "b0", "win_up", "solve_end")}
        h = {}
        t0 = time.perf_counter()
        ev["t0"].record(ts)
        ev["b0"].record(bs)
        if order == "frame-first":
            trk.step(False, pcie=True, wait=False)
        elif order == "split":
            trk.upload()
            ev["img_up"].record(ts)
        h["trk_upload"] = time.perf_counter()
        ba.next_window()
        ev["win_up"].record(bs)
        h["set_problem"] = time.perf_counter()
        ba.start()
        h["start"] = time.perf_counter()
        if order != "frame-first":
            trk.step(False, pcie=True, wait=False, uploaded=order == "split")
        ev["down"].record(ts)
        h["trk_enqueue"] = time.perf_counter()
        trk.sync()
        h["trk_sync"] = time.perf_counter()
        ba.finish(False)
        ev["solve_end"].record(bs)
        h["finish"] = time.perf_counter()
        ba.ba.state(state_out)
        h["state"] = time.perf_counter()
        torch.cuda.synchronize()
        if k >= 10:
            r = {n: 1e3 * ev["t0"].elapsed_time(ev[n]) for n in ("win_up", "solve_end", "down")}
            if order == "split":
                r["img_up"] = 1e3 * ev["t0"].elapsed_time(ev["img_up"])
            r.update({f"host_{n}": 1e6 * (v - t0) for n, v in h.items()})
            rows.append(r)
    keys = rows[0].keys()
    print(f"order {order}: medians over {steps} steps, us from the step's start")
    for n in keys:
        print(f"  {n:18s} {np.median([r[n] for r in rows]):8.1f}")
    torch.cuda.synchronize()
    ba.ba.close()
    trk.close()
    for st in streams:
        st.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 80, sys.argv[2] if len(sys.argv) > 2 else "split",
         not (len(sys.argv) > 3 and sys.argv[3] == "0"))
