"""LK launch time of the config-2 frame (3 batches x 300 features, fwd + bwd = 900 one-wave
workgroups) on a stream restricted to the first k CUs, alone on the device: separates the chain
latency (one wave per SIMD or fewer) from issue contention (several waves per SIMD).
  python tools/lk_cu_sweep.py [steps]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]
import bench  # noqa: E402


def main(steps=40):
    import torch

    import rsvio
    from rsvio._lib import CuStream
    rsvio.require_device(0)
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    for k in (32, 64, 96, 128, 192, n_cu):
        st = CuStream(0, list(range(k)))
        trk = bench.TrackerWorkload(0, st.ptr)
        for _ in range(5):
            trk.step(False)
        trk.sync()
        trk.ev.clear()
        for i in range(steps):
            trk.step(True)
        trk.sync()
        print(f"CUs {k:3d}: LK {1e3 * trk.lk_ms():7.1f} us per frame launch (900 chains, "
              f"{900 / (4 * k):.2f} waves per SIMD)", flush=True)
        trk.close()
        st.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 40)
