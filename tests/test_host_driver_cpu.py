"""The native caller side (rs-vio_amd/driver/{protocol,estimator}.cpp, lib/librsvio_host.so): it
loads without a GPU, and the ctypes mirrors of its structs (bench.NativeProtocol,
rsvio.estimator.NativeEstimator) have the C layout (a mismatch would hand the driver wrong
pointers on the GPU box)."""
import ctypes
from pathlib import Path

import bench

LIB = Path(__file__).resolve().parents[1] / "rs-vio_amd" / "lib" / "librsvio_host.so"


def test_driver_loads_and_struct_layout_matches():
    drv = ctypes.CDLL(str(LIB))
    assert hasattr(drv, "rsvio_protocol_run")
    out = (ctypes.c_int64 * 16)()
    drv.rsvio_protocol_layout.restype = ctypes.c_int
    n = drv.rsvio_protocol_layout(out, 16)
    N = bench.NativeProtocol
    want = [ctypes.sizeof(N.Window), ctypes.sizeof(N.Frame), ctypes.sizeof(N.Api), ctypes.sizeof(N.Setup),
            N.Window.T_C_B2.offset, N.Frame.batches.offset, N.Setup.first_step.offset, N.Setup.lk_events.offset,
            N.Setup.n_lk_events.offset, N.Setup.thresh.offset, N.Setup.valid_bytes.offset,
            N.Setup.order.offset, N.Setup.phase_us.offset, N.Setup.n_tl.offset]
    assert n == len(want)
    assert list(out[:n]) == want


def test_native_estimator_struct_layout_matches():
    from rsvio.estimator import NativeEstimator as N
    drv = ctypes.CDLL(str(LIB))
    out = (ctypes.c_int64 * 16)()
    n = drv.rsvio_est_layout(out, 16)
    want = [ctypes.sizeof(N.Api), ctypes.sizeof(N.Setup), ctypes.sizeof(N.FrameOut), ctypes.sizeof(N.Stats),
            N.Setup.rule.offset, N.Setup.pnp_cfg.offset, N.FrameOut.T_W_B.offset, N.Stats.n_solves.offset]
    assert n == len(want) and list(out[:n]) == want
