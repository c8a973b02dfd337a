"""Estimator::process_frame (src/estimator/estimator.rs:101-262) over the device pieces: the
full per-frame pipeline of BASELINE config 4.

Per frame (estimator.rs:190-248):
  1. StereoPatchTracker::process_frame (feature_tracker.rs:116-187) -- pyramids, LK, FAST grid
     detection, ids -- with Frame::add_{left,right}_feature's unprojection fused on the device;
  2. if the sliding window is full: SlidingWindow::track_motion (sliding_window.rs:490-587,
     PnP against map_points) and the keyframe rule (estimator.rs:195-234); a failed PnP leaves
     the frame a keyframe with T_W_B = I (frame.rs:95);
  3. a keyframe enters the window (add_frame) and, once the window is full, the window is
     optimised (optimize, sliding_window.rs:159-381); map_points feed the next PnP.

The host logic is the reference's, in canonical order (ids in detection scan
order, features by id).  The heavy work is device work behind the C ABI; `Backend` is the seam
the parity tests use to run the same host logic over the CPU restatement.

Estimator.run(frames) runs the tracker ONE FRAME AHEAD: step 1 of frame t + 1 only needs its two
images (estimator.rs:190 hands the tracker nothing from the window), so it is submitted to the
device as soon as frame t's features are back, and frame t's steps 2-3 (host logic, PnP, the BA
upload and start) run while frame t + 1 tracks.  Results equal process_frame's frame by frame.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from .ba import BundleAdjuster, Frame, SlidingWindow


@dataclass
class FrameResult:
    frame_id: int
    is_keyframe: bool
    T_W_B: np.ndarray
    n_left: int
    n_right: int
    pnp_status: int | None       # None: window not full yet (no motion tracking)
    ba_status: int | None        # None: no optimisation this frame
    pnp_iterations: int | None = None   # LM iterations of the motion tracking
    pnp_cost: float | None = None       # its final cost
    ba_iterations: int | None = None    # LM iterations of the window's solve (the retry's, after a fallback)


class DeviceBackend:
    """StereoPatchTracker (+ fused unprojection), MotionTracker and BundleAdjuster on one device."""

    def __init__(self, width, height, cameras, levels, grid_size, max_iterations, thresh, window,
                 translation_threshold, rotation_threshold, device, ba_cus=None):
        from .motion import MotionTracker
        from .tracker import StereoPatchTracker
        self.tracker = StereoPatchTracker(width, height, levels=levels, grid_size=grid_size,
                                          optical_flow_max_iterations=max_iterations,
                                          optical_flow_convergence_threshold=thresh, device=device)
        self.tracker.set_cameras(cameras[0], cameras[1])
        self.motion = MotionTracker(device, translation_threshold, rotation_threshold)
        self.solver = BundleAdjuster(max_keyframes=max(window, 2), device=device)
        # motion tracking and the BA share one stream: PnP of frame t runs after BA(t - 1) was
        # waited for and before BA(t) starts, so the stream is idle when it launches, and the
        # process needs one stream fewer beside the tracker's (HIP maps streams onto 4 hardware
        # queues per process; PnP queued on the tracker's queue waited behind frame t + 1)
        from ._lib import CuStream
        # ba_cus: the CUs (rsvio_stream_create's mask bits) of the BA + PnP stream; None: all of
        # them -- still through a CU mask: a CU-masked stream gets a hardware queue of its own,
        # where a plain stream takes the next of the process's 4 round-robin queues and may land
        # on the tracker's (PnP then waits behind frame t + 1's tracking: 0.23 ms per frame,
        # 2.5k instead of 3.6k frames/s, profiles/r06z7_config4_ba_cus_ab.txt)
        if not ba_cus:
            import ctypes as C
            from ._lib import check, load
            n = C.c_int(0)
            check(load().rsvio_device_info(device, None, 0, C.byref(n)))
            ba_cus = list(range(n.value))
        self._ba_stream = CuStream(device, ba_cus)
        self.solver.set_stream(self._ba_stream.ptr)
        self.motion.set_stream(self._ba_stream.ptr)

    def submit(self, left, right):
        """Enqueue a frame's tracking: host u8 arrays, or device-resident u8 tensors (data_ptr; no
        H2D copy)."""
        if hasattr(left, "data_ptr"):
            self.tracker.submit_device(left.data_ptr(), right.data_ptr())
        else:
            self.tracker.submit(left, right)

    def collect(self):
        """The submitted frame's features: ((ids, undistorted uv) left, (ids, uv) right)."""
        nl, nr = self.tracker.collect_device()
        fl, fr = self.tracker._out_l[:nl], self.tracker._out_r[:nr]
        ul, ur = self.tracker.undistorted()
        return (fl["id"].astype(np.int64), ul), (fr["id"].astype(np.int64), ur)

    def track(self, left, right):
        self.submit(left, right)
        return self.collect()

    def set_map(self, ids, p_W):
        self.motion.set_map(np.asarray(ids, np.uint64), np.asarray(p_W, np.float32))

    def track_motion(self, T_W_B_last_kf, T_C_B2):
        r = self.motion.track_motion_tracker(self.tracker, T_W_B_last_kf, T_C_B2)
        return r.status, r.is_keyframe, r.T_W_B, r.iterations, r.final_cost

    def close(self):
        for o in (self.tracker, self.motion, self.solver, self._ba_stream):
            o.close()


class Estimator:
    """Estimator (estimator.rs:25-262) for a stereo rig; parameters default to
    config/euroc_vio.yaml (6 pyramid levels, grid 50, 20 LK iterations, threshold 0.01, window
    10, keyframe thresholds 0.05 m / 0.05 rad)."""

    def __init__(self, width: int, height: int, cameras, T_B_Cl, T_B_Cr, levels: int = 6, grid_size: int = 50,
                 max_iterations: int = 20, thresh: float = 0.01, window: int = 10,
                 translation_threshold: float = 0.05, rotation_threshold: float = 0.05, device: int = 0,
                 backend=None, pipelined: bool = False):
        self.backend = backend or DeviceBackend(width, height, cameras, levels, grid_size, max_iterations, thresh,
                                                window, translation_threshold, rotation_threshold, device)
        self.window = SlidingWindow(window, device, solver=self.backend.solver)
        self.T_B_Cl = np.asarray(T_B_Cl, np.float64)
        self.T_B_Cr = np.asarray(T_B_Cr, np.float64)
        self.frame_id = 0
        self._map_key = None
        self._tcb_key = None
        # pipelined: a keyframe's BA solve runs on the device while the next frame is tracked
        # (the tracker never reads the window); its result is applied before the window is next
        # read, so every output equals the sequential order's.  The keyframe's FrameResult gets
        # its ba_status at that point (or at flush()).
        self.pipelined = pipelined
        self._pending_frame = None

    def flush(self):
        """Complete an in-flight BA solve (pipelined mode) and fill its frame's ba_status."""
        if self._pending_frame is not None:
            self.window.finish()
            r = self.window.last_result
            out, frame = self._pending_frame
            out.ba_status = None if r is None else int(r.status)
            out.ba_iterations = None if r is None else int(r.iterations)
            out.T_W_B = frame.T_W_B.copy()  # the solve refined this keyframe's pose too
            self._pending_frame = None

    def _T_C_B2(self):
        # extrinsics of the front keyframe (sliding_window.rs:519-520); the rig is fixed here
        front = self.window.keyframes[0]
        key = front.T_B_Cl.tobytes() + front.T_B_Cr.tobytes()
        if self._tcb_key != key:   # the rig's extrinsics: inverted once, not per frame
            self._tcb = np.linalg.inv(np.stack([front.T_B_Cl, front.T_B_Cr])).reshape(2, 16)
            self._tcb_key = key
        return self._tcb

    def process_frame(self, left: np.ndarray, right: np.ndarray) -> FrameResult:
        return self._process_tracked(self.backend.track(left, right))

    def run(self, frames):
        """process_frame over an iterable of (left, right) image pairs, yielding one FrameResult
        per frame, with the tracker one frame ahead (module docstring): frame t + 1 is submitted
        right after frame t's features are collected, before frame t's motion tracking and BA.
        In pipelined mode a keyframe's FrameResult gets its BA outcome when the solve is next
        waited for (at the latest by flush()); frames left unconsumed are collected on exit."""
        it = iter(frames)
        nxt = next(it, None)
        if nxt is None:
            return
        self.backend.submit(*nxt)
        in_flight = True
        try:
            while in_flight:
                feats = self.backend.collect()
                in_flight = False
                nxt = next(it, None)
                if nxt is not None:
                    self.backend.submit(*nxt)
                    in_flight = True
                yield self._process_tracked(feats)
        finally:
            if in_flight:  # the consumer stopped early: the tracker holds no frame in flight after
                self.backend.collect()

    def _process_tracked(self, feats) -> FrameResult:
        """Steps 2-3 of process_frame (estimator.rs:195-248) for a frame whose features are in."""
        self.frame_id += 1
        (ids_l, uv_l), (ids_r, uv_r) = feats
        frame = Frame(frame_id=self.frame_id, T_W_B=np.eye(4), T_B_Cl=self.T_B_Cl, T_B_Cr=self.T_B_Cr,
                      is_keyframe=True, left_features=(ids_l, uv_l), right_features=(ids_r, uv_r))
        pnp_status = pnp_iters = pnp_cost = None
        self.flush()
        if self.window.is_full():
            if self.window.map_version != self._map_key:  # map_points changes only in optimize
                self.backend.set_map(self.window.map_ids, self.window.map_pw)  # ascending ids, f32
                self._map_key = self.window.map_version
            status, is_kf, T_W_B, pnp_iters, pnp_cost = self.backend.track_motion(
                self.window.keyframes[-1].T_W_B, self._T_C_B2())  # keyframes.back() (sliding_window.rs:506)
            pnp_status = status
            if status > 0:
                frame.T_W_B = T_W_B
                frame.is_keyframe = bool(is_kf)
        ba_status = ba_iters = None
        pending = False
        if frame.is_keyframe:
            self.window.add_frame(frame)
            if self.window.is_full():
                if self.pipelined and self.window.optimize_async() is None:
                    pending = True
                else:
                    self.window.optimize()
                    r = self.window.last_result
                    ba_status = None if r is None else int(r.status)
                    ba_iters = None if r is None else int(r.iterations)
        out = FrameResult(self.frame_id, frame.is_keyframe, frame.T_W_B.copy(), len(ids_l), len(ids_r),
                          pnp_status, ba_status, pnp_iterations=pnp_iters, pnp_cost=pnp_cost,
                          ba_iterations=ba_iters)
        if pending:
            self._pending_frame = (out, frame)
        return out

    def trajectory(self):
        """T_W_B of the keyframes in the window."""
        self.flush()
        return self.window.get_keyframe_poses()

    def close(self):
        self.flush()
        if hasattr(self.backend, "close"):
            self.backend.close()


class NativeEstimator:
    """Estimator.run (pipelined, the tracker one frame ahead) with its host logic in C++
    (lib/librsvio_host.so, rs-vio_amd/driver/estimator.cpp): the same steps over the same
    DeviceBackend handles, as the reference's compiled Rust estimator runs them -- no interpreter
    between the device calls.  Frame for frame the same outputs as Estimator(pipelined=True).run
    (tests/test_estimator_gpu.py); `stats` holds the host wall time per stage."""

    _INT_NONE = -(2 ** 31)

    class Api(C.Structure):
        _fields_ = [(n, C.c_void_p) for n in ("submit_device", "collect", "undistorted", "set_map", "track_motion",
                                              "window_problem", "window_apply", "set_problem", "run_async", "wait",
                                              "run", "get_state")]

    class Setup(C.Structure):
        pass

    class FrameOut(C.Structure):
        _fields_ = [("frame_id", C.c_int32), ("is_keyframe", C.c_int32), ("n_left", C.c_int32),
                    ("n_right", C.c_int32), ("pnp_status", C.c_int32), ("pnp_iterations", C.c_int32),
                    ("ba_status", C.c_int32), ("ba_iterations", C.c_int32), ("pnp_cost", C.c_double),
                    ("T_W_B", C.c_double * 16)]

    class Stats(C.Structure):
        _fields_ = [("track", C.c_double), ("track_motion", C.c_double), ("ba", C.c_double),
                    ("ba_wait", C.c_double), ("total", C.c_double), ("n_solves", C.c_int32),
                    ("ba_iterations", C.c_int32), ("fallbacks", C.c_int32), ("reserved", C.c_int32)]

    def __init__(self, backend: DeviceBackend, T_B_Cl, T_B_Cr, window: int = 10):
        from . import _lib
        from .ba import fallback_cfg, lm_cfg
        from .motion import pnp_cfg
        lib = _lib.load()
        self.drv = C.CDLL(str(_lib.LIB_PATH.parent / "librsvio_host.so"))
        self.drv.rsvio_est_run.restype = C.c_int
        self.drv.rsvio_est_run.argtypes = [C.c_void_p] * 6
        fp = lambda f: C.cast(f, C.c_void_p).value  # noqa: E731
        self.api = self.Api(*[fp(getattr(lib, "rsvio_" + n)) for n in (
            "tracker_submit_device", "tracker_collect", "tracker_undistorted", "pnp_set_map", "track_motion_tracker",
            "window_problem", "window_apply", "ba_set_problem", "ba_run_async", "ba_wait", "ba_run", "ba_get_state")])
        T_B_Cl = np.ascontiguousarray(T_B_Cl, np.float64).reshape(16)
        T_B_Cr = np.ascontiguousarray(T_B_Cr, np.float64).reshape(16)
        # the rig's inverse as the Python Estimator computes it (Estimator._T_C_B2: np.linalg.inv)
        tcb = np.linalg.inv(np.stack([T_B_Cl.reshape(4, 4), T_B_Cr.reshape(4, 4)])).reshape(32)
        self.setup = self.Setup(C.addressof(self.api), backend.tracker._h.value,
                                backend.motion._h.value, backend.solver._h.value, window, backend.tracker.cap,
                                (C.c_double * 16)(*T_B_Cl), (C.c_double * 16)(*T_B_Cr), (C.c_double * 32)(*tcb),
                                lm_cfg(), fallback_cfg(), pnp_cfg(), backend.motion.rule)
        self.stats = None

    def run(self, frames):
        """frames: (left, right) device-resident u8 tensors (data_ptr); returns the FrameResults."""
        n = len(frames)
        dl = (C.c_void_p * max(n, 1))(*[l.data_ptr() for l, _ in frames])
        dr = (C.c_void_p * max(n, 1))(*[r.data_ptr() for _, r in frames])
        out = (self.FrameOut * max(n, 1))()
        st = self.Stats()
        rc = self.drv.rsvio_est_run(C.addressof(self.setup), C.addressof(dl), C.addressof(dr), n, C.addressof(out),
                                    C.addressof(st))
        if rc:
            raise RuntimeError(f"rsvio_est_run failed: {rc}")
        self.stats = st
        none = lambda v: None if v == self._INT_NONE else int(v)  # noqa: E731
        res = []
        for o in out[:n]:
            res.append(FrameResult(o.frame_id, bool(o.is_keyframe), np.array(o.T_W_B[:], np.float64).reshape(4, 4),
                                   o.n_left, o.n_right, none(o.pnp_status), none(o.ba_status),
                                   pnp_iterations=none(o.pnp_iterations),
                                   pnp_cost=None if o.pnp_status == self._INT_NONE else float(o.pnp_cost),
                                   ba_iterations=none(o.ba_iterations)))
        return res


def _native_setup_fields():
    from . import _lib
    return [("api", C.c_void_p), ("tracker", C.c_void_p), ("pnp", C.c_void_p), ("ba", C.c_void_p),
            ("window", C.c_int32), ("max_features", C.c_int32), ("T_B_Cl", C.c_double * 16),
            ("T_B_Cr", C.c_double * 16), ("T_C_B2", C.c_double * 32), ("ba_cfg", _lib.LmCfg),
            ("ba_fallback", _lib.LmCfg), ("pnp_cfg", _lib.LmCfg), ("rule", _lib.KeyframeRule)]


NativeEstimator.Setup._fields_ = _native_setup_fields()
