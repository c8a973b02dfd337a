"""Motion tracking (PnP) + keyframe rule over the C ABI (rsvio_pnp_*, rsvio_track_motion*).

Mirrors SlidingWindow::track_motion (src/estimator/sliding_window.rs:490-587) and the
keyframe decision of Estimator::process_frame (src/estimator/estimator.rs:195-234): one
device launch per frame runs the map join, the PnP LM (10 iterations, Huber 2.0), the
success test, T_W_B = inv(SE3) and the translation / euler-angle thresholds.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, ptr


def pnp_cfg(max_iterations=10, cost_tolerance=1e-6, parameter_tolerance=1e-9, huber_delta=2.0, lambda_init=1e-4):
    """sliding_window.rs:494-501 (SparseCholesky; + HuberLoss::new(2.0) at :538)."""
    return _lib.LmCfg(max_iterations, cost_tolerance, parameter_tolerance, huber_delta, lambda_init, 1)


@dataclass
class MotionResult:
    status: int
    iterations: int
    is_keyframe: bool
    n_observations: int
    initial_cost: float
    final_cost: float
    translation_norm: float
    rotation_norm: float
    T_W_B: np.ndarray
    kernel_ms: float = 0.0  # device time of the launch (wall clock; no host or copy time)

    @property
    def success(self) -> bool:
        """is_optimization_successful (sliding_window.rs:384-395)."""
        return self.status > 0


def _result(r: _lib.MotionResult) -> MotionResult:
    return MotionResult(r.status, r.iterations, bool(r.is_keyframe), r.n_observations, r.initial_cost, r.final_cost,
                        r.translation_norm, r.rotation_norm, np.array(r.T_W_B[:], np.float64).reshape(4, 4),
                        r.kernel_ms)


class MotionTracker:
    """Device handle for track_motion; holds the map (ids ascending, p_W as f32)."""

    def __init__(self, device: int = 0, translation_threshold: float = 0.05, rotation_threshold: float = 0.05):
        h = C.c_void_p()
        check(_lib.load().rsvio_pnp_create(device, C.byref(h)))
        self._h = h
        self.rule = _lib.KeyframeRule(translation_threshold, rotation_threshold)
        self.n_map = 0

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().rsvio_pnp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr):
        """Launch on a caller-owned HIP stream (None: the handle's own)."""
        check(_lib.load().rsvio_pnp_set_stream(self._h, stream_ptr))

    def set_map(self, ids, p_W):
        """map_points (sliding_window.rs:466-475); sorted here if the caller's ids are not."""
        ids = np.asarray(ids, np.uint64).reshape(-1)
        p_W = np.asarray(p_W, np.float32).reshape(-1, 3)
        order = np.argsort(ids, kind="stable")
        ids = np.ascontiguousarray(ids[order])
        p_W = np.ascontiguousarray(p_W[order])
        check(_lib.load().rsvio_pnp_set_map(self._h, ptr(ids), ptr(p_W), len(ids)))
        self.n_map = len(ids)

    def track_motion(self, ids_l, uv_l, ids_r, uv_r, T_W_B_last_kf, T_C_B2, cfg=None) -> MotionResult:
        ids_l = np.ascontiguousarray(ids_l, np.uint64).reshape(-1)
        ids_r = np.ascontiguousarray(ids_r, np.uint64).reshape(-1)
        uv_l = np.ascontiguousarray(uv_l, np.float32).reshape(-1, 2)
        uv_r = np.ascontiguousarray(uv_r, np.float32).reshape(-1, 2)
        Tl = np.ascontiguousarray(T_W_B_last_kf, np.float64).reshape(16)
        tcb = np.ascontiguousarray(T_C_B2, np.float64).reshape(32)
        cfg = cfg or pnp_cfg()
        r = _lib.MotionResult()
        check(_lib.load().rsvio_track_motion(self._h, ptr(ids_l), ptr(uv_l), len(ids_l), ptr(ids_r), ptr(uv_r),
                                             len(ids_r), ptr(Tl), ptr(tcb), C.byref(cfg), C.byref(self.rule),
                                             C.byref(r)))
        return _result(r)

    def track_motion_tracker(self, tracker, T_W_B_last_kf, T_C_B2, cfg=None) -> MotionResult:
        """Features of the tracker's last frame, read on the device (no host round trip)."""
        Tl = np.ascontiguousarray(T_W_B_last_kf, np.float64).reshape(16)
        tcb = np.ascontiguousarray(T_C_B2, np.float64).reshape(32)
        cfg = cfg or pnp_cfg()
        r = _lib.MotionResult()
        check(_lib.load().rsvio_track_motion_tracker(self._h, tracker._h, ptr(Tl), ptr(tcb), C.byref(cfg),
                                                     C.byref(self.rule), C.byref(r)))
        return _result(r)
