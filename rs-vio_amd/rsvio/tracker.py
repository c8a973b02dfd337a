"""Host-side mirror of the reference tracker API over the C ABI.

``StereoPatchTracker`` mirrors ``StereoPatchTracker<LEVELS>``
(src/feature_tracker/feature_tracker.rs:91-207): ``new(grid_size, max_iters, thresh)``,
``process_frame(left, right)``, ``get_track_points()``, ``remove_id(ids)``.  The free
functions mirror the reference's module-level ``build_image_pyramid`` (:209-220),
``track_points`` (:252-291) and ``image_utilities::detect_key_points`` (:108-175).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, ptr


def pyramid_bytes(w: int, h: int, levels: int) -> int:
    return int(_lib.load().rsvio_pyramid_bytes(w, h, levels))


def pyramid_levels(pyr: np.ndarray, w: int, h: int, levels: int) -> list[np.ndarray]:
    out, off = [], 0
    for i in range(levels):
        lw, lh = w // (1 << i), h // (1 << i)
        out.append(pyr[off:off + lw * lh].reshape(lh, lw))
        off += lw * lh
    return out


def build_image_pyramid(img: np.ndarray, levels: int) -> np.ndarray:
    """Packed u8 pyramid (level 0 first) of a u8 H x W image."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.empty(pyramid_bytes(w, h, levels), np.uint8)
    check(_lib.load().rsvio_build_pyramid(ptr(img), w, h, levels, ptr(out)))
    return out


def track_points(pyr0: np.ndarray, pyr1: np.ndarray, w: int, h: int, levels: int, aff: np.ndarray,
                 max_iterations: int = 20, thresh: float = 0.01):
    """Forward/backward tracking of n Affine2 states (n x 6 f32); returns (aff_out, valid)."""
    aff = np.ascontiguousarray(aff, np.float32).reshape(-1, 6)
    n = aff.shape[0]
    out = np.empty_like(aff)
    valid = np.zeros(n, np.uint8)
    check(_lib.load().rsvio_track_points(ptr(pyr0), ptr(pyr1), w, h, levels, ptr(aff), n, max_iterations,
                                         C.c_float(thresh), ptr(out), ptr(valid)))
    return out, valid.astype(bool)


def detect_key_points(img: np.ndarray, grid_size: int, existing_xy: np.ndarray | None = None, cap: int = 4096):
    """New corners (k x 2 u32) and their FAST scores in the reference's cell scan order."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    ex = np.zeros((0, 2), np.float32) if existing_xy is None else np.ascontiguousarray(existing_xy, np.float32)
    out = np.zeros((cap, 2), np.uint32)
    score = np.zeros(cap, np.float32)
    n = C.c_int32(0)
    check(_lib.load().rsvio_detect_keypoints(ptr(img), w, h, grid_size, ptr(ex) if len(ex) else None, len(ex),
                                             ptr(out), ptr(score), cap, C.byref(n)))
    return out[:n.value].copy(), score[:n.value].copy()


FEATURE_DTYPE = np.dtype([("id", np.uint64), ("x", np.float32), ("y", np.float32), ("r", np.float32, 4)])


class StereoPatchTracker:
    """Device-resident stereo patch tracker (one HIP stream per instance)."""

    def __init__(self, width: int, height: int, levels: int = 6, grid_size: int = 50,
                 optical_flow_max_iterations: int = 20, optical_flow_convergence_threshold: float = 0.01,
                 device: int = 0, max_features: int = 4096):
        lib = _lib.load()
        p = _lib.TrackerParams(width, height, levels, grid_size, optical_flow_max_iterations,
                               float(optical_flow_convergence_threshold), device, max_features)
        h = C.c_void_p()
        check(lib.rsvio_tracker_create(C.byref(p), C.byref(h)))
        self._h = h
        self.width, self.height, self.levels = width, height, levels
        self.cap = max_features
        self._out_l = np.zeros(max_features, FEATURE_DTYPE)
        self._out_r = np.zeros(max_features, FEATURE_DTYPE)
        self._n = (0, 0)

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().rsvio_tracker_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process_frame(self, left: np.ndarray, right: np.ndarray):
        """Returns (left_features, right_features) structured arrays sorted by id."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        if left.shape != (self.height, self.width) or right.shape != left.shape:
            raise ValueError(f"expected {self.height}x{self.width} images")
        nl, nr = C.c_size_t(0), C.c_size_t(0)
        rc = _lib.load().rsvio_tracker_process_frame(self._h, ptr(left), ptr(right), self.width,
                                                     ptr(self._out_l), self.cap, C.byref(nl),
                                                     ptr(self._out_r), self.cap, C.byref(nr))
        self._n = (nl.value, nr.value)  # RSVIO_ERR_CAPACITY still leaves consistent (truncated) lists
        check(rc)
        return self._out_l[:nl.value].copy(), self._out_r[:nr.value].copy()

    def process_frame_device(self, d_left: int, d_right: int):
        nl, nr = C.c_size_t(0), C.c_size_t(0)
        rc = _lib.load().rsvio_tracker_process_frame_device(self._h, d_left, d_right, ptr(self._out_l), self.cap,
                                                            C.byref(nl), ptr(self._out_r), self.cap, C.byref(nr))
        self._n = (nl.value, nr.value)
        check(rc)
        return nl.value, nr.value

    def submit(self, left: np.ndarray, right: np.ndarray):
        """First half of process_frame (rsvio_tracker_submit): enqueue the frame and return at
        once; the images are borrowed until collect()."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        if left.shape != (self.height, self.width) or right.shape != left.shape:
            raise ValueError(f"expected {self.height}x{self.width} images")
        check(_lib.load().rsvio_tracker_submit(self._h, ptr(left), ptr(right), self.width))
        self._borrowed = (left, right)

    def submit_device(self, d_left: int, d_right: int):
        """rsvio_tracker_submit_device: device images (tightly packed), enqueued; collect() later."""
        check(_lib.load().rsvio_tracker_submit_device(self._h, d_left, d_right))

    def collect_device(self):
        """Second half (rsvio_tracker_collect): wait for the submitted frame; (n_left, n_right),
        the lists in self._out_l / self._out_r."""
        nl, nr = C.c_size_t(0), C.c_size_t(0)
        rc = _lib.load().rsvio_tracker_collect(self._h, ptr(self._out_l), self.cap, C.byref(nl), ptr(self._out_r),
                                               self.cap, C.byref(nr))
        self._n = (nl.value, nr.value)
        self._borrowed = None
        check(rc)
        return nl.value, nr.value

    def collect(self):
        """collect_device() returning (left_features, right_features) like process_frame."""
        nl, nr = self.collect_device()
        return self._out_l[:nl].copy(), self._out_r[:nr].copy()

    def get_track_points(self):
        """[{id: (x, y)} for cam0, cam1] like feature_tracker.rs:188-200."""
        l, r = self._out_l[:self._n[0]], self._out_r[:self._n[1]]
        return [{int(f["id"]): (float(f["x"]), float(f["y"])) for f in l},
                {int(f["id"]): (float(f["x"]), float(f["y"])) for f in r}]

    def set_cameras(self, left, right):
        """Attach the frame's camera models (rsvio.camera.Camera); every process_frame then also
        computes Frame::add_{left,right}_feature's undistorted coordinates on device."""
        if left is None:
            check(_lib.load().rsvio_tracker_set_cameras(self._h, None, None))
            self._cams = False
            return
        self._cl, self._cr = left.struct(), right.struct()
        check(_lib.load().rsvio_tracker_set_cameras(self._h, C.byref(self._cl), C.byref(self._cr)))
        self._cams = True

    def undistorted(self):
        """(n_l x 2, n_r x 2) f32 undistorted coordinates of the last process_frame's features."""
        ul = np.zeros((self._n[0], 2), np.float32)
        ur = np.zeros((self._n[1], 2), np.float32)
        check(_lib.load().rsvio_tracker_undistorted(self._h, ptr(ul), self._n[0], ptr(ur), self._n[1]))
        return ul, ur

    def remove_id(self, ids):
        """StereoPatchTracker::remove_id (feature_tracker.rs:201-206): the device lists are
        compacted in order, so the cached lists are filtered the same way."""
        ids = np.ascontiguousarray(ids, np.uint64)
        check(_lib.load().rsvio_tracker_remove_ids(self._h, ptr(ids), len(ids)))
        n = []
        for out, k in ((self._out_l, self._n[0]), (self._out_r, self._n[1])):
            keep = out[:k][~np.isin(out[:k]["id"], ids)]
            out[:len(keep)] = keep
            n.append(len(keep))
        self._n = tuple(n)
