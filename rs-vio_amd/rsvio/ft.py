"""Host-side mirror of the standalone ``feature_tracker/`` crate's API over the C ABI.

``FeatureTracker`` mirrors ``FeatureTracker`` (feature_tracker/src/feature_tracker.rs:51-194):
``FeatureTracker(config)``, ``process_frame(in_image, frame) -> frame``, ``get_pyramid()``.
``FeatureTrackingConfig`` mirrors the serde struct of :25-38 (defaults = config/config.yaml).
The free functions mirror ``image_operations::build_image_pyramid`` (:47-78),
``feature_tracking::track_points`` (:16-61), ``shi_tomasi_score`` and ``add_points``
(feature_detection.rs:47-164).  Images are f32 luma in [0, 1] (``to_luma32f``).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, ptr

SSD, LSSD = 0, 1   # MatchingCost (patch.rs:6-9)


@dataclass
class FeatureTrackingConfig:
    nlevels: int = 5
    ratio: float = 2.0
    preprocessing_blur: bool = True
    preprocessing_blur_sigma: float = 2.0
    detection_threshold: float = 2.5
    detection_min_dist: int = 15
    detection_blur: float = 6.0
    optical_flow_max_iter: int = 25
    optical_flow_lm_lambda: float = 0.1

    def struct(self, width: int, height: int, matching_cost: int = SSD, device: int = 0,
               max_features: int = 8192) -> _lib.FtConfig:
        return _lib.FtConfig(width, height, self.nlevels, int(self.preprocessing_blur), self.ratio,
                             self.preprocessing_blur_sigma, self.detection_threshold, self.detection_min_dist,
                             self.detection_blur, self.optical_flow_max_iter, self.optical_flow_lm_lambda,
                             matching_cost, device, max_features, 0)


@dataclass
class Feature:
    """feature_tracker.rs:41-48"""
    feature_id: int
    central_point: tuple


@dataclass
class Frame:
    """feature_tracker/src/ext.rs:3-15"""
    frame_id: int
    features: list = field(default_factory=list)


FT_FEATURE_DTYPE = np.dtype([("feature_id", np.uint64), ("x", np.float32), ("y", np.float32)])


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


def pyramid_floats(w: int, h: int, nlevels: int, ratio: float = 2.0) -> int:
    return int(_lib.load().rsvio_ft_pyramid_floats(w, h, nlevels, ratio))


def level_dims(w: int, h: int, nlevels: int, ratio: float = 2.0) -> list[tuple[int, int]]:
    """image_operations.rs:69-70: level l is round(w / ratio^l) x round(h / ratio^l)."""
    out = []
    for l in range(nlevels):
        if l == 0:
            out.append((w, h))
        else:
            p = ratio ** l
            out.append((int(np.floor(w / p + 0.5)), int(np.floor(h / p + 0.5))))
    return out


def pyramid_levels(pyr: np.ndarray, w: int, h: int, nlevels: int, ratio: float = 2.0) -> list[np.ndarray]:
    out, off = [], 0
    for lw, lh in level_dims(w, h, nlevels, ratio):
        out.append(pyr[off:off + lw * lh].reshape(lh, lw))
        off += lw * lh
    return out


def build_image_pyramid(img: np.ndarray, nlevels: int = 5, ratio: float = 2.0, bluring: bool = True,
                        blur_sigma: float = 2.0) -> np.ndarray:
    """Packed f32 pyramid (level 0 first) of an f32 H x W image."""
    img = _f32(img)
    h, w = img.shape
    out = np.empty(pyramid_floats(w, h, nlevels, ratio), np.float32)
    check(_lib.load().rsvio_ft_build_pyramid(ptr(img), w, h, nlevels, ratio, int(bluring), C.c_float(blur_sigma),
                                             ptr(out)))
    return out


def track_points(pyr0: np.ndarray, pyr1: np.ndarray, w: int, h: int, xy: np.ndarray, nlevels: int = 5,
                 ratio: float = 2.0, max_iteration: int = 25, lm_lambda: float = 0.1, matching_cost: int = SSD):
    """Forward/backward tracking of n centres; returns (n x 4 {cos, sin, tx, ty}, keep mask)."""
    xy = _f32(xy).reshape(-1, 2)
    n = len(xy)
    iso = np.zeros((n, 4), np.float32)
    valid = np.zeros(n, np.uint8)
    check(_lib.load().rsvio_ft_track_points(ptr(_f32(pyr0)), ptr(_f32(pyr1)), w, h, nlevels, ratio,
                                            ptr(xy) if n else None, n, max_iteration, C.c_float(lm_lambda),
                                            matching_cost, ptr(iso), ptr(valid)))
    return iso, valid.astype(bool)


def shi_tomasi_score(img: np.ndarray, detection_blur: float = 6.0) -> np.ndarray:
    img = _f32(img)
    out = np.empty_like(img)
    check(_lib.load().rsvio_ft_shi_tomasi_score(ptr(img), img.shape[1], img.shape[0], C.c_float(detection_blur),
                                                ptr(out)))
    return out


def add_points(fine: np.ndarray, tracked_xy=None, threshold: float = 2.5, min_dist: int = 15,
               detection_blur: float = 6.0, cap: int = 1 << 16) -> np.ndarray:
    """New Shi-Tomasi corners (k x 2 u32) in (y, x) order."""
    fine = _f32(fine)
    tr = np.zeros((0, 2), np.float32) if tracked_xy is None else _f32(tracked_xy).reshape(-1, 2)
    out = np.zeros((cap, 2), np.uint32)
    n = C.c_int32(0)
    check(_lib.load().rsvio_ft_add_points(ptr(fine), fine.shape[1], fine.shape[0], ptr(tr) if len(tr) else None,
                                          len(tr), C.c_float(threshold), min_dist, C.c_float(detection_blur),
                                          ptr(out), cap, C.byref(n)))
    return out[:n.value].copy()


class FeatureTracker:
    """Device-resident FeatureTracker (one HIP stream per instance)."""

    def __init__(self, width: int, height: int, config: FeatureTrackingConfig | None = None,
                 matching_cost: int = SSD, device: int = 0, max_features: int = 8192):
        self.config = config or FeatureTrackingConfig()
        self.width, self.height = width, height
        self._cfg = self.config.struct(width, height, matching_cost, device, max_features)
        h = C.c_void_p()
        check(_lib.load().rsvio_ft_create(C.byref(self._cfg), C.byref(h)))
        self._h = h
        self.cap = max_features
        self._out = np.zeros(max_features, FT_FEATURE_DTYPE)
        self.n = 0

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().rsvio_ft_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, in_image: np.ndarray) -> np.ndarray:
        """One frame; returns frame.features as a structured array (feature_id, x, y)."""
        img = _f32(in_image)
        if img.shape != (self.height, self.width):
            raise ValueError(f"expected a {self.height}x{self.width} image")
        n = C.c_size_t(0)
        check(_lib.load().rsvio_ft_process_frame(self._h, ptr(img), self.width, ptr(self._out), self.cap,
                                                 C.byref(n)))
        self.n = n.value
        return self._out[:n.value].copy()

    def process_frame(self, in_image: np.ndarray, frame: Frame) -> Frame:
        """feature_tracker.rs:77-185: fills frame.features (tracked first, then new corners)."""
        for f in self.process(in_image):
            frame.features.append(Feature(int(f["feature_id"]), (float(f["x"]), float(f["y"]))))
        return frame

    def process_frame_device(self, d_img: int) -> int:
        n = C.c_size_t(0)
        check(_lib.load().rsvio_ft_process_frame_device(self._h, d_img, ptr(self._out), self.cap, C.byref(n)))
        self.n = n.value
        return n.value

    def features(self) -> np.ndarray:
        return self._out[:self.n].copy()

    def get_pyramid(self) -> list[np.ndarray]:
        """feature_tracker.rs:190-193: the last frame's pyramid levels."""
        c = self.config
        out = np.empty(pyramid_floats(self.width, self.height, c.nlevels, c.ratio), np.float32)
        check(_lib.load().rsvio_ft_get_pyramid(self._h, ptr(out), len(out)))
        return pyramid_levels(out, self.width, self.height, c.nlevels, c.ratio)

    @property
    def stream(self) -> int:
        return _lib.load().rsvio_ft_stream(self._h)
