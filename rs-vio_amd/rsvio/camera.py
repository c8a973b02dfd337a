"""Camera models and batched unprojection (T12: Frame::add_left_feature / add_right_feature,
src/estimator/frame.rs:107-134) over the C ABI.

`Camera.from_config` mirrors create_camera_models_from_config (src/datasets/mod.rs:93-163):
"EUCM"/"eucm" gives EUCM [fx, fy, cx, cy, alpha, beta], anything else OpenCVModel5
[fx, fy, cx, cy, k1, k2, p1, p2, k3] with the same defaults for missing entries.  The
unproject_one return convention of camera-intrinsic-model 0.7.2 cannot be checked offline, so
it is explicit: "plane" returns (x/z, y/z), "ray" the first two unit-ray components.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, ptr

OPENCV5, EUCM = 0, 1
CONVENTIONS = {"plane": 0, "ray": 1}


@dataclass
class Camera:
    model: int
    params: list = field(default_factory=list)
    convention: str = "plane"
    max_iterations: int = 20

    @classmethod
    def opencv5(cls, fx, fy, cx, cy, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0, convention="plane"):
        return cls(OPENCV5, [fx, fy, cx, cy, k1, k2, p1, p2, k3], convention)

    @classmethod
    def eucm(cls, fx, fy, cx, cy, alpha, beta, convention="plane"):
        return cls(EUCM, [fx, fy, cx, cy, alpha, beta], convention)

    @classmethod
    def from_config(cls, intrinsics, distortion, model: str | None = None, convention="plane"):
        """datasets/mod.rs:101-128 for one camera (defaults of the unwrap_or calls)."""
        def get(v, i, d):
            return float(v[i]) if i < len(v) else d
        if (model or "pinhole-radtan") in ("EUCM", "eucm"):
            return cls.eucm(get(intrinsics, 0, 500.0), get(intrinsics, 1, 500.0), get(intrinsics, 2, 320.0),
                            get(intrinsics, 3, 240.0), get(distortion, 0, 0.5), get(distortion, 1, 1.0),
                            convention)
        return cls.opencv5(get(intrinsics, 0, 500.0), get(intrinsics, 1, 500.0), get(intrinsics, 2, 320.0),
                           get(intrinsics, 3, 240.0), *[get(distortion, i, 0.0) for i in range(5)],
                           convention=convention)

    def struct(self) -> _lib.Camera:
        c = _lib.Camera()
        c.model = self.model
        c.convention = CONVENTIONS[self.convention]
        c.max_iterations = self.max_iterations
        for i, v in enumerate(self.params):
            c.params[i] = float(v)
        return c

    def unproject(self, px):
        """n x 2 pixels -> (n x 2 f32 undistorted, valid bool); NaN where invalid."""
        px = np.ascontiguousarray(px, np.float32).reshape(-1, 2)
        out = np.zeros_like(px)
        valid = np.zeros(len(px), np.uint8)
        cs = self.struct()
        check(_lib.load().rsvio_unproject(C.byref(cs), ptr(px), len(px), ptr(out), ptr(valid)))
        return out, valid.astype(bool)

    def unproject_device(self, d_px: int, n: int, d_out: int, d_valid: int | None, stream: int | None = None):
        """Enqueue on device pointers (no synchronisation)."""
        cs = self.struct()
        check(_lib.load().rsvio_unproject_d(C.byref(cs), d_px, n, d_out, d_valid, stream))


# EuRoC cam0/cam1 (config/euroc_vio.yaml:11-17) and TUM-VI EUCM (config/tum_vi.yaml:11-17)
EUROC = (Camera.from_config([458.654, 457.296, 367.215, 248.375],
                            [-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], "pinhole-radtan"),
         Camera.from_config([457.587, 456.134, 379.999, 255.238],
                            [-0.28368365, 0.07451284, -0.00010473, -3.55590700e-05], "pinhole-radtan"))
TUM_VI = (Camera.from_config([191.75556798912652, 191.74816751185256, 254.9226487139376, 256.8780365577954],
                             [0.6246288732884442, 1.0598071085569876], "EUCM"),
          Camera.from_config([191.12575044002125, 191.1082274072055, 252.55828522469696, 255.0183218515494],
                             [0.6246035984060496, 1.0565986975905006], "EUCM"))
