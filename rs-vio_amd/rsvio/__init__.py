"""rsvio -- MI355X-native RS-VIO hot paths (patch tracker + sliding-window BA).

Python host mirror of the reference's Rust API over the C ABI (include/rsvio_gpu.h).
All compute runs in lib/librsvio_gpu.so (HIP, gfx950); there is no CPU fallback.
"""
from ._lib import RsvioError, load, require_device  # noqa: F401
from .tracker import (StereoPatchTracker, build_image_pyramid, detect_key_points,  # noqa: F401
                      pyramid_bytes, pyramid_levels, track_points)

__all__ = ["RsvioError", "load", "require_device", "StereoPatchTracker", "build_image_pyramid",
           "detect_key_points", "pyramid_bytes", "pyramid_levels", "track_points"]
