"""ctypes binding of the C ABI in include/rsvio_gpu.h (lib/librsvio_gpu.so).

The library is the only compute path: there is no CPU fallback.  Loading fails loudly when
the .so is missing, and every call that returns a negative status raises RsvioError with the
library's own message.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # rs-vio_amd/
LIB_PATH = PKG_ROOT / "lib" / "librsvio_gpu.so"

RSVIO_OK = 0
ERRORS = {
    -1: "RSVIO_ERR_INVALID_ARG", -2: "RSVIO_ERR_HIP", -3: "RSVIO_ERR_NOMEM", -4: "RSVIO_ERR_CAPACITY",
    -5: "RSVIO_ERR_NO_DEVICE", -6: "RSVIO_ERR_INTERNAL", -7: "RSVIO_ERR_RCCL",
}
LM_STATUS = {1: "CostToleranceReached", 2: "ParameterToleranceReached", 3: "MaxIterationsReached",
             4: "TrustRegionRadiusTooSmall", -1: "NumericalFailure", -2: "Skipped", -3: "LinearSolveFailed"}


class RsvioError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class TrackerParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("levels", C.c_int32),
                ("grid_size", C.c_int32), ("max_iterations", C.c_int32),
                ("convergence_threshold", C.c_float), ("device", C.c_int32),
                ("max_features", C.c_int32)]


class Feature(C.Structure):
    _fields_ = [("id", C.c_uint64), ("x", C.c_float), ("y", C.c_float), ("r", C.c_float * 4)]


class TrackBatch(C.Structure):
    _fields_ = [("d_pyr0", C.c_void_p), ("d_pyr1", C.c_void_p), ("d_aff_in", C.c_void_p),
                ("d_aff_out", C.c_void_p), ("d_valid", C.c_void_p), ("n", C.c_int32)]


class LmCfg(C.Structure):
    _fields_ = [("max_iterations", C.c_int32), ("cost_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double), ("huber_delta", C.c_double),
                ("lambda_init", C.c_double), ("linear_solver", C.c_int32)]


class BaResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("iterations", C.c_int32), ("initial_cost", C.c_double),
                ("final_cost", C.c_double), ("solve_ms", C.c_double)]


class Camera(C.Structure):
    _fields_ = [("model", C.c_int32), ("convention", C.c_int32), ("max_iterations", C.c_int32),
                ("reserved", C.c_int32), ("params", C.c_double * 9)]


class KeyframeRule(C.Structure):
    _fields_ = [("translation_threshold", C.c_double), ("rotation_threshold", C.c_double)]


class MotionResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("iterations", C.c_int32), ("is_keyframe", C.c_int32),
                ("n_observations", C.c_int32), ("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("translation_norm", C.c_double), ("rotation_norm", C.c_double), ("T_W_B", C.c_double * 16),
                ("kernel_ms", C.c_double)]


class BaParams(C.Structure):
    _fields_ = [("max_keyframes", C.c_int32), ("max_landmarks", C.c_int32),
                ("max_observations", C.c_int32), ("device", C.c_int32)]


class FtConfig(C.Structure):
    """rsvio_ft_config (64 B): FeatureTrackingConfig (feature_tracker/src/feature_tracker.rs:25-38)."""
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("nlevels", C.c_int32),
                ("preprocessing_blur", C.c_int32), ("ratio", C.c_double), ("preprocessing_blur_sigma", C.c_float),
                ("detection_threshold", C.c_float), ("detection_min_dist", C.c_uint32), ("detection_blur", C.c_float),
                ("optical_flow_max_iter", C.c_int32), ("optical_flow_lm_lambda", C.c_float),
                ("matching_cost", C.c_int32), ("device", C.c_int32), ("max_features", C.c_int32),
                ("reserved", C.c_int32)]


class FtFeature(C.Structure):
    _fields_ = [("feature_id", C.c_uint64), ("x", C.c_float), ("y", C.c_float)]


P = C.c_void_p
SIG = {
    "rsvio_last_error": (C.c_char_p, []),
    "rsvio_device_info": (C.c_int, [C.c_int, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]),
    "rsvio_tracker_create": (C.c_int, [C.POINTER(TrackerParams), C.POINTER(P)]),
    "rsvio_tracker_destroy": (None, [P]),
    "rsvio_tracker_process_frame": (C.c_int, [P, P, P, C.c_size_t, P, C.c_size_t, C.POINTER(C.c_size_t), P,
                                              C.c_size_t, C.POINTER(C.c_size_t)]),
    "rsvio_tracker_process_frame_device": (C.c_int, [P, P, P, P, C.c_size_t, C.POINTER(C.c_size_t), P,
                                                     C.c_size_t, C.POINTER(C.c_size_t)]),
    "rsvio_window_problem": (C.c_int, [C.c_int32, P, P, P, P, P, P, P, C.c_int32, P, P, P, C.c_int32, P, P,
                                       C.POINTER(C.c_int32), C.c_int32, P, P, P, P, C.POINTER(C.c_int32)]),
    "rsvio_window_apply": (C.c_int, [C.c_int32, P, C.c_int32, P, P, P, P, P]),
    "rsvio_tracker_submit": (C.c_int, [P, P, P, C.c_size_t]),
    "rsvio_tracker_submit_device": (C.c_int, [P, P, P]),
    "rsvio_tracker_collect": (C.c_int, [P, P, C.c_size_t, C.POINTER(C.c_size_t), P, C.c_size_t,
                                        C.POINTER(C.c_size_t)]),
    "rsvio_tracker_remove_ids": (C.c_int, [P, P, C.c_size_t]),
    "rsvio_tracker_stream": (P, [P]),
    "rsvio_sincosf": (C.c_int, [P, C.c_size_t, P, P]),
    "rsvio_sincosf_digest": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint32, P]),
    "rsvio_unproject": (C.c_int, [C.POINTER(Camera), P, C.c_size_t, P, P]),
    "rsvio_unproject_d": (C.c_int, [C.POINTER(Camera), P, C.c_size_t, P, P, P]),
    "rsvio_tracker_set_cameras": (C.c_int, [P, C.POINTER(Camera), C.POINTER(Camera)]),
    "rsvio_tracker_undistorted": (C.c_int, [P, P, C.c_size_t, P, C.c_size_t]),
    "rsvio_quat_from_matrix": (C.c_int, [P, C.c_size_t, P]),
    "rsvio_pnp_create": (C.c_int, [C.c_int32, C.POINTER(P)]),
    "rsvio_pnp_destroy": (None, [P]),
    "rsvio_pnp_set_stream": (C.c_int, [P, P]),
    "rsvio_pnp_set_map": (C.c_int, [P, P, P, C.c_int32]),
    "rsvio_track_motion": (C.c_int, [P, P, P, C.c_size_t, P, P, C.c_size_t, P, P, C.POINTER(LmCfg),
                                     C.POINTER(KeyframeRule), C.POINTER(MotionResult)]),
    "rsvio_track_motion_tracker": (C.c_int, [P, P, P, P, C.POINTER(LmCfg), C.POINTER(KeyframeRule),
                                             C.POINTER(MotionResult)]),
    "rsvio_pyramid_bytes": (C.c_size_t, [C.c_int32, C.c_int32, C.c_int32]),
    "rsvio_build_pyramid": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int32, P]),
    "rsvio_track_points": (C.c_int, [P, P, C.c_int32, C.c_int32, C.c_int32, P, C.c_int32, C.c_int32, C.c_float,
                                     P, P]),
    "rsvio_detect_keypoints": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int32, P, C.c_int32, P, P, C.c_int32,
                                         C.POINTER(C.c_int32)]),
    "rsvio_track_ctx_create": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.POINTER(P)]),
    "rsvio_track_ctx_destroy": (None, [P]),
    "rsvio_build_pyramids_d": (C.c_int, [P, P, C.c_int32, P, P]),
    "rsvio_track_points_d": (C.c_int, [P, C.POINTER(TrackBatch), C.c_int32, C.c_int32, C.c_float, P]),
    "rsvio_track_points_table_d": (C.c_int, [P, P, P, C.c_int32, C.c_int32, C.c_int32, C.c_float, P]),
    "rsvio_ba_create": (C.c_int, [C.POINTER(BaParams), C.POINTER(P)]),
    "rsvio_ba_destroy": (None, [P]),
    "rsvio_ba_solve": (C.c_int, [P, C.c_int32, P, P, C.c_int32, P, C.c_int32, P, P, P, P, P,
                                 C.POINTER(LmCfg), C.POINTER(BaResult)]),
    "rsvio_ba_set_problem": (C.c_int, [P, C.c_int32, P, P, C.c_int32, P, C.c_int32, P, P, P, P, P]),
    "rsvio_ba_run": (C.c_int, [P, C.POINTER(LmCfg), C.POINTER(BaResult)]),
    "rsvio_ba_run_async": (C.c_int, [P, C.POINTER(LmCfg)]),
    "rsvio_ba_set_stream": (C.c_int, [P, P]),
    "rsvio_ba_batch_create": (C.c_int, [P, C.c_int32, C.POINTER(P)]),
    "rsvio_ba_batch_run": (C.c_int, [P, C.POINTER(LmCfg), P]),
    "rsvio_ba_batch_destroy": (None, [P]),
    "rsvio_ba_p2p_export": (C.c_int, [P, C.c_int32, C.POINTER(C.c_uint8), C.c_size_t]),
    "rsvio_ba_attach_p2p": (C.c_int, [P, C.c_int32, C.c_int32, C.POINTER(C.c_uint8)]),
    "rsvio_ba_p2p_latency": (C.c_int, [P, C.c_int32, C.c_int32, C.POINTER(C.c_double)]),
    "rsvio_ba_detach_p2p": (C.c_int, [P]),
    "rsvio_ba_p2p_level": (C.c_int, [P, C.POINTER(C.c_int32)]),
    "rsvio_stream_create": (C.c_int, [C.c_int32, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(P)]),
    "rsvio_stream_destroy": (C.c_int, [P]),
    "rsvio_upload_async": (C.c_int, [P, P, C.c_size_t, P]),
    "rsvio_ba_wait": (C.c_int, [P, C.POINTER(BaResult)]),
    "rsvio_ba_get_state": (C.c_int, [P, P, P]),
    "rsvio_ba_build_system": (C.c_int, [P, C.c_double, C.c_double, P, P, C.POINTER(C.c_double)]),
    "rsvio_rccl_unique_id": (C.c_int, [P, C.c_size_t]),
    "rsvio_ba_attach_comm": (C.c_int, [P, C.c_int32, C.c_int32, P]),
    "rsvio_ft_create": (C.c_int, [C.POINTER(FtConfig), C.POINTER(P)]),
    "rsvio_ft_destroy": (None, [P]),
    "rsvio_ft_process_frame": (C.c_int, [P, P, C.c_size_t, P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rsvio_ft_process_frame_device": (C.c_int, [P, P, P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rsvio_ft_get_pyramid": (C.c_int, [P, P, C.c_size_t]),
    "rsvio_ft_stream": (P, [P]),
    "rsvio_ft_pyramid_floats": (C.c_size_t, [C.c_int32, C.c_int32, C.c_int32, C.c_double]),
    "rsvio_ft_build_pyramid": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_int32, C.c_float, P]),
    "rsvio_ft_track_points": (C.c_int, [P, P, C.c_int32, C.c_int32, C.c_int32, C.c_double, P, C.c_int32, C.c_int32,
                                        C.c_float, C.c_int32, P, P]),
    "rsvio_ft_shi_tomasi_score": (C.c_int, [P, C.c_int32, C.c_int32, C.c_float, P]),
    "rsvio_ft_add_points": (C.c_int, [P, C.c_int32, C.c_int32, P, C.c_int32, C.c_float, C.c_int32, C.c_float, P,
                                      C.c_int32, C.POINTER(C.c_int32)]),
}

_lib = None


def load() -> C.CDLL:
    """Load lib/librsvio_gpu.so; raises if it has not been built (no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("RSVIO_LIB", LIB_PATH))
    if not path.exists():
        raise RuntimeError(f"{path} not found: build it with `make -C rs-vio_amd` (hipcc, gfx950); "
                           "rsvio has no CPU fallback")
    # One HIP runtime per process: torch's wheel bundles its own libamdhip64 (loaded under the
    # file name libamdhip64.so, SONAME libamdhip64.so.7).  If librsvio_gpu.so were loaded first
    # it would pull /opt/rocm's copy and a later torch import would bring a second runtime that
    # sees no device.  Importing torch first makes the library bind to the already-loaded one.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(str(path))
    for name, (res, args) in SIG.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:  # tests/test_abi_cpu.py asserts every declared symbol is exported
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(code: int) -> int:
    if code < 0:
        msg = load().rsvio_last_error()
        raise RsvioError(code, msg.decode() if msg else "")
    return code


def ptr(a) -> int | None:
    """Host pointer of a C-contiguous numpy array (or None)."""
    if a is None:
        return None
    ai = a.__array_interface__  # (half the cost of a.ctypes.data; strides None = C-contiguous)
    if ai["strides"] is not None and not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return ai["data"][0]


def require_device(device: int = 0) -> str:
    lib = load()
    name = C.create_string_buffer(64)
    ncu = C.c_int(0)
    check(lib.rsvio_device_info(device, name, 64, C.byref(ncu)))
    return name.value.decode()


class CuStream:
    """A HIP stream restricted to a set of CUs (rsvio_stream_create); .ptr is the hipStream_t."""

    def __init__(self, device: int, cus=None):
        lib = load()
        out = C.c_void_p()
        if cus is None:
            check(lib.rsvio_stream_create(device, None, 0, C.byref(out)))
        else:
            n = max(cus) + 1
            words = (n + 31) // 32
            mask = (C.c_uint32 * words)()
            for c in cus:
                mask[c // 32] |= 1 << (c % 32)
            check(lib.rsvio_stream_create(device, mask, words, C.byref(out)))
        self.ptr = out.value

    def close(self):
        if self.ptr:
            check(load().rsvio_stream_destroy(self.ptr))
            self.ptr = None
