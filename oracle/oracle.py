"""ctypes binding of the CPU oracle (oracle/librsvio_oracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker / the timed CPU baseline -- never as the product path.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "librsvio_oracle.so"

P = C.c_void_p


class LmCfg(C.Structure):
    _fields_ = [("max_iterations", C.c_int), ("cost_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double), ("huber_delta", C.c_double),
                ("lambda_init", C.c_double), ("linear_solver", C.c_int)]


class BaResult(C.Structure):
    _fields_ = [("status", C.c_int), ("iterations", C.c_int), ("initial_cost", C.c_double),
                ("final_cost", C.c_double)]


class OrcFeature(C.Structure):
    _fields_ = [("id", C.c_uint64), ("x", C.c_float), ("y", C.c_float), ("aff", C.c_float * 6)]


class OrcCamera(C.Structure):
    _fields_ = [("model", C.c_int32), ("convention", C.c_int32), ("max_iterations", C.c_int32),
                ("reserved", C.c_int32), ("params", C.c_double * 9)]


class OrcMotionResult(C.Structure):
    _fields_ = [("status", C.c_int), ("iterations", C.c_int), ("is_keyframe", C.c_int), ("n_observations", C.c_int),
                ("initial_cost", C.c_double), ("final_cost", C.c_double), ("translation_norm", C.c_double),
                ("rotation_norm", C.c_double), ("T_W_B", C.c_double * 16), ("pose7", C.c_double * 7)]


_SIG = {
    "orc_ft_level_dims": (None, [C.c_int, C.c_int, C.c_int, C.c_double, P]),
    "orc_ft_pyramid_floats": (C.c_size_t, [C.c_int, C.c_int, C.c_int, C.c_double]),
    "orc_ft_resize_triangle": (None, [P, C.c_int, C.c_int, P, C.c_int, C.c_int]),
    "orc_ft_gaussian_blur": (None, [P, C.c_int, C.c_int, C.c_float, P]),
    "orc_ft_fast_blur": (None, [P, C.c_int, C.c_int, C.c_float, P]),
    "orc_ft_boxes_for_gauss": (None, [C.c_float, C.c_int, P]),
    "orc_ft_build_pyramid": (None, [P, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_float, P]),
    "orc_ft_bicubic": (C.c_int, [P, C.c_int, C.c_int, C.c_float, C.c_float, P]),
    "orc_ft_exp_se2": (None, [P, P]),
    "orc_ft_log_se2": (None, [P, P]),
    "orc_ft_patch_new": (C.c_int, [P, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_int, P, P, P]),
    "orc_ft_track_points": (None, [P, P, C.c_int, C.c_int, C.c_int, C.c_double, P, C.c_int, C.c_int, C.c_float,
                                   C.c_int, P, P]),
    "orc_ft_shi_tomasi_score": (None, [P, C.c_int, C.c_int, C.c_float, P]),
    "orc_ft_suppress_non_maximum": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_float, P, P, C.c_int]),
    "orc_ft_add_points": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, C.c_float, C.c_int, C.c_float, P, C.c_int]),
    "orc_ft_create": (P, [C.c_void_p, C.c_int, C.c_int]),
    "orc_ft_destroy": (None, [P]),
    "orc_ft_process_frame": (C.c_int, [P, P, P, P, C.c_int, C.POINTER(C.c_int)]),
    "orc_track_motion": (C.c_int, [P, P, C.c_int, P, P, C.c_int, P, P, C.c_int, P, P, C.POINTER(LmCfg),
                                   C.c_double, C.c_double, C.POINTER(OrcMotionResult)]),
    "orc_unproject": (C.c_int, [C.POINTER(OrcCamera), P, C.c_size_t, P, P]),
    "orc_project": (C.c_int, [C.POINTER(OrcCamera), P, C.c_size_t, P, P]),
    "orc_set_ba_threads": (None, [C.c_int]),
    "orc_libm_sincosf_digest": (None, [C.c_uint64, C.c_uint64, C.c_uint32, C.c_int, P]),
    "orc_se2_exp": (None, [P, P]),
    "orc_pyramid_offset": (C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    "orc_pyramid_bytes": (C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    "orc_build_pyramid": (None, [P, C.c_int, C.c_int, C.c_int, P]),
    "orc_build_pyramid_mt": (None, [P, C.c_int, C.c_int, C.c_int, P, C.c_int]),
    "orc_resize_triangle": (None, [P, C.c_int, C.c_int, P, C.c_int, C.c_int]),
    "orc_pattern52_new": (C.c_int, [P, C.c_int, C.c_int, C.c_float, C.c_float, P, P, P]),
    "orc_track_one_point": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P, C.c_int, C.c_float, P]),
    "orc_track_points": (None, [P, P, C.c_int, C.c_int, C.c_int, P, C.c_int, C.c_int, C.c_float, P, P, C.c_int]),
    "orc_fast9_scores": (C.c_int, [P, C.c_int, C.c_int, C.c_int, P]),
    "orc_detect_keypoints": (C.c_int, [P, C.c_int, C.c_int, C.c_int, P, C.c_int, P, P, C.c_int]),
    "orc_tracker_create": (P, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float]),
    "orc_tracker_destroy": (None, [P]),
    "orc_tracker_set_threads": (None, [P, C.c_int]),
    "orc_tracker_process_frame": (C.c_int, [P, P, P, P, C.c_int, C.POINTER(C.c_int), P, C.c_int,
                                            C.POINTER(C.c_int)]),
    "orc_tracker_remove_ids": (None, [P, P, C.c_int]),
    "orc_ba_factor_linearize": (None, [P, P, P, P, P, P, P]),
    "orc_ba_build_system": (C.c_int, [C.c_int, P, P, C.c_int, P, C.c_int, P, P, P, P, P, C.c_double,
                                      C.c_double, P, P, C.POINTER(C.c_double)]),
    "orc_ba_solve": (C.c_int, [C.c_int, P, P, C.c_int, P, C.c_int, P, P, P, P, P, C.POINTER(LmCfg),
                               C.POINTER(BaResult)]),
    "orc_se3_plus": (None, [P, P, P]),
    "orc_quat_from_rotation": (None, [P, P]),
    "orc_quat_from_matrix": (None, [P, P]),
}

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = C.CDLL(str(LIB))
        for k, (r, a) in _SIG.items():
            f = getattr(lib, k)
            f.restype = r
            f.argtypes = a
        _lib = lib
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def libm_sincosf_digest(first: int, count: int, chunk_log2: int, nthreads: int = 8):
    """libm sinf/cosf digests per 2^chunk_log2 inputs (rsvio_sincosf_digest's definition)."""
    n = (count + (1 << chunk_log2) - 1) >> chunk_log2
    out = np.zeros(n, np.uint64)
    load().orc_libm_sincosf_digest(first, count, chunk_log2, nthreads, out.ctypes.data)
    return out


def se2_exp(twist):
    tw = np.ascontiguousarray(twist, np.float32)
    out = np.zeros((3, 3), np.float32)
    load().orc_se2_exp(_p(tw), _p(out))
    return out


def pyramid_bytes(w, h, levels):
    return int(load().orc_pyramid_bytes(w, h, levels))


def build_pyramid(img: np.ndarray, levels: int, n_threads: int = 1) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.empty(pyramid_bytes(w, h, levels), np.uint8)
    if n_threads > 1:
        load().orc_build_pyramid_mt(_p(img), w, h, levels, _p(out), n_threads)
    else:
        load().orc_build_pyramid(_p(img), w, h, levels, _p(out))
    return out


def resize_triangle(img: np.ndarray, nw: int, nh: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.empty((nh, nw), np.uint8)
    load().orc_resize_triangle(_p(img), w, h, _p(out), nw, nh)
    return out


def pattern52(img: np.ndarray, px: float, py: float):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    data = np.zeros(52, np.float32)
    hj = np.zeros((3, 52), np.float32)
    mean = C.c_float(0)
    v = load().orc_pattern52_new(_p(img), w, h, px, py, _p(data), _p(hj), C.byref(mean))
    return bool(v), data, hj, mean.value


def track_points(pyr0, pyr1, w, h, levels, aff, max_iterations=20, thresh=0.01, n_threads=1):
    aff = np.ascontiguousarray(aff, np.float32).reshape(-1, 6)
    n = aff.shape[0]
    out = np.empty_like(aff)
    valid = np.zeros(n, np.uint8)
    load().orc_track_points(_p(pyr0), _p(pyr1), w, h, levels, _p(aff), n, max_iterations, C.c_float(thresh),
                            _p(out), _p(valid), n_threads)
    return out, valid.astype(bool)


def fast9_scores(img, threshold):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), np.uint8)
    load().orc_fast9_scores(_p(img), w, h, threshold, _p(out))
    return out


def detect_key_points(img, grid, existing_xy=None, cap=4096):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    ex = np.zeros((0, 2), np.float32) if existing_xy is None else np.ascontiguousarray(existing_xy, np.float32)
    out = np.zeros((cap, 2), np.uint32)
    sc = np.zeros(cap, np.float32)
    n = load().orc_detect_keypoints(_p(img), w, h, grid, _p(ex) if len(ex) else None, len(ex), _p(out), _p(sc), cap)
    return out[:n].copy(), sc[:n].copy()


class StereoTracker:
    def __init__(self, w, h, levels=6, grid=50, max_iter=20, thresh=0.01, cap=4096, threads=1):
        self.h = load().orc_tracker_create(w, h, levels, grid, max_iter, C.c_float(thresh))
        if threads > 1:  # the all-cores CPU leg: pyramid levels and features in parallel (rayon)
            load().orc_tracker_set_threads(self.h, threads)
        self.cap = cap
        self.ol = (OrcFeature * cap)()
        self.orr = (OrcFeature * cap)()

    def process_frame(self, left, right):
        nl, nr = C.c_int(0), C.c_int(0)
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        load().orc_tracker_process_frame(self.h, _p(left), _p(right), C.cast(self.ol, P), self.cap, C.byref(nl),
                                         C.cast(self.orr, P), self.cap, C.byref(nr))

        def conv(arr, n):
            return [(int(f.id), float(f.x), float(f.y), tuple(float(v) for v in f.aff)) for f in arr[:n]]
        return conv(self.ol, nl.value), conv(self.orr, nr.value)

    def remove_ids(self, ids):
        ids = np.ascontiguousarray(ids, np.uint64)
        load().orc_tracker_remove_ids(self.h, _p(ids), len(ids))

    def __del__(self):
        try:
            load().orc_tracker_destroy(self.h)
        except Exception:
            pass


def camera(model: int, params, convention: int = 0, max_iterations: int = 20) -> OrcCamera:
    c = OrcCamera()
    c.model, c.convention, c.max_iterations = model, convention, max_iterations
    for i, v in enumerate(params):
        c.params[i] = float(v)
    return c


def unproject(cam: OrcCamera, px):
    """frame.rs:118-119 restated: n x 2 f32 pixels -> (n x 2 f32 undistorted, valid bool)."""
    px = np.ascontiguousarray(px, np.float32).reshape(-1, 2)
    out = np.zeros_like(px)
    valid = np.zeros(len(px), np.uint8)
    load().orc_unproject(C.byref(cam), _p(px), len(px), _p(out), _p(valid))
    return out, valid.astype(bool)


def project(cam: OrcCamera, pts):
    pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
    out = np.zeros((len(pts), 2), np.float64)
    valid = np.zeros(len(pts), np.uint8)
    load().orc_project(C.byref(cam), _p(pts), len(pts), _p(out), _p(valid))
    return out, valid.astype(bool)


def track_motion(ids_l, uv_l, ids_r, uv_r, map_ids, map_pw, T_W_B_last_kf, T_C_B2, cfg=None,
                 thr_t=0.05, thr_r=0.05) -> OrcMotionResult:
    """sliding_window.rs:490-587 + estimator.rs:195-234 restated (map ids ascending)."""
    a = [np.ascontiguousarray(ids_l, np.uint64).reshape(-1), np.ascontiguousarray(uv_l, np.float32).reshape(-1, 2),
         np.ascontiguousarray(ids_r, np.uint64).reshape(-1), np.ascontiguousarray(uv_r, np.float32).reshape(-1, 2),
         np.ascontiguousarray(map_ids, np.uint64).reshape(-1), np.ascontiguousarray(map_pw, np.float32).reshape(-1, 3),
         np.ascontiguousarray(T_W_B_last_kf, np.float64).reshape(16),
         np.ascontiguousarray(T_C_B2, np.float64).reshape(32)]
    cfg = cfg or lm_cfg(max_iterations=10)
    r = OrcMotionResult()
    load().orc_track_motion(_p(a[0]) if len(a[0]) else None, _p(a[1]) if len(a[0]) else None, len(a[0]),
                            _p(a[2]) if len(a[2]) else None, _p(a[3]) if len(a[2]) else None, len(a[2]),
                            _p(a[4]) if len(a[4]) else None, _p(a[5]) if len(a[4]) else None, len(a[4]),
                            _p(a[6]), _p(a[7]), C.byref(cfg), thr_t, thr_r, C.byref(r))
    return r


def lm_cfg(max_iterations=20, cost_tolerance=1e-6, parameter_tolerance=1e-9, huber_delta=2.0, lambda_init=1e-4,
           linear_solver=0):
    """linear_solver 0: SparseSchurComplement; 1: the SparseCholesky fallback (dense full system here)."""
    return LmCfg(max_iterations, cost_tolerance, parameter_tolerance, huber_delta, lambda_init, linear_solver)


def set_ba_threads(threads: int):
    """Threads of the BA restatement (1: the sequential reference order)."""
    load().orc_set_ba_threads(int(threads))


def ba_solve(prob, cfg=None):
    """Returns (pose7, p_W, BaResult) after the oracle's LM; prob is a synthetic.BAProblem-like."""
    cfg = cfg or lm_cfg()
    a = _problem_arrays(prob)
    pose = a[0].copy()
    pw = a[2].copy()
    res = BaResult()
    load().orc_ba_solve(pose.shape[0], _p(pose), _p(a[1]), pw.shape[0], _p(pw), len(a[3]), _p(a[3]), _p(a[4]),
                        _p(a[5]), _p(a[6]), _p(a[7]), C.byref(cfg), C.byref(res))
    return pose, pw, res


def ba_build_system(prob, lam, huber_delta=2.0):
    nfree = int((np.asarray(prob.kf_fixed) == 0).sum())
    n = 6 * nfree
    S = np.zeros((n, n))
    b = np.zeros(n)
    cost = C.c_double(0)
    a = _problem_arrays(prob)  # keep the contiguous copies alive across the call
    load().orc_ba_build_system(a[0].shape[0], _p(a[0]), _p(a[1]), a[2].shape[0], _p(a[2]), len(a[3]), _p(a[3]),
                               _p(a[4]), _p(a[5]), _p(a[6]), _p(a[7]), huber_delta, lam, _p(S), _p(b), C.byref(cost))
    return S, b, cost.value


def _problem_arrays(prob):
    return (np.ascontiguousarray(prob.pose7, np.float64), np.ascontiguousarray(prob.kf_fixed, np.uint8),
            np.ascontiguousarray(prob.p_W, np.float64), np.ascontiguousarray(prob.obs_lm, np.int32),
            np.ascontiguousarray(prob.obs_kf, np.int32), np.ascontiguousarray(prob.obs_cam, np.uint8),
            np.ascontiguousarray(prob.obs_uv, np.float64), np.ascontiguousarray(prob.T_C_B2, np.float64))


def factor_linearize(p_W, pose7, T_C_B, uv, T_B_W_fixed=None):
    r = np.zeros(2)
    J = np.zeros((2, 9))
    keep = [None if v is None else np.ascontiguousarray(v, np.float64) for v in (p_W, pose7, T_B_W_fixed, T_C_B, uv)]
    load().orc_ba_factor_linearize(*[_p(v) for v in keep], _p(r), _p(J))
    return r, J


def se3_plus(pose7, delta):
    out = np.zeros(7)
    a, d = np.ascontiguousarray(pose7, np.float64), np.ascontiguousarray(delta, np.float64)
    load().orc_se3_plus(_p(a), _p(d), _p(out))
    return out


def quat_from_matrix(R):
    """UnitQuaternion::from_matrix (w, i, j, k) of one row-major 3x3 matrix."""
    q = np.zeros(4)
    m = np.ascontiguousarray(R, np.float64)
    load().orc_quat_from_matrix(_p(m), _p(q))
    return q


def quat_from_rotation(R):
    """UnitQuaternion::from_rotation_matrix (closed form only), (w, i, j, k)."""
    q = np.zeros(4)
    m = np.ascontiguousarray(R, np.float64)
    load().orc_quat_from_rotation(_p(m), _p(q))
    return q


# ---------------- feature_tracker/ crate (secondary variant) ----------------

class FtConfig(C.Structure):
    """feature_tracker/src/feature_tracker.rs:25-38 (FeatureTrackingConfig) + the matching cost."""
    _fields_ = [("nlevels", C.c_int32), ("ratio", C.c_double), ("preprocessing_blur", C.c_int32),
                ("preprocessing_blur_sigma", C.c_float), ("detection_threshold", C.c_float),
                ("detection_min_dist", C.c_uint32), ("detection_blur", C.c_float),
                ("optical_flow_max_iter", C.c_int32), ("optical_flow_lm_lambda", C.c_float),
                ("matching_cost", C.c_int32)]


def ft_config(nlevels=5, ratio=2.0, preprocessing_blur=True, preprocessing_blur_sigma=2.0, detection_threshold=2.5,
              detection_min_dist=15, detection_blur=6.0, optical_flow_max_iter=25, optical_flow_lm_lambda=0.1,
              matching_cost=0):
    """Defaults = feature_tracker/config/config.yaml; matching_cost 0 = SSD (feature_tracker.rs:125)."""
    return FtConfig(nlevels, ratio, int(preprocessing_blur), preprocessing_blur_sigma, detection_threshold,
                    detection_min_dist, detection_blur, optical_flow_max_iter, optical_flow_lm_lambda, matching_cost)


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


def ft_level_dims(w, h, nlevels, ratio=2.0):
    d = np.zeros(2 * nlevels, np.int32)
    load().orc_ft_level_dims(w, h, nlevels, ratio, _p(d))
    return [(int(d[2 * i]), int(d[2 * i + 1])) for i in range(nlevels)]


def ft_split_pyramid(pyr, w, h, nlevels, ratio=2.0):
    out, o = [], 0
    for lw, lh in ft_level_dims(w, h, nlevels, ratio):
        out.append(pyr[o:o + lw * lh].reshape(lh, lw))
        o += lw * lh
    return out


def ft_build_pyramid(img, nlevels=5, ratio=2.0, blur=True, sigma=2.0):
    img = _f32(img)
    h, w = img.shape
    out = np.empty(int(load().orc_ft_pyramid_floats(w, h, nlevels, ratio)), np.float32)
    load().orc_ft_build_pyramid(_p(img), w, h, nlevels, ratio, int(blur), C.c_float(sigma), _p(out))
    return out


def ft_resize_triangle(img, nw, nh):
    img = _f32(img)
    h, w = img.shape
    out = np.empty((nh, nw), np.float32)
    load().orc_ft_resize_triangle(_p(img), w, h, _p(out), nw, nh)
    return out


def ft_gaussian_blur(img, sigma):
    img = _f32(img)
    out = np.empty_like(img)
    load().orc_ft_gaussian_blur(_p(img), img.shape[1], img.shape[0], C.c_float(sigma), _p(out))
    return out


def ft_fast_blur(img, sigma):
    img = _f32(img)
    out = np.empty_like(img)
    load().orc_ft_fast_blur(_p(img), img.shape[1], img.shape[0], C.c_float(sigma), _p(out))
    return out


def ft_boxes_for_gauss(sigma, n=3):
    out = np.zeros(n, np.int32)
    load().orc_ft_boxes_for_gauss(C.c_float(sigma), n, _p(out))
    return out.tolist()


def ft_bicubic(img, x, y):
    img = _f32(img)
    out = np.zeros(3, np.float32)
    ok = load().orc_ft_bicubic(_p(img), img.shape[1], img.shape[0], C.c_float(x), C.c_float(y), _p(out))
    return (out if ok else None)


def ft_exp_se2(twist):
    tw = _f32(twist)
    out = np.zeros(4, np.float32)
    load().orc_ft_exp_se2(_p(tw), _p(out))
    return out


def ft_log_se2(iso):
    a = _f32(iso)
    out = np.zeros(3, np.float32)
    load().orc_ft_log_se2(_p(a), _p(out))
    return out


def ft_patch_new(img, cx, cy, lam=0.1, cost=0):
    img = _f32(img)
    data = np.zeros(52, np.float32)
    jac = np.zeros((52, 3), np.float32)
    hinv = np.zeros((3, 3), np.float32)
    ok = load().orc_ft_patch_new(_p(img), img.shape[1], img.shape[0], C.c_float(cx), C.c_float(cy), C.c_float(lam),
                                 cost, _p(data), _p(jac), _p(hinv))
    return bool(ok), data, jac, hinv


def ft_track_points(pyr0, pyr1, w, h, xy, nlevels=5, ratio=2.0, max_iter=25, lam=0.1, cost=0):
    xy = _f32(xy).reshape(-1, 2)
    n = len(xy)
    iso = np.zeros((n, 4), np.float32)
    valid = np.zeros(n, np.uint8)
    load().orc_ft_track_points(_p(pyr0), _p(pyr1), w, h, nlevels, ratio, _p(xy) if n else None, n, max_iter,
                               C.c_float(lam), cost, _p(iso), _p(valid))
    return iso, valid.astype(bool)


def ft_shi_tomasi_score(img, blur=6.0):
    img = _f32(img)
    out = np.empty_like(img)
    load().orc_ft_shi_tomasi_score(_p(img), img.shape[1], img.shape[0], C.c_float(blur), _p(out))
    return out


def ft_suppress_non_maximum(score, radius=1, threshold=2.5, cap=1 << 20):
    score = _f32(score)
    xy = np.zeros((cap, 2), np.uint32)
    sc = np.zeros(cap, np.float32)
    n = load().orc_ft_suppress_non_maximum(_p(score), score.shape[1], score.shape[0], radius, C.c_float(threshold),
                                           _p(xy), _p(sc), cap)
    return xy[:n].copy(), sc[:n].copy()


def ft_add_points(fine, tracked_xy=None, threshold=2.5, min_dist=15, blur=6.0, cap=1 << 16):
    fine = _f32(fine)
    tr = np.zeros((0, 2), np.float32) if tracked_xy is None else _f32(tracked_xy).reshape(-1, 2)
    out = np.zeros((cap, 2), np.uint32)
    n = load().orc_ft_add_points(_p(fine), fine.shape[1], fine.shape[0], _p(tr) if len(tr) else None, len(tr),
                                 C.c_float(threshold), min_dist, C.c_float(blur), _p(out), cap)
    return out[:n].copy()


class FeatureTracker:
    """feature_tracker/src/feature_tracker.rs:51-185 restated: process_frame(img) -> (ids, xy)."""

    def __init__(self, w, h, cfg=None, cap=1 << 16):
        self.cfg = cfg or ft_config()
        self.h = load().orc_ft_create(C.byref(self.cfg), w, h)
        self.cap = cap
        self.ids = np.zeros(cap, np.uint64)
        self.xy = np.zeros((cap, 2), np.float32)

    def process_frame(self, img):
        img = _f32(img)
        n = C.c_int(0)
        rc = load().orc_ft_process_frame(self.h, _p(img), _p(self.ids), _p(self.xy), self.cap, C.byref(n))
        assert rc == 0, rc
        return self.ids[:n.value].copy(), self.xy[:n.value].copy()

    def __del__(self):
        try:
            load().orc_ft_destroy(self.h)
        except Exception:
            pass
