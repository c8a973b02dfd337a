"""Host-side mirror of the reference's bundle-adjustment API over the C ABI.

* ``BundleAdjuster`` -- the solver handle (rsvio_ba_*): replaces the apex-solver
  ``LevenbergMarquardt::optimize`` call of ``SlidingWindow::optimize``
  (src/estimator/sliding_window.rs:325) with the HIP Schur-complement LM; optional landmark
  sharding over ranks with an RCCL all-reduce (``attach_comm``).
* ``SlidingWindow`` -- mirrors ``SlidingWindow`` (sliding_window.rs:21-486): keyframe FIFO,
  problem assembly (stereo-landmark rule, depth-2 initialisation, KF_0 fixed), guards,
  rollback on failure, map points kept as f32.
"""
from __future__ import annotations

import ctypes as C
import math
from collections import deque
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, ptr


SOLVER_SCHUR, SOLVER_CHOLESKY = 0, 1        # LinearSolverType::{SparseSchurComplement, SparseCholesky}
LINEAR_SOLVE_FAILED = -3                    # RSVIO_LM_LINEAR_SOLVE_FAILED


def lm_cfg(max_iterations=20, cost_tolerance=1e-6, parameter_tolerance=1e-9, huber_delta=2.0, lambda_init=1e-4,
           linear_solver=SOLVER_SCHUR):
    """sliding_window.rs:126-135 (max 20 iterations, cost tol 1e-6, parameter tol 1e-9) + Huber(2.0);
    linear_solver SOLVER_CHOLESKY is the fallback configuration of :334-341 (same tolerances)."""
    return _lib.LmCfg(max_iterations, cost_tolerance, parameter_tolerance, huber_delta, lambda_init, linear_solver)


_DEFAULT_CFG = lm_cfg()


def fallback_cfg(cfg=None):
    """The SparseCholesky configuration the reference retries with (sliding_window.rs:333-341)."""
    c = cfg or lm_cfg()
    return lm_cfg(c.max_iterations, c.cost_tolerance, c.parameter_tolerance, c.huber_delta, c.lambda_init,
                  SOLVER_CHOLESKY)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _all_min(x: float) -> float:
    import torch
    import torch.distributed as dist
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def attach_agreed(ba, world: int, rank: int, collective: str = "auto", rccl_ok: bool = True, log=None) -> str:
    """Every rank of the torch.distributed control group takes the SAME branch: the RCCL
    communicator first (the fallback; only when rccl_ok -- RCCL refuses two ranks on one GPU),
    then the P2P one-shot all-reduce, kept only if EVERY rank exported a buffer and passed the
    self-test (which also fails on every rank when their exchange settings differ).  Otherwise the
    ranks that attached detach, and all go on over RCCL -- or, without it, all raise RuntimeError.
    Returns "p2p" or "rccl".  `ba` needs p2p_export / attach_p2p / detach_p2p / attach_comm /
    rccl_unique_id (BundleAdjuster's)."""
    import torch.distributed as dist
    say = log or (lambda m: None)
    have_rccl = False
    if collective in ("auto", "rccl") and rccl_ok:
        obj = [ba.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ba.attach_comm(world, rank, obj[0])
        have_rccl = True
    if collective == "rccl":
        if not have_rccl:
            raise RuntimeError("RCCL requested but not available")
        return "rccl"
    mine = None
    try:
        mine = ba.p2p_export(world)
    except Exception as e:  # noqa: BLE001 - reported, then agreed on below
        say(f"rank {rank}: p2p export failed: {e}")
    handles = [None] * world
    dist.all_gather_object(handles, mine)
    ok = all(h is not None for h in handles)
    if ok:
        try:
            ba.attach_p2p(world, rank, handles)
        except Exception as e:  # noqa: BLE001
            say(f"rank {rank}: p2p attach failed: {e}")
            ok = False
    all_ok = world == 1 and ok or world > 1 and _all_min(1.0 if ok else 0.0) > 0.5
    if all_ok:
        return "p2p"
    if ok:
        ba.detach_p2p()
    if not have_rccl:
        raise RuntimeError("P2P exchange unavailable on some rank and no RCCL communicator attached")
    return "rccl"


class BundleAdjuster:
    """One device-resident BA solver (one HIP stream)."""

    def __init__(self, max_keyframes=21, max_landmarks=1 << 16, max_observations=1 << 20, device=0):
        lib = _lib.load()
        p = _lib.BaParams(max_keyframes, max_landmarks, max_observations, device)
        h = C.c_void_p()
        check(lib.rsvio_ba_create(C.byref(p), C.byref(h)))
        self._h = h
        self.n_kf = self.n_lm = 0

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().rsvio_ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def attach_comm(self, nranks: int, rank: int, unique_id: bytes):
        buf = (C.c_uint8 * len(unique_id)).from_buffer_copy(unique_id)
        check(_lib.load().rsvio_ba_attach_comm(self._h, nranks, rank, buf))

    def p2p_export(self, nranks: int) -> bytes:
        """IPC handle (64 bytes) of this handle's P2P exchange buffer (rsvio_ba_p2p_export)."""
        buf = (C.c_uint8 * 64)()
        check(_lib.load().rsvio_ba_p2p_export(self._h, nranks, buf, 64))
        return bytes(buf)

    def attach_p2p(self, nranks: int, rank: int, handles) -> None:
        """Switch the sharded exchanges to the P2P one-shot all-reduce (self-tested; raises
        RsvioError and keeps the previous collective on failure)."""
        blob = b"".join(handles)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        check(_lib.load().rsvio_ba_attach_p2p(self._h, nranks, rank, buf))

    def p2p_latency_us(self, reps: int = 200, n: int = 4) -> float:
        """Average device microseconds of one P2P exchange of n doubles (collective: every
        attached rank calls it with the same arguments)."""
        us = C.c_double(0.0)
        check(_lib.load().rsvio_ba_p2p_latency(self._h, reps, n, C.byref(us)))
        return us.value

    def p2p_level(self) -> int:
        """The exchange form of the current problem's iterations (rsvio_ba_p2p_level): -1 not
        P2P-sharded, else the fold level taken (3 only while K6's grid fits the stream's CUs)."""
        v = C.c_int32(0)
        check(_lib.load().rsvio_ba_p2p_level(self._h, C.byref(v)))
        return v.value

    def detach_p2p(self) -> None:
        check(_lib.load().rsvio_ba_detach_p2p(self._h))

    def attach_sharded(self, world: int, rank: int, collective: str = "auto", rccl_ok: bool = True,
                       log=None) -> str:
        """Attach this rank's landmark shard (sliding_window.rs:325's solve, split over ranks) to
        its peers over the initialised torch.distributed control group; see attach_agreed."""
        return attach_agreed(self, world, rank, collective, rccl_ok, log)

    @staticmethod
    def rccl_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        check(_lib.load().rsvio_rccl_unique_id(buf, 128))
        return bytes(buf)

    @staticmethod
    def _marshal(pose7, kf_fixed, p_W, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2):
        """The C arguments of rsvio_ba_set_problem: contiguous arrays of the C types, their sizes
        and pointers."""
        keep = [_c(pose7, np.float64), _c(kf_fixed, np.uint8), _c(p_W, np.float64).reshape(-1, 3),
                _c(obs_lm, np.int32), _c(obs_kf, np.int32), _c(obs_cam, np.uint8),
                _c(obs_uv, np.float64).reshape(-1, 2), _c(T_C_B2, np.float64).reshape(2, 16)]
        pose, fixed, pw, lm, kf, cam, uv, tcb = keep
        args = (pose.shape[0], ptr(pose), ptr(fixed), pw.shape[0], ptr(pw), len(lm), ptr(lm), ptr(kf), ptr(cam),
                ptr(uv), ptr(tcb))
        return keep, args

    def _set(self, keep, args):
        self._keep = keep
        self.n_kf, self.n_lm = args[0], args[3]
        check(_lib.load().rsvio_ba_set_problem(self._h, *args))

    def set_problem(self, pose7, kf_fixed, p_W, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2):
        self._set(*self._marshal(pose7, kf_fixed, p_W, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2))

    _FIELDS = ("pose7", "kf_fixed", "p_W", "obs_lm", "obs_kf", "obs_cam", "obs_uv", "T_C_B2")

    def set_problem_from(self, prob):
        """set_problem with the fields of a problem object.  Its marshalled arguments are kept on
        the object for as long as its fields are the same array objects AND marshalling used them
        as they are (the C types, contiguous): in-place edits are then seen and the pointers stay
        valid -- a Rust caller hands its slices over as they are, while ctypes pointer extraction
        costs ~2 us per array, a fifth of the C call.  A field that had to be converted (another
        dtype, non-contiguous) is a copy, so such a problem is re-marshalled on every call."""
        src = tuple(getattr(prob, f) for f in self._FIELDS)
        m = prob.__dict__.get("_rsvio_marshal")
        if m is None or any(a is not b for a, b in zip(m[0], src)):
            keep, args = self._marshal(*src)
            # a reshape of the source is a view: in-place edits of the source reach it
            if not all(k is s or (k.base is not None and (k.base is s or k.base is getattr(s, "base", None)))
                       for k, s in zip(keep, src)):
                self._set(keep, args)
                return
            m = (src, (keep, args))
            object.__setattr__(prob, "_rsvio_marshal", m)
        self._set(*m[1])

    def run(self, cfg=None) -> _lib.BaResult:
        res = _lib.BaResult()
        check(_lib.load().rsvio_ba_run(self._h, C.byref(cfg or lm_cfg()), C.byref(res)))
        return res

    def set_stream(self, stream_ptr) -> None:
        """Enqueue on a caller-owned HIP stream (rsvio.cu_stream), None = the handle's own."""
        check(_lib.load().rsvio_ba_set_stream(self._h, stream_ptr))

    def run_async(self, cfg=None) -> None:
        """Enqueue the solve and return (rsvio_ba_run_async); wait() completes it."""
        self._cfg = cfg or _DEFAULT_CFG  # kept alive until wait() (the C side only reads it)
        check(_lib.load().rsvio_ba_run_async(self._h, C.byref(self._cfg)))

    def wait(self) -> _lib.BaResult:
        res = _lib.BaResult()
        check(_lib.load().rsvio_ba_wait(self._h, C.byref(res)))
        return res

    def state(self, out=None):
        """The optimised state (rsvio_ba_get_state): poses (n_kf x 7) and points (n_lm x 3), into
        `out` = (pose, p_W) f64 C-contiguous arrays of those shapes when given (reused buffers)."""
        if out is None:
            pose, pw = np.empty((self.n_kf, 7)), np.empty((self.n_lm, 3))
        else:
            pose, pw = out
            if pose.shape != (self.n_kf, 7) or pw.shape != (self.n_lm, 3) or pose.dtype != np.float64 \
                    or pw.dtype != np.float64:
                raise ValueError("state(out=...): arrays of shape (n_kf, 7) and (n_lm, 3), float64")
        check(_lib.load().rsvio_ba_get_state(self._h, ptr(pose), ptr(pw)))
        return pose, pw

    def build_system(self, lam, huber_delta=2.0):
        nfree = int((self._keep[1] == 0).sum())
        S = np.zeros((6 * nfree, 6 * nfree))
        b = np.zeros(6 * nfree)
        cost = C.c_double()
        check(_lib.load().rsvio_ba_build_system(self._h, lam, huber_delta, ptr(S), ptr(b), C.byref(cost)))
        return S, b, cost.value

    def camera_step(self, lam, huber_delta=2.0):
        """Diagnostic (rsvio_dbg_ba_camera_step): the reduced system at lam and its dense camera
        solve (K4c + K5) on the current state -> dc (6 n_free)."""
        lib = _lib.load()
        fn = lib.rsvio_dbg_ba_camera_step
        fn.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_void_p]
        fn.restype = C.c_int
        nfree = int((self._keep[1] == 0).sum())
        dc = np.zeros(6 * nfree)
        check(fn(self._h, lam, huber_delta, ptr(dc)))
        return dc

    def solve(self, pose7, kf_fixed, p_W, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2, cfg=None):
        """rsvio_ba_solve: returns (pose7, p_W, result); inputs are not modified."""
        pose = _c(pose7, np.float64).copy()
        pw = _c(p_W, np.float64).reshape(-1, 3).copy()
        lm, kf, cam = _c(obs_lm, np.int32), _c(obs_kf, np.int32), _c(obs_cam, np.uint8)
        uv, tcb, fixed = _c(obs_uv, np.float64).reshape(-1, 2), _c(T_C_B2, np.float64), _c(kf_fixed, np.uint8)
        res = _lib.BaResult()
        check(_lib.load().rsvio_ba_solve(self._h, pose.shape[0], ptr(pose), ptr(fixed), pw.shape[0], ptr(pw), len(lm),
                                         ptr(lm), ptr(kf), ptr(cam), ptr(uv), ptr(tcb), C.byref(cfg or lm_cfg()),
                                         C.byref(res)))
        self.n_kf, self.n_lm = pose.shape[0], pw.shape[0]
        return pose, pw, res


# --------------------------------------------------------------------------------------------
# SlidingWindow mirror
# --------------------------------------------------------------------------------------------
@dataclass
class Frame:
    """The fields of estimator::Frame (src/estimator/frame.rs:20-47) that the BA reads."""
    frame_id: int
    T_W_B: np.ndarray = field(default_factory=lambda: np.eye(4))
    T_B_Cl: np.ndarray = field(default_factory=lambda: np.eye(4))
    T_B_Cr: np.ndarray = field(default_factory=lambda: np.eye(4))
    is_keyframe: bool = True
    # per camera, in feature order: (ids, undistorted uv) arrays or [(feature_id, (x, y))]
    left_features: list = field(default_factory=list)
    right_features: list = field(default_factory=list)


def _feature_lists(feats):
    """(ids u64, uv f32 n x 2) C-contiguous from a frame's features: (ids, uv) arrays or
    (id, (x, y)) pairs (Feature::undistorted_coord is f32, frame.rs:118-119)."""
    if isinstance(feats, tuple) and len(feats) == 2 and isinstance(feats[0], np.ndarray):
        ids, uv = feats
        if ids.dtype == np.int64 and uv.dtype == np.float32 and uv.ndim == 2:  # the Estimator's lists
            return ids.view(np.uint64), uv
    else:
        ids = [fid for fid, _ in feats]
        uv = [xy for _, xy in feats]
    ids = np.ascontiguousarray(np.asarray(ids, np.int64).reshape(-1)).view(np.uint64)
    return ids, np.ascontiguousarray(np.asarray(uv, np.float32).reshape(-1, 2))


def quat_from_matrix(R) -> np.ndarray:
    """UnitQuaternion::from_matrix (sliding_window.rs:221,511): nalgebra's iterative
    Rotation3::from_matrix_eps then from_rotation_matrix, (w, i, j, k); n x 3 x 3 -> n x 4
    (rsvio_quat_from_matrix, host code of the library)."""
    R = np.ascontiguousarray(R, np.float64).reshape(-1, 9)
    q = np.zeros((len(R), 4))
    check(_lib.load().rsvio_quat_from_matrix(ptr(R), len(R), ptr(q)))
    return q


def se3_matrix(p7) -> np.ndarray:
    """apex SE3::from([t; w, i, j, k]).matrix(): the quaternion normalised, then nalgebra's
    to_rotation_matrix (the same formula as the kernels' pose_from7, se3.hpp)."""
    w, x, y, z = (float(v) for v in p7[3:7])
    n = 1.0 / math.sqrt(w * w + x * x + y * y + z * z)
    w, x, y, z = w * n, x * n, y * n, z * n
    ww, xx, yy, zz = w * w, x * x, y * y, z * z
    xy, wz, wy = x * y * 2.0, w * z * 2.0, w * y * 2.0
    xz, yz, wx = x * z * 2.0, y * z * 2.0, w * x * 2.0
    T = np.eye(4)
    T[:3, :3] = [[ww + xx - yy - zz, xy - wz, wy + xz],
                 [wz + xy, ww - xx + yy - zz, yz - wx],
                 [xz - wy, wx + yz, ww - xx - yy + zz]]
    T[:3, 3] = p7[:3]
    return T


class BundleBatch:
    """Batched mode (rsvio_ba_batch_*): the problems of several BundleAdjuster handles solved by
    one launch chain; run() returns one BaResult per window, state() is read on each handle."""

    def __init__(self, adjusters):
        self.adjusters = list(adjusters)
        arr = (C.c_void_p * len(self.adjusters))(*[a._h.value for a in self.adjusters])
        h = C.c_void_p()
        check(_lib.load().rsvio_ba_batch_create(arr, len(self.adjusters), C.byref(h)))
        self._h = h

    def run(self, cfg=None):
        res = (_lib.BaResult * len(self.adjusters))()
        check(_lib.load().rsvio_ba_batch_run(self._h, C.byref(cfg or lm_cfg()), res))
        return list(res)

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().rsvio_ba_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SlidingWindow:
    """Keyframe FIFO + BA problem assembly (sliding_window.rs:21-486) over the GPU solver."""

    def __init__(self, max_frames: int, device: int = 0, solver: BundleAdjuster | None = None):
        self.max_frames = max_frames
        self.keyframes: deque[Frame] = deque()
        # map_points (feature id -> [f32; 3], sliding_window.rs:466-475) as ascending ids + an f32
        # n x 3 array: what the next problem build and the PnP map upload read, with no per-point
        # Python work (map_points is the dict view of the same map)
        self.map_ids = np.zeros(0, np.int64)
        self.map_pw = np.zeros((0, 3), np.float32)
        self.map_version = 0                           # bumped whenever the map is replaced
        self.fallbacks = 0                             # SparseCholesky retries (diagnostic)
        self.solver = solver or BundleAdjuster(max_keyframes=max(max_frames, 2), device=device)
        self.last_result = None
        self._pending = None                           # landmark ids of a solve in flight (optimize_async)

    @property
    def map_points(self) -> dict:
        return dict(zip(self.map_ids.tolist(), self.map_pw))

    @map_points.setter
    def map_points(self, mp: dict):
        ids = np.fromiter(mp.keys(), np.int64, len(mp))
        pw = (np.stack([np.asarray(v, np.float32) for v in mp.values()]) if len(mp)
              else np.zeros((0, 3), np.float32))
        srt = np.argsort(ids, kind="stable")
        self.map_ids, self.map_pw = ids[srt], pw[srt].reshape(-1, 3)

    def add_frame(self, frame: Frame) -> bool:
        if not frame.is_keyframe:
            return False
        if len(self.keyframes) >= self.max_frames:
            self.keyframes.popleft()
        self.keyframes.append(frame)
        return True

    def __len__(self):
        return len(self.keyframes)

    def is_full(self) -> bool:
        return len(self.keyframes) >= self.max_frames

    def get_keyframe_poses(self):
        return [f.T_W_B.copy() for f in self.keyframes]

    def build_problem(self):
        """sliding_window.rs:174-300 in canonical order (frames, left then right, feature order):
        landmarks = ids seen at least once left and once right in the window, indexed by first
        appearance; initial point from map_points (f32) or the depth-2.0 ray of its first
        observation (sliding_window.rs:248-272).  Assembled by the library's host code
        (rsvio_window_problem, csrc/window.hip) in one call."""
        kfs = list(self.keyframes)
        n = len(kfs)
        lists = [_feature_lists(feats) for f in kfs for feats in (f.left_features, f.right_features)]
        ids_a = np.concatenate([i for i, _ in lists])
        uv_a = np.concatenate([u for _, u in lists])
        n_feat = np.array([len(i) for i, _ in lists], np.int32)
        tot = len(ids_a)
        T_W_B = np.ascontiguousarray(np.stack([f.T_W_B for f in kfs]), np.float64)
        T_B_C2 = np.ascontiguousarray(np.stack([kfs[0].T_B_Cl, kfs[0].T_B_Cr]), np.float64)
        map_ids = self.map_ids.view(np.uint64) if self.map_ids.dtype == np.int64 else self.map_ids
        pose7, fixed, tcb = np.empty((n, 7)), np.empty(n, np.uint8), np.empty((2, 16))
        lm_ids, p_init = np.empty(max(tot, 1), np.uint64), np.empty((max(tot, 1), 3))
        obs_lm, obs_kf = np.empty(max(tot, 1), np.int32), np.empty(max(tot, 1), np.int32)
        obs_cam, obs_uv = np.empty(max(tot, 1), np.uint8), np.empty((max(tot, 1), 2))
        n_lm, n_obs = C.c_int32(0), C.c_int32(0)
        check(_lib.load().rsvio_window_problem(
            n, ptr(T_W_B), ptr(T_B_C2), ptr(ids_a) if tot else None, ptr(uv_a) if tot else None, ptr(n_feat), ptr(map_ids) if len(map_ids) else None,
            ptr(self.map_pw) if len(map_ids) else None, len(map_ids), ptr(pose7), ptr(fixed), ptr(tcb),
            max(tot, 1), ptr(lm_ids), ptr(p_init), C.byref(n_lm), max(tot, 1), ptr(obs_lm), ptr(obs_kf),
            ptr(obs_cam), ptr(obs_uv), C.byref(n_obs)))
        L, O = n_lm.value, n_obs.value
        return (pose7, fixed, p_init[:L], obs_lm[:O], obs_kf[:O], obs_cam[:O], obs_uv[:O], tcb,
                lm_ids[:L].view(np.int64))

    def optimize(self, cfg=None) -> bool:
        """Returns Ok(true)/Ok(false) as a bool; raises RuntimeError for a non-full window (:137-149)."""
        if not self.keyframes:
            raise RuntimeError("Window is empty")
        if len(self.keyframes) < self.max_frames:
            raise RuntimeError("Need more keyframes")
        pose7, fixed, p_init, lm, kf, cam, uv, tcb, ids = self.build_problem()
        num_vars = len(self.keyframes) + len(p_init)  # KF_0 is in initial_values too (:217-226)
        if len(lm) < 6 or len(lm) < num_vars:
            self.last_result = None
            return False
        pose, pw, res = self.solver.solve(pose7, fixed, p_init, lm, kf, cam, uv, tcb, cfg)
        if res.status == LINEAR_SOLVE_FAILED:
            # sliding_window.rs:326-353: a singular Schur solve is retried from the same initial
            # values with SparseCholesky; if that fails too the window reverts (_apply: Ok(false))
            self.fallbacks += 1
            pose, pw, res = self.solver.solve(pose7, fixed, p_init, lm, kf, cam, uv, tcb, fallback_cfg(cfg))
        return self._apply(ids, pose, pw, res)

    def _apply(self, ids, pose, pw, res) -> bool:
        """process_optimization_result (sliding_window.rs:418-486), by the library's host code
        (rsvio_window_apply): map points as f32 by ascending id, T_W_B = inverse(SE3(pose7))."""
        self.last_result = res
        if res.status <= 0:
            return False  # revert: nothing was modified
        n, m = len(self.keyframes), len(ids)
        pose = np.ascontiguousarray(pose, np.float64)
        pw = np.ascontiguousarray(pw, np.float64).reshape(-1, 3)
        ids = np.ascontiguousarray(ids, np.int64)
        T_W_B = np.empty((n, 4, 4))
        map_ids, map_pw = np.empty(m, np.int64), np.empty((m, 3), np.float32)
        check(_lib.load().rsvio_window_apply(n, ptr(pose), m, ptr(ids) if m else None, ptr(pw) if m else None,
                                             ptr(T_W_B), ptr(map_ids) if m else None, ptr(map_pw) if m else None))
        self.map_ids, self.map_pw = map_ids, map_pw
        self.map_version += 1
        for f, T in zip(self.keyframes, T_W_B):
            f.T_W_B = T
        return True

    def optimize_async(self, cfg=None):
        """optimize() in two halves: assemble the problem, enqueue the solve on the device
        (rsvio_ba_run_async) and return None; finish() waits and applies the result.  The window
        must not be read or changed in between (the Estimator calls finish() before its next use
        of the window, so the result is the same as optimize()'s).  Returns optimize()'s bool when
        nothing was enqueued (guards, or a solver without an asynchronous path)."""
        self.finish()
        if not self.keyframes:
            raise RuntimeError("Window is empty")
        if len(self.keyframes) < self.max_frames:
            raise RuntimeError("Need more keyframes")
        if not hasattr(self.solver, "run_async"):
            return self.optimize(cfg)
        pose7, fixed, p_init, lm, kf, cam, uv, tcb, ids = self.build_problem()
        num_vars = len(self.keyframes) + len(p_init)
        if len(lm) < 6 or len(lm) < num_vars:
            self.last_result = None
            return False
        self.solver.set_problem(pose7, fixed, p_init, lm, kf, cam, uv, tcb)
        self.solver.run_async(cfg)
        self._pending = (ids, cfg)
        return None

    def finish(self):
        """Complete a solve started by optimize_async (no-op otherwise); returns its bool."""
        if self._pending is None:
            return None
        (ids, cfg), self._pending = self._pending, None
        res = self.solver.wait()
        if res.status == LINEAR_SOLVE_FAILED:  # the SparseCholesky retry (:326-353), same problem
            self.fallbacks += 1
            res = self.solver.run(fallback_cfg(cfg))
        pose, pw = self.solver.state()
        return self._apply(ids, pose, pw, res)
