"""Seeded synthetic inputs shaped like BASELINE.json's configurations.

No EuRoC / TUM-VI data exists offline, so every workload is procedural:

* ``stereo_sequence`` -- config 2: 752x480 u8 stereo frames.  A continuous texture of 6000
  Gaussian blobs (amplitude U(-60, 60), sigma U(1.5, 8)) around 128 plus 2*N(0,1) pixel noise;
  the right image sees the texture shifted by the disparity d(y) = 4 + 8*y/480; frame t+1
  is frame t moved by (1.7, -0.9) px and rotated by 0.2 degrees.  (SURVEY.md 8d sketched 400
  blobs / sigma 2-12 / noise 8 / d = 8..32 px: with that texture the reference algorithm keeps
  < 50 % of its tracks and a 3-level pyramid cannot reach 32 px of disparity, so most of the
  measured work would be early exits.  The denser texture keeps ~98 % of temporal tracks.)
* ``track_features`` -- 300 feature positions (FAST-9 corners at t=20, >= 20 px apart, inside
  [20, 732) x [20, 460), topped up with seeded uniform points) for config 2.
* ``ba_problem`` -- config 3: 10 keyframes (KF_0 fixed), EuRoC extrinsics, 2000 landmarks,
  each seen by both cameras in 6 consecutive keyframes (24,000 observations), noisy
  observations and perturbed initial values.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# config/euroc_vio.yaml:21-30 (T_B_Cl, T_B_Cr) and :10-16 (intrinsics)
T_B_CL = np.array([
    [0.0148655429818, -0.999880929698, 0.00414029679422, -0.0216401454975],
    [0.999557249008, 0.0149672133247, 0.025715529948, -0.064676986768],
    [-0.0257744366974, 0.00375618835797, 0.999660727178, 0.00981073058949],
    [0.0, 0.0, 0.0, 1.0]])
T_B_CR = np.array([
    [0.0125552670891, -0.999755099723, 0.0182237714554, -0.0198435579556],
    [0.999598781151, 0.0130119051815, 0.0251588363115, 0.0453689425024],
    [-0.0253898008918, 0.0179005838253, 0.999517347078, 0.00786212447038],
    [0.0, 0.0, 0.0, 1.0]])
FX_LEFT = 458.654


# ----------------------------------------------------------------------------------------
# Tracker workload (config 2)
# ----------------------------------------------------------------------------------------
@dataclass
class Texture:
    mu: np.ndarray      # (K, 2) blob centres in texture coordinates
    amp: np.ndarray     # (K,)
    sigma: np.ndarray   # (K,)


def make_texture(w: int, h: int, n_blobs: int = 6000, seed: int = 20260320) -> Texture:
    rng = np.random.default_rng(seed)
    margin = 80.0
    mu = np.stack([rng.uniform(-margin, w + margin, n_blobs), rng.uniform(-margin, h + margin, n_blobs)], 1)
    return Texture(mu=mu, amp=rng.uniform(-60, 60, n_blobs), sigma=rng.uniform(1.5, 8, n_blobs))


def _render(tex: Texture, w: int, h: int, t: int, right: bool, noise: np.ndarray) -> np.ndarray:
    """I(x) = 128 + sum_k A_k exp(-|warp(x) - mu_k|^2 / 2 sigma_k^2) + noise, clamped to u8.

    warp(x) maps pixel x of frame t (left or right camera) to texture coordinates; each blob is
    evaluated only in a pixel window around its forward-mapped centre.
    """
    ang = math.radians(0.2) * t
    ca, sa = math.cos(ang), math.sin(ang)
    sx, sy = 1.7 * t, -0.9 * t
    cx, cy = w / 2.0, h / 2.0
    acc = np.full((h, w), 128.0)
    for (mx, my), a, sg in zip(tex.mu, tex.amp, tex.sigma):
        # forward map of the blob centre: p = R(ang) (mu - c) + c + s  (then - d(y) on the right)
        px_ = ca * (mx - cx) - sa * (my - cy) + cx + sx
        py_ = sa * (mx - cx) + ca * (my - cy) + cy + sy
        if right:
            px_ -= disparity(py_)
        r = 4.0 * sg + 3.0
        x0, x1 = max(0, int(px_ - r)), min(w, int(px_ + r) + 2)
        y0, y1 = max(0, int(py_ - r)), min(h, int(py_ + r) + 2)
        if x0 >= x1 or y0 >= y1:
            continue
        ys, xs = np.mgrid[y0:y1, x0:x1].astype(np.float64)
        x = xs - cx - sx
        y = ys - cy - sy
        if right:
            x = x + disparity(ys)
        u = ca * x + sa * y + cx
        v = -sa * x + ca * y + cy
        du = u - mx
        dv = v - my
        acc[y0:y1, x0:x1] += a * np.exp(-(du * du + dv * dv) / (2.0 * sg * sg))
    acc += noise
    return np.clip(np.rint(acc), 0, 255).astype(np.uint8)


def stereo_sequence(n_frames: int, w: int = 752, h: int = 480, seed: int = 20260320):
    """Yield (left, right) u8 frames of config 2."""
    tex = make_texture(w, h, seed=seed)
    rng = np.random.default_rng(seed + 1)
    for t in range(n_frames):
        left = _render(tex, w, h, t, False, 2.0 * rng.standard_normal((h, w)))
        right = _render(tex, w, h, t, True, 2.0 * rng.standard_normal((h, w)))
        yield left, right


def fast9_mask(img: np.ndarray, t: int) -> np.ndarray:
    """Vectorised FAST-9 corner test (contiguous arc of >= 9 of 16 brighter/darker by > t)."""
    im = img.astype(np.int16)
    h, w = im.shape
    off = [(0, -3), (1, -3), (2, -2), (3, -1), (3, 0), (3, 1), (2, 2), (1, 3), (0, 3), (-1, 3),
           (-2, 2), (-3, 1), (-3, 0), (-3, -1), (-2, -2), (-1, -3)]
    c = im[3:h - 3, 3:w - 3]
    ring = np.stack([im[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in off])
    out = np.zeros((h, w), bool)
    for sign in (1, -1):
        ok = (sign * (ring - c[None])) > t
        ok2 = np.concatenate([ok, ok[:8]], 0)
        run = np.zeros_like(c, dtype=np.int16)
        best = np.zeros_like(c, dtype=np.int16)
        for k in range(ok2.shape[0]):
            run = np.where(ok2[k], run + 1, 0)
            best = np.maximum(best, run)
        out[3:h - 3, 3:w - 3] |= best >= 9
    return out


def track_features(img: np.ndarray, n: int = 300, seed: int = 20260320, spacing: float = 20.0) -> np.ndarray:
    """Config-2 feature positions as an (n, 6) Affine2 array {1, 0, 0, 1, x, y}."""
    h, w = img.shape
    mask = fast9_mask(img, 20)
    ys, xs = np.nonzero(mask)
    pts: list[tuple[float, float]] = []
    for x, y in zip(xs, ys):
        if not (20 <= x < w - 20 and 20 <= y < h - 20):
            continue
        if all((x - px) ** 2 + (y - py) ** 2 >= spacing ** 2 for px, py in pts[-64:]) and \
                all((x - px) ** 2 + (y - py) ** 2 >= spacing ** 2 for px, py in pts):
            pts.append((float(x), float(y)))
            if len(pts) == n:
                break
    rng = np.random.default_rng(seed + 7)
    while len(pts) < n:
        pts.append((float(rng.uniform(20, w - 20)), float(rng.uniform(20, h - 20))))
    aff = np.zeros((n, 6), np.float32)
    aff[:, 0] = 1.0
    aff[:, 3] = 1.0
    aff[:, 4:6] = np.asarray(pts, np.float32)
    return aff


def disparity(y):
    return 4.0 + 8.0 * y / 480.0


def stereo_shift(aff: np.ndarray) -> np.ndarray:
    """Where a left-image feature appears in the right image (x - d(y))."""
    out = aff.copy()
    out[:, 4] = aff[:, 4] - disparity(aff[:, 5])
    return out


# ----------------------------------------------------------------------------------------
# Bundle-adjustment workload (config 3)
# ----------------------------------------------------------------------------------------
def rot_z(a: float) -> np.ndarray:
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def quat_from_rot(R: np.ndarray) -> np.ndarray:
    """nalgebra UnitQuaternion::from_rotation_matrix branch structure; returns (w, x, y, z)."""
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0.0:
        d = math.sqrt(tr + 1.0) * 2.0
        return np.array([0.25 * d, (R[2, 1] - R[1, 2]) / d, (R[0, 2] - R[2, 0]) / d, (R[1, 0] - R[0, 1]) / d])
    if R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        d = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2.0
        return np.array([(R[2, 1] - R[1, 2]) / d, 0.25 * d, (R[0, 1] + R[1, 0]) / d, (R[0, 2] + R[2, 0]) / d])
    if R[1, 1] > R[2, 2]:
        d = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2.0
        return np.array([(R[0, 2] - R[2, 0]) / d, (R[0, 1] + R[1, 0]) / d, 0.25 * d, (R[1, 2] + R[2, 1]) / d])
    d = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2.0
    return np.array([(R[1, 0] - R[0, 1]) / d, (R[0, 2] + R[2, 0]) / d, (R[1, 2] + R[2, 1]) / d, 0.25 * d])


def rot_from_quat(q: np.ndarray) -> np.ndarray:
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([
        [w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (w * y + x * z)],
        [2 * (w * z + x * y), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (w * x + y * z), w * w - x * x - y * y + z * z]])


def pose7_from_T_W_B(T_W_B: np.ndarray) -> np.ndarray:
    """sliding_window.rs:218-224: T_B_W = inv(T_W_B) -> [t_B_W, q_B_W (w, x, y, z)]."""
    R = T_W_B[:3, :3].T
    t = -R @ T_W_B[:3, 3]
    return np.concatenate([t, quat_from_rot(R)])


def small_rot(rng, sigma_rad: float) -> np.ndarray:
    v = rng.normal(0.0, sigma_rad, 3)
    th = np.linalg.norm(v)
    if th < 1e-15:
        return np.eye(3)
    k = v / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


@dataclass
class BAProblem:
    pose7: np.ndarray       # (n_kf, 7) initial T_B_W
    kf_fixed: np.ndarray    # (n_kf,) u8
    p_W: np.ndarray         # (n_lm, 3) initial
    obs_lm: np.ndarray      # (n_obs,) i32
    obs_kf: np.ndarray      # (n_obs,) i32
    obs_cam: np.ndarray     # (n_obs,) u8
    obs_uv: np.ndarray      # (n_obs, 2) f64 normalised coordinates
    T_C_B2: np.ndarray      # (2, 16) row-major T_Cl_B, T_Cr_B
    true_pose7: np.ndarray
    true_p_W: np.ndarray

    @property
    def n_kf(self):
        return self.pose7.shape[0]

    @property
    def n_lm(self):
        return self.p_W.shape[0]

    @property
    def n_obs(self):
        return self.obs_lm.shape[0]

    def shard(self, rank: int, world: int) -> "BAProblem":
        """Contiguous landmark range of this rank (observations follow their landmark)."""
        lo = self.n_lm * rank // world
        hi = self.n_lm * (rank + 1) // world
        sel = (self.obs_lm >= lo) & (self.obs_lm < hi)
        return BAProblem(self.pose7.copy(), self.kf_fixed.copy(), self.p_W[lo:hi].copy(),
                         (self.obs_lm[sel] - lo).astype(np.int32), self.obs_kf[sel].copy(),
                         self.obs_cam[sel].copy(), self.obs_uv[sel].copy(), self.T_C_B2.copy(),
                         self.true_pose7.copy(), self.true_p_W[lo:hi].copy())


def ba_problem(n_kf: int = 10, n_lm: int = 2000, kf_per_lm: int = 6, seed: int = 7,
               noise_px: float = 0.5, init_seed: int = 11, pose_noise=(0.02, math.radians(0.5)),
               depth_noise: float = 0.05) -> BAProblem:
    """Config 3 (and, with other arguments, config 5's shape).  The observations are f32 values
    widened to f64, as the reference's are: SlidingWindow::optimize builds each factor from a
    feature's f32 undistorted_coord cast to f64 (sliding_window.rs:276)."""
    rng = np.random.default_rng(seed)
    T_W_B = []
    for k in range(n_kf):
        T = np.eye(4)
        T[:3, :3] = rot_z(0.01 * k)
        T[:3, 3] = [0.08 * k, 0.01 * math.sin(k), 0.0]
        T_W_B.append(T)
    T_C_B = [np.linalg.inv(T_B_CL), np.linalg.inv(T_B_CR)]
    # landmarks in cam0 of KF_0: U([-3,3] x [-2,2] x [2,8])
    p_c0 = np.stack([rng.uniform(-3, 3, n_lm), rng.uniform(-2, 2, n_lm), rng.uniform(2, 8, n_lm)], 1)
    T_W_C0 = T_W_B[0] @ T_B_CL
    p_W = (T_W_C0[:3, :3] @ p_c0.T).T + T_W_C0[:3, 3]
    start = rng.integers(0, n_kf - kf_per_lm + 1, n_lm)
    obs_lm, obs_kf, obs_cam, obs_uv = [], [], [], []
    sig = noise_px / FX_LEFT
    for l in range(n_lm):
        for k in range(start[l], start[l] + kf_per_lm):
            T_B_W = np.linalg.inv(T_W_B[k])
            for c in range(2):
                T = T_C_B[c] @ T_B_W
                pc = T[:3, :3] @ p_W[l] + T[:3, 3]
                uv = pc[:2] / pc[2] + rng.normal(0.0, sig, 2)
                obs_lm.append(l)
                obs_kf.append(k)
                obs_cam.append(c)
                obs_uv.append(uv)
    true_pose7 = np.stack([pose7_from_T_W_B(T) for T in T_W_B])
    rng2 = np.random.default_rng(init_seed)
    pose7 = true_pose7.copy()
    for k in range(1, n_kf):
        T = T_W_B[k].copy()
        T[:3, :3] = small_rot(rng2, pose_noise[1]) @ T[:3, :3]
        T[:3, 3] += rng2.normal(0.0, pose_noise[0] / math.sqrt(3.0), 3)
        pose7[k] = pose7_from_T_W_B(T)
    # 5 % depth error along the KF_0 cam0 ray
    scale = 1.0 + rng2.uniform(-depth_noise, depth_noise, n_lm)
    p_init = (T_W_C0[:3, :3] @ (p_c0 * scale[:, None]).T).T + T_W_C0[:3, 3]
    kf_fixed = np.zeros(n_kf, np.uint8)
    kf_fixed[0] = 1
    p_init = np.ascontiguousarray(p_init)
    p_W = np.ascontiguousarray(p_W)
    return BAProblem(pose7=pose7, kf_fixed=kf_fixed, p_W=p_init,
                     obs_lm=np.asarray(obs_lm, np.int32), obs_kf=np.asarray(obs_kf, np.int32),
                     obs_cam=np.asarray(obs_cam, np.uint8),
                     obs_uv=np.asarray(obs_uv, np.float64).astype(np.float32).astype(np.float64),
                     T_C_B2=np.stack([T_C_B[0].reshape(16), T_C_B[1].reshape(16)]),
                     true_pose7=true_pose7, true_p_W=p_W)


def eucm_project(params, xy: np.ndarray) -> np.ndarray:
    """EUCM projection (Khomutenko et al.; camera-intrinsic-model's EUCM, src/datasets/mod.rs:102-113)
    of the rays (x, y, 1): u = fx x / (alpha d + (1 - alpha) z) + cx, d = sqrt(beta (x^2 + y^2) + z^2).
    Config 5's pixel observations -- input generation, f64 in, f32 pixels out."""
    fx, fy, cx, cy, alpha, beta = params[:6]
    x, y = xy[:, 0], xy[:, 1]
    d = np.sqrt(beta * (x * x + y * y) + 1.0)
    den = alpha * d + (1.0 - alpha)
    return np.stack([fx * x / den + cx, fy * y / den + cy], 1).astype(np.float32)


def config5_problem(cams, seed: int = 55, init_seed: int = 56):
    """BASELINE config 5: window 20 (19 free keyframes), 5,000 landmarks x 8 consecutive keyframes x
    2 cameras = 80,000 observations, observed as EUCM pixels (TUM-VI cam0/cam1).  Returns the
    problem (obs_uv still the true normalised coordinates) and the f32 pixel observations."""
    prob = ba_problem(n_kf=20, n_lm=5000, kf_per_lm=8, seed=seed, init_seed=init_seed)
    px = np.empty((prob.n_obs, 2), np.float32)
    for c in range(2):
        sel = prob.obs_cam == c
        px[sel] = eucm_project(cams[c].params, prob.obs_uv[sel])
    return prob, px


@dataclass
class MotionFrame:
    """One frame for track_motion: the map (ids ascending, p_W f32), the frame's features per
    camera (ids, undistorted coordinates f32), the last keyframe's T_W_B, the true T_W_B and
    T_C_B2 (T_Cl_B, T_Cr_B)."""
    map_ids: np.ndarray
    map_pw: np.ndarray
    ids_l: np.ndarray
    uv_l: np.ndarray
    ids_r: np.ndarray
    uv_r: np.ndarray
    T_W_B_last_kf: np.ndarray
    T_W_B_true: np.ndarray
    T_C_B2: np.ndarray


def motion_frame(n_map: int = 2000, n_feat: int = 300, seed: int = 3, step=(0.03, math.radians(1.0)),
                 noise_px: float = 0.5, map_noise: float = 0.01, outlier_frac: float = 0.0,
                 unmapped: int = 40) -> MotionFrame:
    """Config-4-like motion tracking input: map points in front of the
    last keyframe's left camera, a frame moved by `step` (translation m, rotation rad), the
    features the frame sees (left ids + right ids, some unmapped), normalised observations
    with pixel noise, and map points perturbed by `map_noise` m and stored as f32."""
    rng = np.random.default_rng(seed)
    T_last = np.eye(4)
    T_last[:3, :3] = rot_z(0.1)
    T_last[:3, 3] = [0.5, -0.2, 0.1]
    T_true = T_last.copy()
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    a = step[1]
    dR = np.eye(3) + math.sin(a) * K + (1 - math.cos(a)) * (K @ K)
    dt = rng.normal(size=3)
    dt *= step[0] / np.linalg.norm(dt)
    T_true[:3, :3] = T_last[:3, :3] @ dR
    T_true[:3, 3] = T_last[:3, 3] + T_last[:3, :3] @ dt
    T_C_B = [np.linalg.inv(T_B_CL), np.linalg.inv(T_B_CR)]
    p_c0 = np.stack([rng.uniform(-3, 3, n_map), rng.uniform(-2, 2, n_map), rng.uniform(2, 8, n_map)], 1)
    T_W_C0 = T_last @ T_B_CL
    p_W = (T_W_C0[:3, :3] @ p_c0.T).T + T_W_C0[:3, 3]
    map_ids = np.sort(rng.choice(np.arange(10, 10 * n_map + 10), n_map, replace=False)).astype(np.uint64)
    map_pw = (p_W + rng.normal(0.0, map_noise, p_W.shape)).astype(np.float32)
    sig = noise_px / FX_LEFT
    seen = np.sort(rng.choice(n_map, min(n_feat, n_map), replace=False))
    T_B_W = np.linalg.inv(T_true)
    feats = []
    for c in range(2):
        T = T_C_B[c] @ T_B_W
        ids, uv = [], []
        for l in seen:
            pc = T[:3, :3] @ p_W[l] + T[:3, 3]
            if pc[2] <= 0.1:
                continue
            o = pc[:2] / pc[2] + rng.normal(0.0, sig, 2)
            if rng.uniform() < outlier_frac:
                o = o + rng.uniform(-6.0, 6.0, 2)   # beyond the Huber knee (delta 2)
            ids.append(map_ids[l])
            uv.append(o)
        # features without a map point (new tracks): ids not in the map
        for u in range(unmapped):
            ids.append(np.uint64(10 * n_map + 100 + 7 * u + c))
            uv.append(rng.uniform(-0.5, 0.5, 2))
        ids = np.asarray(ids, np.uint64)
        uv = np.asarray(uv, np.float64).astype(np.float32)
        order = np.argsort(ids, kind="stable")   # the tracker returns features sorted by id
        feats.append((ids[order], uv[order]))
    return MotionFrame(map_ids=map_ids, map_pw=map_pw, ids_l=feats[0][0], uv_l=feats[0][1], ids_r=feats[1][0],
                       uv_r=feats[1][1], T_W_B_last_kf=T_last, T_W_B_true=T_true,
                       T_C_B2=np.stack([T_C_B[0].reshape(16), T_C_B[1].reshape(16)]))


# ---------------- feature_tracker/ crate variant (mono, f32 in [0, 1]) ----------------

def make_mosaic(w: int, h: int, n_rects: int = 1500, seed: int = 20260321, size=(8.0, 60.0)):
    """Rectangle mosaic in texture coordinates: strong, well-separated corners for Shi-Tomasi
    (the blob texture of config 2 has too little corner energy at detection_threshold 2.5)."""
    rng = np.random.default_rng(seed)
    margin = 60.0
    x0 = rng.uniform(-margin, w + margin, n_rects)
    y0 = rng.uniform(-margin, h + margin, n_rects)
    ww = rng.uniform(size[0], size[1], n_rects)
    hh = rng.uniform(size[0], size[1], n_rects)
    val = rng.uniform(0.05, 0.95, n_rects)
    return np.stack([x0, y0, x0 + ww, y0 + hh, val], 1)


def render_mosaic(rects: np.ndarray, w: int, h: int, t: int, noise: np.ndarray) -> np.ndarray:
    """Frame t: texture warped by the config-2 motion (0.2 deg/frame about the centre, then a
    (1.7, -0.9) px/frame shift), painter's order, plus noise; f32 clamped to [0, 1]."""
    ang = math.radians(0.2) * t
    ca, sa = math.cos(ang), math.sin(ang)
    sx, sy = 1.7 * t, -0.9 * t
    cx, cy = w / 2.0, h / 2.0
    img = np.full((h, w), 0.5)
    for x0, y0, x1, y1, v in rects:
        cs = np.array([[x0, y0], [x1, y0], [x0, y1], [x1, y1]])
        px = ca * (cs[:, 0] - cx) - sa * (cs[:, 1] - cy) + cx + sx
        py = sa * (cs[:, 0] - cx) + ca * (cs[:, 1] - cy) + cy + sy
        a0, a1 = max(0, int(px.min()) - 1), min(w, int(px.max()) + 2)
        b0, b1 = max(0, int(py.min()) - 1), min(h, int(py.max()) + 2)
        if a0 >= a1 or b0 >= b1:
            continue
        ys, xs = np.mgrid[b0:b1, a0:a1].astype(np.float64)
        x = xs - cx - sx
        y = ys - cy - sy
        u = ca * x + sa * y + cx
        v_ = -sa * x + ca * y + cy
        m = (u >= x0) & (u < x1) & (v_ >= y0) & (v_ < y1)
        img[b0:b1, a0:a1][m] = v
    return np.clip(img + noise, 0.0, 1.0).astype(np.float32)


def mono_sequence(n_frames: int, w: int = 752, h: int = 480, seed: int = 20260321):
    """Yield f32 frames (luma in [0, 1], as DynamicImage::to_luma32f) for the crate tracker."""
    rects = make_mosaic(w, h, seed=seed)
    rng = np.random.default_rng(seed + 1)
    for t in range(n_frames):
        yield render_mosaic(rects, w, h, t, 0.01 * rng.standard_normal((h, w)))


# ----------------------------------------------------------------------------------------
# Full-pipeline stream (config 4): rendered stereo of a piecewise-planar scene
# ----------------------------------------------------------------------------------------
# config/euroc_vio.yaml:11-17 (cam0 / cam1 intrinsics and radtan distortion)
EUROC_INTRINSICS = ((458.654, 457.296, 367.215, 248.375, -0.28340811, 0.07395907, 0.00019359, 1.76187114e-05),
                    (457.587, 456.134, 379.999, 255.238, -0.28368365, 0.07451284, -0.00010473, -3.55590700e-05))


def radtan_undistort_map(params, w: int, h: int, iterations: int = 20) -> np.ndarray:
    """Normalised undistorted (x, y) of every pixel centre (h x w x 2, f64): Newton on the
    radtan model x_d = x (1 + k1 r^2 + k2 r^4) + 2 p1 x y + p2 (r^2 + 2 x^2) (and y)."""
    fx, fy, cx, cy, k1, k2, p1, p2 = params
    v, u = np.mgrid[0:h, 0:w].astype(np.float64)
    xd, yd = (u - cx) / fx, (v - cy) / fy
    x, y = xd.copy(), yd.copy()
    for _ in range(iterations):
        r2 = x * x + y * y
        rad = 1.0 + k1 * r2 + k2 * r2 * r2
        fxv = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x) - xd
        fyv = y * rad + 2 * p2 * x * y + p1 * (r2 + 2 * y * y) - yd
        drad = 2 * k1 + 4 * k2 * r2
        j11 = rad + x * x * drad + 2 * p1 * y + 6 * p2 * x
        j12 = x * y * drad + 2 * p1 * x + 2 * p2 * y
        j21 = x * y * drad + 2 * p2 * y + 2 * p1 * x
        j22 = rad + y * y * drad + 2 * p2 * x + 6 * p1 * y
        det = j11 * j22 - j12 * j21
        x = x - (j22 * fxv - j12 * fyv) / det
        y = y - (-j21 * fxv + j11 * fyv) / det
    return np.stack([x, y], -1)


@dataclass
class SceneStream:
    """Config-4 input: rendered stereo frames, their true body poses and the rig."""
    frames: list            # [(left u8 h x w, right u8 h x w)]
    T_W_B: list             # true body poses (4 x 4)
    T_B_Cl: np.ndarray
    T_B_Cr: np.ndarray
    intrinsics: tuple       # (cam0, cam1) radtan parameters (fx, fy, cx, cy, k1, k2, p1, p2)


def _scene_setup(n_frames, w, h, step, seed):
    rng = np.random.default_rng(seed)
    s = w / 752.0
    intr = tuple((p[0] * s, p[1] * s, p[2] * s, p[3] * (h / 480.0)) + tuple(p[4:]) for p in EUROC_INTRINSICS)
    tex_w, tex_h = 1536, 1024
    tex = make_texture(tex_w, tex_h, n_blobs=int(6000 * tex_w * tex_h / (752 * 480)), seed=seed + 100)
    T = _render(tex, tex_w, tex_h, 0, False, np.zeros((tex_h, tex_w))).astype(np.float64)
    bands = []  # (y0, y1, z, texture offset)
    y = -3.0
    while y < 3.0 + step * n_frames + 3.0:
        wdt = rng.uniform(0.6, 1.6)
        bands.append((y, y + wdt, rng.uniform(3.0, 8.0), rng.uniform(0, tex_w * 0.004)))
        y += wdt
    bands.append((-1e9, 1e9, 12.0, 0.77))
    rays = [radtan_undistort_map(p[:8], w, h) for p in intr]
    return rng, intr, T, bands, rays


def _scene_image(xp, T, bands, ray, T_W_C):
    """Noise-free image of the plane scene through one camera; xp is numpy or torch (same math,
    f64).  Each pixel's ray hits the nearest band plane; texture sampled bilinearly, periodic."""
    res = 0.004
    tex_h, tex_w = T.shape
    R, o = T_W_C[:3, :3], T_W_C[:3, 3]
    d = [ray[..., 0] * R[i, 0] + ray[..., 1] * R[i, 1] + R[i, 2] for i in range(3)]
    best = xp.full(ray.shape[:2], float("inf"), **xp.kw)
    u = xp.zeros(ray.shape[:2], **xp.kw)
    v = xp.zeros(ray.shape[:2], **xp.kw)
    for (y0, y1, z, off) in bands:
        tt = (z - o[2]) / d[2]
        X = o[0] + tt * d[0]
        Y = o[1] + tt * d[1]
        hit = (tt > 0) & (Y >= y0) & (Y < y1) & (tt < best)
        best = xp.where(hit, tt, best)
        u = xp.where(hit, (Y + off) / res, u)
        v = xp.where(hit, X / res, v)
    u = u % (tex_w - 1)
    v = v % (tex_h - 1)
    iu, iv = xp.floor(u), xp.floor(v)
    fu, fv = u - iu, v - iv
    iu, iv = xp.long(iu), xp.long(iv)
    iu1, iv1 = xp.minimum(iu + 1, tex_w - 1), xp.minimum(iv + 1, tex_h - 1)
    return (1 - fv) * ((1 - fu) * T[iv, iu] + fu * T[iv, iu1]) + fv * ((1 - fu) * T[iv1, iu] + fu * T[iv1, iu1])


class _NumpyOps:
    kw = {}
    where, floor, minimum, full, zeros = np.where, np.floor, np.minimum, np.full, np.zeros

    @staticmethod
    def long(a):
        return a.astype(np.int64)


def euroc_scene_stream(n_frames: int, w: int = 752, h: int = 480, step: float = 0.02, seed: int = 4,
                       noise: float = 2.0) -> SceneStream:
    """BASELINE config 4: stereo renderings of textured planes at 3-8 m with the
    EuRoC rig (intrinsics, radtan distortion, T_B_Cl / T_B_Cr) moving `step` m per frame along
    the body y axis (the cameras' x axis).  Planes are world z = const over bands of world y,
    a background plane at 12 m; each plane carries a blob texture (4 mm texels, periodic),
    sampled bilinearly, plus `noise` * N(0, 1) per pixel.  Intrinsics scale with w / 752."""
    rng, intr, T, bands, rays = _scene_setup(n_frames, w, h, step, seed)
    T_B_C = (T_B_CL, T_B_CR)
    frames, poses = [], []
    for t in range(n_frames):
        T_W_B = np.eye(4)
        T_W_B[1, 3] = step * t
        poses.append(T_W_B)
        pair = []
        for c in range(2):
            img = _scene_image(_NumpyOps, T, bands, rays[c], T_W_B @ T_B_C[c])
            img += noise * rng.standard_normal((h, w))
            pair.append(np.clip(np.rint(img), 0, 255).astype(np.uint8))
        frames.append(tuple(pair))
    return SceneStream(frames=frames, T_W_B=poses, T_B_Cl=T_B_CL.copy(), T_B_Cr=T_B_CR.copy(), intrinsics=intr)


def euroc_scene_stream_device(n_frames: int, device, w: int = 752, h: int = 480, step: float = 0.02, seed: int = 4,
                              noise: float = 2.0) -> SceneStream:
    """euroc_scene_stream rendered with torch on `device` (bench input generation: 500 frames in
    seconds, resident in HBM).  Same scene and poses; the noise comes from torch's generator, so
    frames differ from the numpy stream by the noise only.  frames: [(left, right)] u8 tensors."""
    import torch

    class Ops:
        kw = {"dtype": torch.float64, "device": device}
        where, floor = torch.where, torch.floor

        @staticmethod
        def minimum(a, b):
            return torch.clamp(a, max=b)

        @staticmethod
        def full(shape, val, **kw):
            return torch.full(tuple(shape), val, **kw)

        @staticmethod
        def zeros(shape, **kw):
            return torch.zeros(tuple(shape), **kw)

        @staticmethod
        def long(a):
            return a.long()

    _, intr, T, bands, rays = _scene_setup(n_frames, w, h, step, seed)
    T = torch.as_tensor(T, device=device)
    rays = [torch.as_tensor(r, device=device) for r in rays]
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    T_B_C = (T_B_CL, T_B_CR)
    frames, poses = [], []
    for t in range(n_frames):
        T_W_B = np.eye(4)
        T_W_B[1, 3] = step * t
        poses.append(T_W_B)
        pair = []
        for c in range(2):
            img = _scene_image(Ops, T, bands, rays[c], T_W_B @ T_B_C[c])
            img += noise * torch.randn((h, w), generator=gen, dtype=torch.float64, device=device)
            pair.append(torch.clamp(torch.round(img), 0, 255).to(torch.uint8).contiguous())
        frames.append(tuple(pair))
    return SceneStream(frames=frames, T_W_B=poses, T_B_Cl=T_B_CL.copy(), T_B_Cr=T_B_CR.copy(), intrinsics=intr)
