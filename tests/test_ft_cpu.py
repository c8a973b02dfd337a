"""CPU tests of the feature_tracker/ crate restatement (oracle/ft_oracle.cpp): the reference
crate's own known-answer tests, properties the published third-party algorithms fix, and the
committed golden vectors (tests/golden/ft_small.npz)."""
import hashlib
import math
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def iso_matrix(iso):
    c, s, tx, ty = (float(v) for v in iso)
    return np.array([[c, -s], [s, c]]), np.array([tx, ty])


def test_exp_se2_known_answers(oracle):
    # feature_tracker/src/feature_tracker/feature_tracking.rs:264-283, twist [theta, vx, vy], tol 1e-6
    pi = np.float32(math.pi)
    R, t = iso_matrix(oracle.ft_exp_se2([0.0, 0.0, 0.0]))
    assert np.allclose(R, np.eye(2), atol=1e-6) and np.allclose(t, 0, atol=1e-6)
    R, t = iso_matrix(oracle.ft_exp_se2([pi, 0.0, 0.0]))
    assert np.allclose(R, -np.eye(2), atol=1e-6) and np.allclose(t, 0, atol=1e-6)
    R, t = iso_matrix(oracle.ft_exp_se2([0.0, 1.32, -1.56]))
    assert np.allclose(R, np.eye(2), atol=1e-6) and np.allclose(t, [1.32, -1.56], atol=1e-6)


@pytest.mark.parametrize("twist", [(0.0, 0.0, 0.0), (math.pi / 3, 1.0, 2.5), (1.795, 1.0, 2.5), (1e-8, 1.0, 2.5),
                                   (1e-7, 1.0, 2.5), (2e-7, 1.0, 2.5)])
def test_exp_log_round_trip(oracle, twist):
    # feature_tracking.rs:251-262,285-290: log(exp(tau)) == tau (theta modulo 2 pi), rel/abs 1e-6
    tau = np.array(twist, np.float32)
    back = oracle.ft_log_se2(oracle.ft_exp_se2(tau)).astype(np.float64)
    two_pi = 2 * math.pi
    tau = tau.astype(np.float64)
    tau[0] -= math.floor(tau[0] / two_pi) * two_pi
    back[0] -= math.floor(back[0] / two_pi) * two_pi
    assert np.allclose(back, tau, rtol=1e-6, atol=1e-6)


def test_pyramid_dimensions(oracle):
    # feature_tracker/src/image_operations.rs:84-94: 120x60 -> 60x30 -> 30x15
    assert oracle.ft_level_dims(120, 60, 3) == [(120, 60), (60, 30), (30, 15)]
    img = np.full((60, 120), 5 / 255, np.float32)
    pyr = oracle.ft_build_pyramid(img, 3, blur=False)
    assert pyr.size == 120 * 60 + 60 * 30 + 30 * 15
    # ratio 1.5 and odd sizes: round(w / ratio^l), each level from the previous one
    assert oracle.ft_level_dims(752, 480, 5, 1.5) == [(752, 480), (501, 320), (334, 213), (223, 142), (149, 95)]


def test_constant_image_is_a_fixed_point(oracle):
    img = np.full((61, 97), 0.37, np.float32)
    for blur in (False, True):
        lv = oracle.ft_split_pyramid(oracle.ft_build_pyramid(img, 4, blur=blur), 97, 61, 4)
        for l in lv:
            assert np.abs(l - np.float32(0.37)).max() < 1e-6
    assert np.abs(oracle.ft_fast_blur(img, 6.0) - np.float32(0.37)).max() < 1e-6
    assert np.all(oracle.ft_shi_tomasi_score(img) == 0)
    assert len(oracle.ft_add_points(img)) == 0


def test_resample_clamps_to_unit_interval(oracle):
    # image 0.25: f32 resampling output is clamped to [0, 1] (Primitive::DEFAULT_MAX_VALUE = 1.0)
    rng = np.random.default_rng(0)
    img = rng.uniform(-1, 2, (40, 50)).astype(np.float32)
    out = oracle.ft_resize_triangle(img, 25, 20)
    assert out.min() >= 0 and out.max() <= 1
    blur = oracle.ft_gaussian_blur(img, 2.0)
    assert blur.min() >= 0 and blur.max() <= 1


def test_boxes_for_gauss(oracle):
    # image 0.25 fast_blur: n = 3 box widths approximating a Gaussian of sigma
    assert oracle.ft_boxes_for_gauss(6.0) == [11, 11, 13]   # config.yaml detection_blur
    assert oracle.ft_boxes_for_gauss(2.0) == [3, 3, 5]
    for s in (1.0, 3.3, 6.0, 9.5):
        assert all(b % 2 == 1 for b in oracle.ft_boxes_for_gauss(s))


def test_bicubic_smoke_and_bounds(oracle):
    # image_operations.rs:292-300 (smoke), :150-154 (valid cells 1..=w-3)
    z = np.zeros((100, 100), np.float32)
    assert oracle.ft_bicubic(z, 1.0, 2.0)[0] == 0
    assert oracle.ft_bicubic(z, 0.99, 2.0) is None
    assert oracle.ft_bicubic(z, 97.99, 2.0) is not None
    assert oracle.ft_bicubic(z, 98.0, 2.0) is None


def test_bicubic_derivative_finite_difference(oracle):
    # image_operations.rs:305-368: analytic derivatives vs central differences, tol = 50 sqrt(eps)
    rng = np.random.default_rng(7)
    img = rng.standard_normal((32, 32)).astype(np.float32)
    delta = np.float32(np.sqrt(np.finfo(np.float32).eps))
    tol = 50 * delta
    for _ in range(200):
        x, y = rng.uniform(2.1, 28.9, 2)
        fx, fy = math.floor(x), math.floor(y)
        x = float(np.clip(x, fx + 2 * delta, fx + 1 - 2 * delta))
        y = float(np.clip(y, fy + 2 * delta, fy + 1 - 2 * delta))
        _, gx, gy = oracle.ft_bicubic(img, x, y)
        dx = (oracle.ft_bicubic(img, x + delta, y)[0] - oracle.ft_bicubic(img, x - delta, y)[0]) / (2 * delta)
        dy = (oracle.ft_bicubic(img, x, y + delta)[0] - oracle.ft_bicubic(img, x, y - delta)[0]) / (2 * delta)
        assert abs(dx - gx) <= tol * max(1.0, abs(gx)) and abs(dy - gy) <= tol * max(1.0, abs(gy))


def test_shi_tomasi_finds_square_corners(oracle):
    img = np.full((96, 128), 0.2, np.float32)
    img[30:70, 40:90] = 0.8
    pts = oracle.ft_add_points(img)
    assert len(pts) == 4
    for cx, cy in ((40, 30), (89, 30), (40, 69), (89, 69)):
        assert np.min(np.abs(pts.astype(int) - [cx, cy]).sum(1)) <= 8   # blurred: a few px inside
    # (y, x) order, inside [md, w - md) x [md, h - md)
    assert list(map(tuple, pts[np.lexsort((pts[:, 0], pts[:, 1]))])) == list(map(tuple, pts))
    # a tracked feature at a corner suppresses the new corner there (feature_detection.rs:61-68)
    pts2 = oracle.ft_add_points(img, np.array([[41.0, 31.0]], np.float32))
    assert len(pts2) == 3


def test_track_points_recovers_translation(oracle):
    from rsvio import synthetic as S
    w, h = 160, 120
    rects = S.make_mosaic(w, h, n_rects=160, seed=5, size=(6.0, 28.0))
    f0 = S.render_mosaic(rects, w, h, 0, np.zeros((h, w)))
    f1 = S.render_mosaic(rects, w, h, 1, np.zeros((h, w)))
    p0, p1 = oracle.ft_build_pyramid(f0, 3), oracle.ft_build_pyramid(f1, 3)
    xy = oracle.ft_add_points(p0[:w * h].reshape(h, w)).astype(np.float32)
    assert len(xy) >= 5
    iso, ok = oracle.ft_track_points(p0, p1, w, h, xy, nlevels=3)
    assert ok.mean() > 0.6
    ang = math.radians(0.2)
    for (x, y), T, k in zip(xy, iso, ok):
        if not k:
            continue
        R, t = iso_matrix(T)
        got = R @ [x, y] + t
        exp = [math.cos(ang) * (x - w / 2) - math.sin(ang) * (y - h / 2) + w / 2 + 1.7,
               math.sin(ang) * (x - w / 2) + math.cos(ang) * (y - h / 2) + h / 2 - 0.9]
        assert np.hypot(*(got - exp)) < 1.0   # the mosaic is point-sampled: edges move in whole pixels


def test_golden_vectors(oracle):
    g = np.load(GOLD / "ft_small.npz", allow_pickle=False)
    w, h, L = int(g["w"]), int(g["h"]), int(g["levels"])
    frames = g["frames"]
    pyr0 = oracle.ft_build_pyramid(frames[0], L)
    pyr1 = oracle.ft_build_pyramid(frames[1], L)
    assert sha(pyr0) == str(g["sha_pyr0"]) and sha(pyr1) == str(g["sha_pyr1"])
    assert sha(oracle.ft_build_pyramid(frames[0], L, blur=False)) == str(g["sha_pyr0_noblur"])
    fine0 = pyr0[:w * h].reshape(h, w)
    assert sha(oracle.ft_shi_tomasi_score(fine0)) == str(g["sha_score0"])
    assert np.array_equal(oracle.ft_add_points(fine0), g["new0"])
    assert np.array_equal(oracle.ft_add_points(fine0, g["trk_xy"]), g["new0_tr"])
    for cost, key in ((0, "ssd"), (1, "lssd")):
        iso, ok = oracle.ft_track_points(pyr0, pyr1, w, h, g["xy"], nlevels=L, cost=cost)
        assert np.array_equal(ok, g["v_" + key]) and np.array_equal(iso, g["iso_" + key])
    ft = oracle.FeatureTracker(w, h, oracle.ft_config(nlevels=L))
    rows = []
    for k in range(len(frames)):
        ids, xy = ft.process_frame(frames[k])
        rows += [(k, int(i), float(p[0]), float(p[1])) for i, p in zip(ids, xy)]
    assert np.array_equal(np.array(rows, np.float64), g["pipe"])


def test_feature_tracker_bookkeeping(oracle):
    """feature_tracker.rs:115-176: tracked features keep their ids and previous order, new
    corners get consecutive fresh ids after them."""
    from rsvio import synthetic as S
    w, h = 320, 240
    rects = S.make_mosaic(w, h, n_rects=400, seed=11, size=(6.0, 40.0))
    ft = oracle.FeatureTracker(w, h, oracle.ft_config(nlevels=4))
    prev_ids, next_id = [], 0
    for t in range(4):
        ids, xy = ft.process_frame(S.render_mosaic(rects, w, h, t, np.zeros((h, w))))
        ids = ids.tolist()
        assert len(set(ids)) == len(ids)
        n_tr = sum(1 for i in ids if i < next_id)
        assert ids[:n_tr] == [i for i in prev_ids if i in set(ids[:n_tr])]
        assert ids[n_tr:] == list(range(next_id, next_id + len(ids) - n_tr))
        if t > 0:
            assert n_tr >= 0.6 * len(prev_ids)
        next_id += len(ids) - n_tr
        prev_ids = ids
