"""T12 (Frame::add_*_feature unprojection, src/estimator/frame.rs:107-134) on CPU: the oracle's
restatement of camera-intrinsic-model's OpenCVModel5 / EUCM unproject_one, checked by the
properties the published models fix (the crate itself is not available offline, so the
algorithm is "parity unpinned" -- DESIGN.md §6), and the host-side config mirror of
create_camera_models_from_config (src/datasets/mod.rs:93-163)."""
import numpy as np
import pytest

EUROC0 = [458.654, 457.296, 367.215, 248.375, -0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.0]
TUM0 = [191.75556798912652, 191.74816751185256, 254.9226487139376, 256.8780365577954,
        0.6246288732884442, 1.0598071085569876]


def _grid(w, h, n=41):
    xs, ys = np.meshgrid(np.linspace(0, w - 1, n), np.linspace(0, h - 1, n))
    return np.stack([xs.ravel(), ys.ravel()], 1).astype(np.float32)


def test_radtan_without_distortion_is_the_pinhole_inverse(oracle):
    """k = p = 0: one Newton step with a zero residual; the result is exactly (u-cx)/fx."""
    cam = oracle.camera(0, [400.0, 410.0, 320.5, 240.25, 0, 0, 0, 0, 0])
    px = _grid(640, 480)
    out, ok = oracle.unproject(cam, px)
    assert ok.all()
    exp = np.stack([(px[:, 0].astype(np.float64) - 320.5) / 400.0,
                    (px[:, 1].astype(np.float64) - 240.25) / 410.0], 1).astype(np.float32)
    assert np.array_equal(out, exp)


@pytest.mark.parametrize("model,params,w,h", [(0, EUROC0, 752, 480), (1, TUM0, 512, 512)])
def test_project_unproject_round_trip(oracle, model, params, w, h):
    cam = oracle.camera(model, params)
    px = _grid(w, h)
    xy, ok = oracle.unproject(cam, px)
    # plane convention: EUCM pixels beyond 90 degrees (fisheye corners) have z <= 0 -> invalid
    assert ok.mean() > (0.99 if model == 0 else 0.9)
    pts = np.concatenate([xy[ok].astype(np.float64), np.ones((ok.sum(), 1))], 1)
    uv, vok = oracle.project(cam, pts)
    assert vok.all()
    # the f32 narrowing of (x, y) (frame.rs:119) is the only loss: <= ~2e-5 px at these focals
    assert np.abs(uv - px[ok]).max() < 5e-5


def test_ray_convention_is_the_normalised_plane_point(oracle):
    plane = oracle.camera(0, EUROC0, 0)
    ray = oracle.camera(0, EUROC0, 1)
    px = _grid(752, 480, 21)
    a, _ = oracle.unproject(plane, px)
    b, _ = oracle.unproject(ray, px)
    a64 = a.astype(np.float64)
    n = np.sqrt((a64 ** 2).sum(1) + 1.0)
    assert np.abs(b - a64 / n[:, None]).max() < 1e-6
    # at the image corners the two conventions differ by ~20 %
    assert np.abs(a[0] / b[0] - 1).max() > 0.15


def test_eucm_outside_the_valid_cone_is_nan(oracle):
    """alpha > 1/2: r^2 > 1 / (beta (2 alpha - 1)) has no preimage."""
    cam = oracle.camera(1, TUM0, 1)
    fx, cx, cy = TUM0[0], TUM0[2], TUM0[3]
    alpha, beta = TUM0[4], TUM0[5]
    r_max = np.sqrt(1.0 / (beta * (2 * alpha - 1)))
    px = np.array([[cx + fx * r_max * 1.01, cy], [cx + fx * r_max * 0.99, cy]], np.float32)
    out, ok = oracle.unproject(cam, px)
    assert ok.tolist() == [False, True]
    assert np.isnan(out[0]).all() and np.isfinite(out[1]).all()


def test_radtan_non_convergence_is_flagged(oracle):
    cam = oracle.camera(0, EUROC0, 0, max_iterations=1)
    out, ok = oracle.unproject(cam, np.array([[10.0, 10.0], [367.215, 248.375]], np.float32))
    assert ok.tolist() == [False, True]      # the principal point converges in one step
    assert np.isnan(out[0]).all()


def test_camera_from_config_mirrors_dataset_defaults():
    from rsvio.camera import EUCM, EUROC, OPENCV5, Camera
    c = Camera.from_config([], [], None)
    assert c.model == OPENCV5 and c.params == [500.0, 500.0, 320.0, 240.0, 0, 0, 0, 0, 0]
    e = Camera.from_config([1, 2, 3, 4], [], "eucm")
    assert e.model == EUCM and e.params == [1, 2, 3, 4, 0.5, 1.0]
    assert EUROC[0].params[:8] == EUROC0[:8] and EUROC[0].params[8] == 0.0
    s = EUROC[1].struct()
    assert s.model == 0 and s.convention == 0 and s.max_iterations == 20
