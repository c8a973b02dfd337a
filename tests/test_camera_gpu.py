"""T12 on the GPU: rsvio_unproject / rsvio_unproject_d / the tracker's fused unprojection are
bit-exact with the oracle (f64 arithmetic with IEEE division and sqrt on both sides, outputs
narrowed to f32 like src/estimator/frame.rs:119), including the invalid points (NaN, valid = 0).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b):
    """bitwise equality with NaN == NaN"""
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _ocam(oracle, cam):
    from rsvio.camera import CONVENTIONS
    return oracle.camera(cam.model, cam.params, CONVENTIONS[cam.convention], cam.max_iterations)


def _pixels(w, h, n, seed):
    rng = np.random.default_rng(seed)
    px = np.stack([rng.uniform(-20, w + 20, n), rng.uniform(-20, h + 20, n)], 1).astype(np.float32)
    xs, ys = np.meshgrid(np.arange(w, dtype=np.float32), np.arange(0, h, 7, dtype=np.float32))
    return np.concatenate([px, np.stack([xs.ravel(), ys.ravel()], 1)])


@pytest.mark.parametrize("which", ["euroc", "tum"])
@pytest.mark.parametrize("convention", ["plane", "ray"])
def test_unproject_bit_exact_vs_oracle(gpu, oracle, which, convention):
    import dataclasses

    from rsvio.camera import EUROC, TUM_VI
    cams, (w, h) = (EUROC, (752, 480)) if which == "euroc" else (TUM_VI, (512, 512))
    for k, cam in enumerate(cams):
        cam = dataclasses.replace(cam, convention=convention)
        px = _pixels(w, h, 20000, 3 + k)
        out, ok = cam.unproject(px)
        ref, rok = oracle.unproject(_ocam(oracle, cam), px)
        assert np.array_equal(ok, rok)
        assert _same(out, ref)
        assert ok.mean() > 0.85


def test_unproject_edge_cases(gpu, oracle):
    import dataclasses

    from rsvio.camera import EUROC, Camera
    # empty input
    out, ok = EUROC[0].unproject(np.zeros((0, 2), np.float32))
    assert out.shape == (0, 2) and ok.shape == (0,)
    # non-convergence (1 Newton step) and non-finite pixels are flagged identically
    cam = dataclasses.replace(EUROC[0], max_iterations=1)
    px = np.array([[10, 10], [367.215, 248.375], [np.nan, 3], [np.inf, 1]], np.float32)
    out, ok = cam.unproject(px)
    ref, rok = oracle.unproject(_ocam(oracle, cam), px)
    assert np.array_equal(ok, rok) and _same(out, ref)
    assert ok.tolist() == [False, True, False, False]
    # no distortion: the pinhole inverse
    pin = Camera.opencv5(400.0, 410.0, 320.5, 240.25)
    px = _pixels(640, 480, 1000, 9)
    out, ok = pin.unproject(px)
    exp = np.stack([(px[:, 0].astype(np.float64) - 320.5) / 400.0,
                    (px[:, 1].astype(np.float64) - 240.25) / 410.0], 1).astype(np.float32)
    assert ok.all() and np.array_equal(out, exp)


def test_unproject_device_max_size(gpu, oracle):
    """Config 5's batch shape scaled up: 2**21 points through the device entry point on a
    stream, checked bit-exact against the oracle."""
    import torch

    from rsvio.camera import TUM_VI
    cam = TUM_VI[0]
    n = 1 << 21
    rng = np.random.default_rng(5)
    px = np.stack([rng.uniform(0, 512, n), rng.uniform(0, 512, n)], 1).astype(np.float32)
    d_px = torch.from_numpy(px).cuda()
    d_out = torch.empty_like(d_px)
    d_ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    cam.unproject_device(d_px.data_ptr(), n, d_out.data_ptr(), d_ok.data_ptr(), s.cuda_stream)
    s.synchronize()
    ref, rok = oracle.unproject(_ocam(oracle, cam), px)
    assert np.array_equal(d_ok.cpu().numpy().astype(bool), rok)
    assert _same(d_out.cpu().numpy(), ref)


def test_tracker_fused_unprojection(gpu, oracle, stereo_frames):
    """Frame::add_left_feature / add_right_feature on the tracker's own output: the fused
    undistorted coordinates equal the oracle's unprojection of the returned pixels."""
    from rsvio.camera import EUROC
    trk = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50)
    trk.set_cameras(*EUROC)
    try:
        for left, right in stereo_frames[:3]:
            fl, fr = trk.process_frame(left, right)
            ul, ur = trk.undistorted()
            assert len(ul) == len(fl) > 50 and len(ur) == len(fr)
            for f, u, cam in ((fl, ul, EUROC[0]), (fr, ur, EUROC[1])):
                px = np.stack([f["x"], f["y"]], 1)
                ref, _ = oracle.unproject(_ocam(oracle, cam), px)
                assert _same(u, ref)
        trk.set_cameras(None, None)
        trk.process_frame(*stereo_frames[3])
        with pytest.raises(gpu.RsvioError):
            trk.undistorted()
    finally:
        trk.close()
