"""GPU parity of the feature_tracker/ crate variant against the CPU oracle,
through the C ABI (lib/librsvio_gpu.so).

Bars:
  * pyramid (blur + Triangle resizes), Shi-Tomasi score map: bit-exact f32;
  * add_points (NMS + local maxima vs tracked features): identical corner lists (integer);
  * track_points (bicubic LK, SSD and LSSD): bit-exact against the oracle, whose exp_se2 calls
    glibc sinf/cosf as Rust's f32::sin/cos do (the kernel's restatement: test_trig_gpu.py);
  * FeatureTracker: identical ids, order and (bitwise) positions frame by frame.
"""
import hashlib
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
W, H = 752, 480


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def ftg(gpu):
    from rsvio import ft
    return ft


@pytest.fixture(scope="module")
def mono_frames():
    from rsvio import synthetic as S
    return list(S.mono_sequence(6))


@pytest.mark.parametrize("shape,levels,ratio,blur", [((480, 752), 5, 2.0, True), ((480, 752), 5, 2.0, False),
                                                     ((61, 97), 4, 2.0, True), ((480, 752), 4, 1.5, True),
                                                     ((120, 160), 3, 2.0, True), ((33, 40), 2, 2.0, True)])
def test_pyramid_bitexact(ftg, oracle, shape, levels, ratio, blur):
    rng = np.random.default_rng(shape[0] + levels)
    img = rng.uniform(0, 1, shape).astype(np.float32)
    ref = oracle.ft_build_pyramid(img, levels, ratio, blur)
    out = ftg.build_image_pyramid(img, levels, ratio, blur)
    assert out.shape == ref.shape
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_pyramid_dimensions(ftg):
    # feature_tracker/src/image_operations.rs:84-94: 120x60 -> 60x30 -> 30x15
    pyr = ftg.build_image_pyramid(np.full((60, 120), 5 / 255, np.float32), 3, 2.0, False)
    assert [x.shape for x in ftg.pyramid_levels(pyr, 120, 60, 3)] == [(60, 120), (30, 60), (15, 30)]


def test_score_bitexact(ftg, oracle, mono_frames):
    fine = oracle.ft_build_pyramid(mono_frames[0], 5)[:W * H].reshape(H, W)
    assert np.array_equal(ftg.shi_tomasi_score(fine).view(np.uint32), oracle.ft_shi_tomasi_score(fine).view(np.uint32))
    rng = np.random.default_rng(3)
    small = rng.uniform(0, 1, (61, 97)).astype(np.float32)
    for blur in (6.0, 2.0):
        assert np.array_equal(ftg.shi_tomasi_score(small, blur), oracle.ft_shi_tomasi_score(small, blur))


@pytest.mark.parametrize("blur", [0.5, 25.0, 40.0, 80.0])
def test_score_box_radii(ftg, oracle, blur):
    """fast_blur box radii across the kernel variants: 2-segment tiles (r <= 31), 3-segment tiles
    (r <= 63) and the any-radius fallback (r = 79 at sigma 80), on a ragged 130 x 200 image."""
    rng = np.random.default_rng(int(blur * 10))
    img = rng.uniform(0, 1, (130, 200)).astype(np.float32)
    a, b = ftg.shi_tomasi_score(img, blur), oracle.ft_shi_tomasi_score(img, blur)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_add_points_identical(ftg, oracle, mono_frames):
    fine = oracle.ft_build_pyramid(mono_frames[0], 5)[:W * H].reshape(H, W)
    ref = oracle.ft_add_points(fine)
    assert len(ref) > 50
    assert np.array_equal(ftg.add_points(fine), ref)
    # with tracked features (every third corner, shifted), including ones off the image
    tr = ref[::3].astype(np.float32) + np.float32(0.4)
    tr = np.concatenate([tr, np.array([[-3.0, 5.0], [W + 4.0, 100.0], [300.0, H - 0.2]], np.float32)])
    ref2 = oracle.ft_add_points(fine, tr)
    assert np.array_equal(ftg.add_points(fine, tr), ref2)
    assert len(ref2) < len(ref)
    # thresholds / min_dist variants
    for thr, md in ((1.0, 15), (5.0, 8), (2.5, 30)):
        assert np.array_equal(ftg.add_points(fine, tr, thr, md), oracle.ft_add_points(fine, tr, thr, md))


def test_golden(ftg):
    g = np.load(GOLD / "ft_small.npz", allow_pickle=False)
    w, h, L = int(g["w"]), int(g["h"]), int(g["levels"])
    frames = g["frames"]
    pyr0 = ftg.build_image_pyramid(frames[0], L)
    pyr1 = ftg.build_image_pyramid(frames[1], L)
    assert sha(pyr0) == str(g["sha_pyr0"]) and sha(pyr1) == str(g["sha_pyr1"])
    assert sha(ftg.build_image_pyramid(frames[0], L, 2.0, False)) == str(g["sha_pyr0_noblur"])
    fine0 = pyr0[:w * h].reshape(h, w)
    assert sha(ftg.shi_tomasi_score(fine0)) == str(g["sha_score0"])
    assert np.array_equal(ftg.add_points(fine0), g["new0"])
    assert np.array_equal(ftg.add_points(fine0, g["trk_xy"]), g["new0_tr"])
    for cost, key in ((0, "ssd"), (1, "lssd")):
        iso, ok = ftg.track_points(pyr0, pyr1, w, h, g["xy"], nlevels=L, matching_cost=cost)
        assert np.array_equal(ok, g["v_" + key]) and np.array_equal(iso, g["iso_" + key])
    t = ftg.FeatureTracker(w, h, ftg.FeatureTrackingConfig(nlevels=L))
    rows = []
    for k in range(len(frames)):
        f = t.process(frames[k])
        rows += [(k, int(r["feature_id"]), float(r["x"]), float(r["y"])) for r in f]
    t.close()
    assert np.array_equal(np.array(rows, np.float64), g["pipe"])


def _track_inputs(oracle, mono_frames):
    p0 = oracle.ft_build_pyramid(mono_frames[0], 5)
    p1 = oracle.ft_build_pyramid(mono_frames[1], 5)
    xy = oracle.ft_add_points(p0[:W * H].reshape(H, W)).astype(np.float32)
    rng = np.random.default_rng(11)
    extra = np.stack([rng.uniform(-5, W + 5, 64), rng.uniform(-5, H + 5, 64)], 1).astype(np.float32)
    edge = np.array([[0, 0], [1.5, 1.5], [W - 1, H - 1], [W - 2.5, 10], [10, H - 2.5], [3.2, 200]], np.float32)
    return p0, p1, np.concatenate([xy, extra, edge])


@pytest.mark.parametrize("cost", [0, 1])
def test_track_points_bitexact(ftg, oracle, mono_frames, cost):
    p0, p1, xy = _track_inputs(oracle, mono_frames)
    ref_iso, ref_ok = oracle.ft_track_points(p0, p1, W, H, xy, nlevels=5, cost=cost)
    iso, ok = ftg.track_points(p0, p1, W, H, xy, nlevels=5, matching_cost=cost)
    assert np.array_equal(ok, ref_ok)
    assert np.array_equal(iso.view(np.uint32), ref_iso.view(np.uint32))
    if cost == 0:
        assert ref_ok[:len(xy) - 70].mean() > 0.8


def test_track_points_far_frames(ftg, oracle, mono_frames):
    """Frames 0 -> 4 (four frames of motion, larger rotation increments): still bit-exact."""
    p0 = oracle.ft_build_pyramid(mono_frames[0], 5)
    p1 = oracle.ft_build_pyramid(mono_frames[4], 5)
    xy = oracle.ft_add_points(p0[:W * H].reshape(H, W)).astype(np.float32)
    ref_iso, ref_ok = oracle.ft_track_points(p0, p1, W, H, xy, nlevels=5)
    iso, ok = ftg.track_points(p0, p1, W, H, xy, nlevels=5)
    assert np.array_equal(ok, ref_ok)
    assert np.array_equal(iso.view(np.uint32), ref_iso.view(np.uint32))


def test_track_points_empty(ftg):
    p = np.zeros(ftg.pyramid_floats(W, H, 5), np.float32)
    iso, ok = ftg.track_points(p, p, W, H, np.zeros((0, 2), np.float32))
    assert iso.shape == (0, 4) and ok.shape == (0,)


@pytest.mark.parametrize("cost,nframes", [(0, 6), (1, 3)])
def test_feature_tracker_pipeline(ftg, oracle, mono_frames, cost, nframes):
    ref = oracle.FeatureTracker(W, H, oracle.ft_config(matching_cost=cost))
    t = ftg.FeatureTracker(W, H, matching_cost=cost)
    for k in range(nframes):
        rid, rxy = ref.process_frame(mono_frames[k])
        f = t.process(mono_frames[k])
        assert np.array_equal(f["feature_id"], rid), k
        assert np.array_equal(np.stack([f["x"], f["y"]], 1).view(np.uint32), rxy.view(np.uint32)), k
    assert len(rid) > 100
    # get_pyramid (feature_tracker.rs:190-193) is the last frame's pyramid
    lv = t.get_pyramid()
    ref_lv = oracle.ft_split_pyramid(oracle.ft_build_pyramid(mono_frames[nframes - 1], 5), W, H, 5)
    assert all(np.array_equal(a, b) for a, b in zip(lv, ref_lv))
    t.close()


def test_feature_tracker_frame_api(ftg, mono_frames):
    t = ftg.FeatureTracker(W, H)
    fr = t.process_frame(mono_frames[0], ftg.Frame(0))
    assert fr.frame_id == 0 and len(fr.features) > 0
    assert [f.feature_id for f in fr.features] == list(range(len(fr.features)))
    t.close()


def test_capacity_error(ftg, mono_frames):
    from rsvio import RsvioError
    t = ftg.FeatureTracker(W, H, max_features=16)
    with pytest.raises(RsvioError) as e:
        t.process(mono_frames[0])
    assert e.value.code == -4
    t.close()
