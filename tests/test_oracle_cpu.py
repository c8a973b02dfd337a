"""CPU-only checks of the oracle: the reference's own known-answer tests, the golden vectors,
and internal consistency of the restated third-party arithmetic."""
import math
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"


def test_exp_se2_known_answers(oracle):
    # feature_tracker/src/feature_tracker/feature_tracking.rs:264-291 (crate twist [theta, vx, vy];
    # the main crate's se2_exp_matrix takes [vx, vy, theta], image_utilities.rs:82-106)
    tol = 1e-6
    E = oracle.se2_exp([0.0, 0.0, 0.0])
    assert np.allclose(E, np.eye(3), atol=tol)
    E = oracle.se2_exp([0.0, 0.0, math.pi])
    assert np.allclose(E[:2, :2], [[-1, 0], [0, -1]], atol=tol) and np.allclose(E[:2, 2], 0, atol=tol)
    E = oracle.se2_exp([1.32, -1.56, 0.0])
    assert np.allclose(E[:2, :2], np.eye(2), atol=tol) and np.allclose(E[:2, 2], [1.32, -1.56], atol=tol)
    # exp/log round trip property at the crate's twists (closed-form SE(2) log)
    for th, vx, vy in [(math.pi / 3, 1.0, 2.5), (1.795, 1.0, 2.5), (1e-8, 1.0, 2.5), (1e-7, 1.0, 2.5),
                       (2e-7, 1.0, 2.5)]:
        E = oracle.se2_exp([vx, vy, th]).astype(np.float64)
        t = math.atan2(E[1, 0], E[0, 0])
        half = t / 2
        diag = half / math.tan(half) if abs(t) > 1e-3 else 1 - t * t / 12
        v = np.array([[diag, half], [-half, diag]]) @ E[:2, 2]
        assert abs(t - th) < 1e-6 and np.allclose(v, [vx, vy], atol=1e-5)


def test_pyramid_dimensions(oracle):
    # feature_tracker/src/image_operations.rs:84-94: 120x60 -> 60x30 -> 30x15
    assert oracle.pyramid_bytes(120, 60, 3) == 120 * 60 + 60 * 30 + 30 * 15
    pyr = oracle.build_pyramid(np.zeros((60, 120), np.uint8), 3)
    assert pyr.size == 120 * 60 + 60 * 30 + 30 * 15


def test_triangle_resize_weights(oracle):
    # ratio 2 -> taps [1/8, 3/8, 3/8, 1/8]; a vertical impulse shows them
    img = np.zeros((16, 16), np.uint8)
    img[8, :] = 200
    out = oracle.resize_triangle(img, 16, 8)
    col = out[:, 3].astype(float)
    # output row 4 covers input rows 7..10 (row 8 weight 3/8); row 3 covers rows 5..8 (1/8)
    assert col[4] == round(200 * 3 / 8) and col[3] == round(200 * 1 / 8) and col[5] == 0 and col[2] == 0
    # identity size is a copy; constant image stays constant
    assert np.array_equal(oracle.resize_triangle(img, 16, 16), img)
    assert np.all(oracle.resize_triangle(np.full((30, 40), 93, np.uint8), 13, 7) == 93)


def _fast_closed_form(img, t):
    """score = max over 9-arcs of min |I_p - I_c| - 1 (used by the GPU kernel)."""
    im = img.astype(np.int32)
    h, w = im.shape
    off = [(0, -3), (1, -3), (2, -2), (3, -1), (3, 0), (3, 1), (2, 2), (1, 3), (0, 3), (-1, 3),
           (-2, 2), (-3, 1), (-3, 0), (-3, -1), (-2, -2), (-1, -3)]
    c = im[3:h - 3, 3:w - 3]
    d = np.stack([im[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] - c for dx, dy in off])
    d2 = np.concatenate([d, d[:8]])
    sb = np.max(np.stack([d2[a:a + 9].min(0) for a in range(16)]), 0)
    sd = np.max(np.stack([(-d2[a:a + 9]).min(0) for a in range(16)]), 0)
    s = np.maximum(sb, sd) - 1
    out = np.zeros((h, w), np.int32)
    out[3:h - 3, 3:w - 3] = np.where(s >= t, s, 0)
    return out


@pytest.mark.parametrize("t", [10, 20, 40])
def test_fast9_binary_search_equals_closed_form(oracle, t):
    rng = np.random.default_rng(t)
    img = rng.integers(0, 256, (70, 90), dtype=np.uint8)
    img[20:40, 20:40] = 30
    img[25:35, 25:35] = 220
    ref = oracle.fast9_scores(img, t).astype(np.int32)
    assert np.array_equal(ref, _fast_closed_form(img, t))


def test_golden_tracker_reproduced(oracle):
    g = np.load(GOLD / "tracker_small.npz", allow_pickle=False)
    w, h, L = int(g["w"]), int(g["h"]), int(g["levels"])
    assert np.array_equal(oracle.build_pyramid(g["left"][0], L), g["pyr_l0"])
    assert np.array_equal(oracle.build_pyramid(g["noise_img"], 5), g["pyr_noise5"])
    a, v = oracle.track_points(g["pyr_l0"], g["pyr_l1"], w, h, L, g["aff"])
    assert np.array_equal(v, g["t_valid"].astype(bool)) and np.array_equal(a, g["t_aff"])
    xy, sc = oracle.detect_key_points(g["left"][0], 30, None)
    assert np.array_equal(xy, g["det_xy"]) and np.array_equal(sc, g["det_score"])


def test_track_recovers_translation(oracle):
    # an integer shift of a textured image is recovered to well below a pixel
    from rsvio import synthetic as S
    tex = S.make_texture(200, 160, n_blobs=1500, seed=4)
    img = S._render(tex, 200, 160, 0, False, np.zeros((160, 200)))
    shifted = np.zeros_like(img)
    shifted[:, 2:] = img[:, :-2]
    p0, p1 = oracle.build_pyramid(img, 3), oracle.build_pyramid(shifted, 3)
    aff = S.track_features(img, 20, spacing=15.0)
    aff = aff[(aff[:, 4] > 30) & (aff[:, 4] < 170) & (aff[:, 5] > 30) & (aff[:, 5] < 130)]
    out, valid = oracle.track_points(p0, p1, 200, 160, 3, aff)
    assert valid.mean() > 0.8
    d = out[valid, 4:6] - aff[valid, 4:6]
    assert np.abs(np.median(d[:, 0]) - 2.0) < 0.05 and np.abs(np.median(d[:, 1])) < 0.05


def test_stereo_tracker_canonical_ids(oracle):
    g = np.load(GOLD / "tracker_small.npz", allow_pickle=False)
    tr = oracle.StereoTracker(int(g["w"]), int(g["h"]), 3, 30, 20, 0.01)
    ids_seen = []
    for k in range(4):
        fl, fr = tr.process_frame(g["left"][k], g["right"][k])
        ids = [f[0] for f in fl]
        assert ids == sorted(ids) and len(set(ids)) == len(ids)
        ids_seen.append(set(ids))
    # ids are never reused
    assert max(max(s) for s in ids_seen if s) < 10_000


def test_threaded_oracle_legs_match_sequential(oracle):
    """The all-cores CPU baseline legs: the threaded Schur BA (landmark ranges summed in range
    order) is tolerance-equal to the sequential reference order, and the threaded tracker
    (pyramid levels and features in parallel) is bit-identical."""
    from rsvio import synthetic as S
    prob = S.ba_problem(n_kf=6, n_lm=300, kf_per_lm=4, seed=21, init_seed=22)
    p1, w1, r1 = oracle.ba_solve(prob)
    oracle.set_ba_threads(4)
    try:
        p4, w4, r4 = oracle.ba_solve(prob)
    finally:
        oracle.set_ba_threads(1)
    assert (r1.status, r1.iterations) == (r4.status, r4.iterations)
    assert np.abs(p1 - p4).max() < 1e-9 and np.abs(w1 - w4).max() < 1e-8
    frames = list(S.stereo_sequence(2, 320, 240))
    outs = []
    for threads in (1, 4):
        t = oracle.StereoTracker(320, 240, 3, 30, 20, 0.01, threads=threads)
        outs.append([t.process_frame(l, r) for l, r in frames])
    assert outs[0] == outs[1]


def test_oracle_solve_reproduces_the_ba_golden():
    """tests/golden/ba_small.npz (made by tests/golden/make_golden.py from this oracle): the oracle
    still solves it to the same status, iteration count and bits -- the golden pins the oracle's
    LM against drift on CPU, as test_ba_gpu pins the device against it."""
    from pathlib import Path
    from types import SimpleNamespace

    import numpy as np

    from oracle import oracle as O
    g = np.load(Path(__file__).resolve().parent / "golden" / "ba_small.npz", allow_pickle=False)
    prob = SimpleNamespace(**{k: g[k] for k in ("pose7", "kf_fixed", "p_W", "obs_lm", "obs_kf", "obs_cam",
                                                 "obs_uv", "T_C_B2")})
    po, pwo, ro = O.ba_solve(prob)
    assert (ro.status, ro.iterations) == (int(g["status"]), int(g["iterations"]))
    assert np.array_equal(po, g["sol_pose7"]) and np.array_equal(pwo, g["sol_p_W"])
    assert ro.final_cost == float(g["final_cost"])
