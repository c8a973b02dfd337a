"""B8 on the GPU: rsvio_track_motion / rsvio_track_motion_tracker (one single-workgroup launch
per frame) against the oracle's restatement of SlidingWindow::track_motion + the keyframe rule.

Parity: integer outcomes (status, iterations, observation count, keyframe flag) are equal;
poses and costs agree to 1e-9 -- the GPU sums H, g and the cost in a fixed tree order, the
oracle sequentially, so f64 rounding differs in the last bits.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-9


def _oracle(oracle, m, **kw):
    return oracle.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.map_ids, m.map_pw, m.T_W_B_last_kf, m.T_C_B2,
                               **kw)


def _check(r, o):
    assert (r.status, r.iterations, r.n_observations, int(r.is_keyframe)) == \
        (o.status, o.iterations, o.n_observations, o.is_keyframe)
    To = np.array(o.T_W_B[:]).reshape(4, 4)
    assert np.abs(r.T_W_B - To).max() <= POSE_TOL
    for a, b in ((r.initial_cost, o.initial_cost), (r.final_cost, o.final_cost)):
        assert abs(a - b) <= 1e-9 * max(1.0, abs(b))
    assert abs(r.translation_norm - o.translation_norm) <= 1e-9
    assert abs(r.rotation_norm - o.rotation_norm) <= 1e-9
    assert 0.0 < r.kernel_ms < 100.0  # the launch's own device time (wall clock), a one-workgroup LM


@pytest.fixture(scope="module")
def motion(gpu):
    from rsvio.motion import MotionTracker
    mt = MotionTracker()
    yield mt
    mt.close()


@pytest.mark.parametrize("seed,step,outliers", [(1, (0.03, 0.017), 0.0), (2, (0.09, 0.005), 0.0),
                                                 (3, (0.01, 0.07), 0.0), (7, (0.03, 0.017), 0.05)])
def test_track_motion_matches_oracle(motion, oracle, seed, step, outliers):
    from rsvio import synthetic as S
    m = S.motion_frame(seed=seed, step=step, outlier_frac=outliers)
    motion.set_map(m.map_ids, m.map_pw)
    r = motion.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.T_W_B_last_kf, m.T_C_B2)
    _check(r, _oracle(oracle, m))
    assert r.success


def test_track_motion_thresholds_and_large_map(motion, oracle):
    """A map larger than the LDS-staged join (global binary search) and the TUM-VI thresholds."""
    from rsvio import synthetic as S
    from rsvio.motion import MotionTracker
    m = S.motion_frame(seed=11, n_map=9000, n_feat=800, step=(0.2, math.radians(10)))
    lax = MotionTracker(translation_threshold=0.4, rotation_threshold=0.25)
    try:
        lax.set_map(m.map_ids, m.map_pw)
        r = lax.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.T_W_B_last_kf, m.T_C_B2)
        _check(r, _oracle(oracle, m, thr_t=0.4, thr_r=0.25))
        assert r.n_observations > 1500
    finally:
        lax.close()


def test_track_motion_failure_and_limits(motion, oracle):
    from rsvio import RsvioError
    from rsvio import synthetic as S
    m = S.motion_frame(seed=12)
    motion.set_map(m.map_ids, m.map_pw)
    # no feature in the map: failed optimisation, keyframe at identity
    off = np.uint64(10 ** 9)
    r = motion.track_motion(m.ids_l + off, m.uv_l, m.ids_r + off, m.uv_r, m.T_W_B_last_kf, m.T_C_B2)
    o = oracle.track_motion(m.ids_l + off, m.uv_l, m.ids_r + off, m.uv_r, m.map_ids, m.map_pw, m.T_W_B_last_kf,
                            m.T_C_B2)
    _check(r, o)
    assert r.is_keyframe and np.array_equal(r.T_W_B, np.eye(4))
    # empty frame
    e = np.zeros(0, np.uint64)
    r = motion.track_motion(e, np.zeros((0, 2)), e, np.zeros((0, 2)), m.T_W_B_last_kf, m.T_C_B2)
    assert r.status == -2 and r.is_keyframe
    # more than 4096 features in one frame
    big = np.arange(5000, dtype=np.uint64)
    with pytest.raises(RsvioError):
        motion.track_motion(big, np.zeros((5000, 2)), e, np.zeros((0, 2)), m.T_W_B_last_kf, m.T_C_B2)
    # map ids must be ascending (the wrapper sorts; the ABI checks)
    import ctypes as C

    from rsvio import _lib
    ids = np.array([5, 3], np.uint64)
    pw = np.zeros((2, 3), np.float32)
    assert _lib.load().rsvio_pnp_set_map(motion._h, ids.ctypes.data, pw.ctypes.data, 2) == -1
    assert C.sizeof(_lib.MotionResult) == 184


def test_track_motion_from_the_tracker(gpu, oracle, stereo_frames):
    """Tracker -> fused unprojection -> PnP + keyframe rule on the device: the result equals
    the oracle's on the same (ids, undistorted coordinates) read back from the tracker."""
    from rsvio import synthetic as S
    from rsvio.camera import EUROC
    from rsvio.motion import MotionTracker
    trk = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50)
    trk.set_cameras(*EUROC)
    mt = MotionTracker()
    try:
        trk.process_frame(*stereo_frames[0])
        fl, fr = trk.process_frame(*stereo_frames[1])
        ul, ur = trk.undistorted()
        # a map for the tracked ids: points 4 m along the left rays of the last keyframe
        T_last = np.eye(4)
        T_C_B2 = np.stack([np.linalg.inv(S.T_B_CL).reshape(16), np.linalg.inv(S.T_B_CR).reshape(16)])
        T_B_C = S.T_B_CL
        ids = fl["id"].astype(np.uint64)
        rays = np.concatenate([ul.astype(np.float64), np.ones((len(ul), 1))], 1) * 4.0
        p_W = (T_B_C[:3, :3] @ rays.T).T + T_B_C[:3, 3]
        keep = np.arange(len(ids)) % 3 != 0          # a third of the tracks are not in the map
        mt.set_map(ids[keep], p_W[keep].astype(np.float32))
        r = mt.track_motion_tracker(trk, T_last, T_C_B2)
        o = oracle.track_motion(ids, ul, fr["id"].astype(np.uint64), ur, ids[keep],
                                p_W[keep].astype(np.float32), T_last, T_C_B2)
        _check(r, o)
        assert r.n_observations > 100
        # the host-array entry point on the same inputs gives the same result
        r2 = mt.track_motion(ids, ul, fr["id"], ur, T_last, T_C_B2)
        _check(r2, o)
    finally:
        mt.close()
        trk.close()


def test_track_motion_reads_the_collected_frame_while_the_next_tracks(gpu, oracle, stereo_frames):
    """The Estimator's look-ahead (rsvio_tracker_submit / _collect): with frame t + 1 submitted
    (in flight or done on the tracker's stream), rsvio_track_motion_tracker still reads frame t's
    output slot -- the same result as before the submit -- and after frame t + 1 is collected it
    reads frame t + 1's; both equal the oracle on the lists read back.  One frame in flight per
    handle: a second submit, a process_frame, remove_ids or set_cameras while one is, and a collect
    without one, are refused."""
    from rsvio import RsvioError
    from rsvio import synthetic as S
    from rsvio.camera import EUROC
    from rsvio.motion import MotionTracker
    trk = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50)
    trk.set_cameras(*EUROC)
    mt = MotionTracker()
    T_last = np.eye(4)
    T_C_B2 = np.stack([np.linalg.inv(S.T_B_CL).reshape(16), np.linalg.inv(S.T_B_CR).reshape(16)])

    def frame_map(fl, ul):
        ids = fl["id"].astype(np.uint64)
        rays = np.concatenate([ul.astype(np.float64), np.ones((len(ul), 1))], 1) * 4.0
        p_W = (S.T_B_CL[:3, :3] @ rays.T).T + S.T_B_CL[:3, 3]
        return ids, p_W.astype(np.float32)

    try:
        trk.submit(*stereo_frames[0])
        with pytest.raises(RsvioError):
            trk.submit(*stereo_frames[1])
        with pytest.raises(RsvioError):
            trk.process_frame(*stereo_frames[1])
        trk.collect()
        with pytest.raises(RsvioError):
            trk.collect()
        trk.submit(*stereo_frames[1])
        fl, fr = trk.collect()
        ul, ur = trk.undistorted()
        ids, p_W = frame_map(fl, ul)
        mt.set_map(ids, p_W)
        r_before = mt.track_motion_tracker(trk, T_last, T_C_B2)
        o = oracle.track_motion(ids, ul, fr["id"].astype(np.uint64), ur, ids, p_W, T_last, T_C_B2)
        _check(r_before, o)
        trk.submit(*stereo_frames[2])                      # frame t + 1 in flight
        for call in (lambda: trk.remove_id(fl["id"][:1]), lambda: trk.set_cameras(*EUROC)):
            with pytest.raises(RsvioError):
                call()
        r_during = mt.track_motion_tracker(trk, T_last, T_C_B2)
        assert np.array_equal(r_during.T_W_B, r_before.T_W_B)
        assert (r_during.status, r_during.iterations, r_during.n_observations) == \
               (r_before.status, r_before.iterations, r_before.n_observations)
        import torch
        torch.cuda.synchronize()  # the submitted frame's read-back copies have landed by now
        # undistorted() is still the collected frame's: the in-flight frame copied into the other slot
        assert all(np.array_equal(a, b) for a, b in zip(trk.undistorted(), (ul, ur)))
        fl2, fr2 = trk.collect()
        ul2, ur2 = trk.undistorted()
        r_after = mt.track_motion_tracker(trk, T_last, T_C_B2)
        o2 = oracle.track_motion(fl2["id"].astype(np.uint64), ul2, fr2["id"].astype(np.uint64), ur2, ids, p_W,
                                 T_last, T_C_B2)
        _check(r_after, o2)
        # the look-ahead's lists equal process_frame's on a fresh tracker
        ref = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50)
        ref.set_cameras(*EUROC)
        for f in stereo_frames[:2]:
            ref.process_frame(*f)
        gl, gr = ref.process_frame(*stereo_frames[2])
        assert np.array_equal(gl, fl2) and np.array_equal(gr, fr2)
        assert all(np.array_equal(a, b) for a, b in zip(ref.undistorted(), (ul2, ur2)))
        ref.close()
    finally:
        mt.close()
        trk.close()
