"""Estimator host logic (estimator.rs:101-262 over sliding_window.rs:174-300) on CPU.

* `SlidingWindow.build_problem` (vectorised) against a per-observation loop restatement of
  sliding_window.rs:174-300 -- landmark selection (seen left and right in the window), first-
  appearance indexing, map_points vs depth-2.0 ray initialisation, f32 coordinates.
* The Estimator over the oracle backend on config 4's rendered stream: keyframe
  cadence, PnP / BA outcomes and the trajectory against the rendering's true poses.
"""
import numpy as np
import pytest

from rsvio.ba import Frame, SlidingWindow
from rsvio.synthetic import T_B_CL, T_B_CR


def _loop_build(kfs, map_points):
    """sliding_window.rs:174-300 restated observation by observation."""
    T_Cl_B = np.linalg.inv(kfs[0].T_B_Cl)
    T_Cr_B = np.linalg.inv(kfs[0].T_B_Cr)
    cnt_l, cnt_r = {}, {}
    for f in kfs:
        for fid, _ in f.left_features:
            cnt_l[fid] = cnt_l.get(fid, 0) + 1
        for fid, _ in f.right_features:
            cnt_r[fid] = cnt_r.get(fid, 0) + 1
    index, p_init, lm, kf, cam, uv = {}, [], [], [], [], []
    for i, f in enumerate(kfs):
        for c, (feats, T_C_B) in enumerate(((f.left_features, T_Cl_B), (f.right_features, T_Cr_B))):
            for fid, xy in feats:
                if not cnt_l.get(fid) or not cnt_r.get(fid):
                    continue
                x, y = float(np.float32(xy[0])), float(np.float32(xy[1]))
                if fid not in index:
                    index[fid] = len(p_init)
                    if fid in map_points:
                        p_init.append(np.asarray(map_points[fid], np.float32).astype(np.float64))
                    else:
                        T_B_C = np.linalg.inv(T_C_B)
                        p_B = T_B_C[:3, :3] @ np.array([x, y, 2.0]) + T_B_C[:3, 3]
                        p_init.append(f.T_W_B[:3, :3] @ p_B + f.T_W_B[:3, 3])
                lm.append(index[fid])
                kf.append(i)
                cam.append(c)
                uv.append([x, y])
    return np.array(p_init).reshape(-1, 3), np.array(lm), np.array(kf), np.array(cam), np.array(uv).reshape(-1, 2), \
        sorted(index, key=index.get)


def _random_window(rng, n_kf=6, n_ids=120):
    sw = SlidingWindow(n_kf, solver=object())
    for k in range(n_kf):
        T = np.eye(4)
        T[:3, 3] = rng.normal(0, 0.2, 3)
        c, s = np.cos(0.1 * k), np.sin(0.1 * k)
        T[:2, :2] = [[c, -s], [s, c]]
        feats = []
        for cam in range(2):
            ids = np.sort(rng.choice(n_ids, rng.integers(20, 60), replace=False))
            feats.append([(int(i), tuple(rng.normal(0, 0.3, 2))) for i in ids])
        sw.add_frame(Frame(frame_id=k, T_W_B=T, T_B_Cl=T_B_CL, T_B_Cr=T_B_CR, left_features=feats[0],
                           right_features=feats[1]))
    return sw


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_build_problem_matches_loop(seed):
    rng = np.random.default_rng(seed)
    sw = _random_window(rng)
    sw.map_points = {int(i): rng.normal(0, 3, 3).astype(np.float32) for i in rng.choice(120, 50, replace=False)}
    pose7, fixed, p_init, lm, kf, cam, uv, tcb, ids = sw.build_problem()
    p_ref, lm_ref, kf_ref, cam_ref, uv_ref, ids_ref = _loop_build(list(sw.keyframes), sw.map_points)
    assert [int(x) for x in ids] == ids_ref
    assert np.array_equal(lm, lm_ref) and np.array_equal(kf, kf_ref) and np.array_equal(cam, cam_ref)
    assert np.array_equal(uv, uv_ref)
    assert np.abs(p_init - p_ref).max() <= 1e-12
    assert fixed.tolist() == [1] + [0] * (len(sw.keyframes) - 1)
    assert pose7.shape == (len(sw.keyframes), 7)


def test_build_problem_array_features_equal_pairs():
    rng = np.random.default_rng(5)
    sw = _random_window(rng)
    a = sw.build_problem()
    for f in sw.keyframes:
        for name in ("left_features", "right_features"):
            pairs = getattr(f, name)
            setattr(f, name, (np.array([p[0] for p in pairs], np.int64), np.array([p[1] for p in pairs])))
    b = sw.build_problem()
    for x, y in zip(a[:-1], b[:-1]):
        assert np.array_equal(x, y)
    assert np.array_equal(a[-1], b[-1])


@pytest.mark.slow
def test_estimator_oracle_pipeline(oracle, scene_stream):
    """Config 4's host logic over the oracle: the window fills, PnP tracks every later frame,
    a keyframe every few frames (0.02 m/frame against the 0.05 m threshold) and the tracked
    trajectory stays within 1 cm of the rendering's true poses."""
    from oracle.estimator import OracleBackend
    from rsvio.camera import Camera
    from rsvio.estimator import Estimator
    s, win = scene_stream
    cams = [Camera.opencv5(*p) for p in s.intrinsics]
    w = s.frames[0][0].shape[1]
    h = s.frames[0][0].shape[0]
    est = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=win, backend=OracleBackend(oracle, w, h, cams))
    out = [est.process_frame(l, r) for l, r in s.frames]
    assert all(r.n_left > 30 and r.n_right > 30 for r in out)
    assert [r.is_keyframe for r in out[:win]] == [True] * win
    assert out[win - 1].ba_status is not None and out[win - 1].ba_status > 0
    tracked = out[win:]
    assert all(r.pnp_status is not None and r.pnp_status > 0 for r in tracked)
    kf = [r.is_keyframe for r in tracked]
    assert 0.2 <= np.mean(kf) <= 0.6
    assert all(r.ba_status > 0 for r in tracked if r.is_keyframe)
    err = [np.linalg.norm(r.T_W_B[:3, 3] - T[:3, 3]) for r, T in zip(tracked, s.T_W_B[win:])]
    assert max(err) < 0.01


class _DeferredSolver:
    """The oracle solver behind the asynchronous interface SlidingWindow.optimize_async uses
    (set_problem / run_async / wait / state); the solve happens at wait()."""

    def __init__(self, solver):
        self.s = solver
        self.in_flight = 0

    def solve(self, *a, **k):
        return self.s.solve(*a, **k)

    def set_problem(self, *a):
        assert self.in_flight == 0
        self.args = a

    def run_async(self, cfg=None):
        self.cfg, self.in_flight = cfg, 1

    def wait(self):
        assert self.in_flight == 1
        self.in_flight = 0
        self.pose, self.pw, res = self.s.solve(*self.args, self.cfg)
        return res

    def state(self):
        return self.pose, self.pw


def test_estimator_pipelined_equals_sequential(oracle, scene_stream):
    """Pipelined mode (a keyframe's BA completes during the next frame's tracking): every frame
    result (after flush), the trajectory and the map equal the sequential order's exactly."""
    from oracle.estimator import OracleBackend
    from rsvio.camera import Camera
    from rsvio.estimator import Estimator
    s, win = scene_stream
    cams = [Camera.opencv5(*p) for p in s.intrinsics]
    h, w = s.frames[0][0].shape
    seq = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=win, backend=OracleBackend(oracle, w, h, cams))
    be = OracleBackend(oracle, w, h, cams)
    be.solver = _DeferredSolver(be.solver)
    pip = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=win, backend=be, pipelined=True)
    a = [seq.process_frame(l, r) for l, r in s.frames]
    b = []
    deferred = 0
    for l, r in s.frames:
        b.append(pip.process_frame(l, r))
        deferred += be.solver.in_flight
        if b[-1].is_keyframe and len(pip.window) == win:
            assert b[-1].ba_status is None or be.solver.in_flight == 0
    pip.flush()
    assert deferred > 0
    for x, y in zip(a, b):
        assert (x.is_keyframe, x.pnp_status, x.ba_status, x.n_left, x.n_right, x.pnp_iterations, x.ba_iterations) == \
               (y.is_keyframe, y.pnp_status, y.ba_status, y.n_left, y.n_right, y.pnp_iterations, y.ba_iterations)
        assert np.array_equal(x.T_W_B, y.T_W_B)
    for Ta, Tb in zip(seq.trajectory(), pip.trajectory()):
        assert np.array_equal(Ta, Tb)
    ma, mb = seq.window.map_points, pip.window.map_points
    assert sorted(ma) == sorted(mb) and all(np.array_equal(ma[i], mb[i]) for i in ma)


class _OrderSpy:
    """Records the order of the backend calls the Estimator makes."""

    def __init__(self, be):
        self.be, self.solver, self.log = be, be.solver, []

    def submit(self, l, r):
        self.log.append("submit")
        return self.be.submit(l, r)

    def collect(self):
        self.log.append("collect")
        return self.be.collect()

    def track_motion(self, *a):
        self.log.append("pnp")
        return self.be.track_motion(*a)

    def __getattr__(self, k):
        return getattr(self.be, k)


def test_estimator_lookahead_equals_sequential(oracle, scene_stream):
    """Estimator.run: the tracker one frame ahead (frame t + 1 submitted right after frame t's
    features are collected, before frame t's PnP and BA), pipelined BA on top: every frame result
    -- statuses and LM iteration counts included -- the trajectory and the map equal the
    sequential process_frame order's exactly, and the call order is the look-ahead's."""
    from oracle.estimator import OracleBackend
    from rsvio.camera import Camera
    from rsvio.estimator import Estimator
    s, win = scene_stream
    cams = [Camera.opencv5(*p) for p in s.intrinsics]
    h, w = s.frames[0][0].shape
    seq = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=win, backend=OracleBackend(oracle, w, h, cams))
    a = [seq.process_frame(l, r) for l, r in s.frames]
    be = OracleBackend(oracle, w, h, cams)
    be.solver = _DeferredSolver(be.solver)
    spy = _OrderSpy(be)
    la = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=win, backend=spy, pipelined=True)
    b = list(la.run(s.frames))
    la.flush()
    assert len(b) == len(a)
    for x, y in zip(a, b):
        assert (x.is_keyframe, x.pnp_status, x.ba_status, x.n_left, x.n_right, x.pnp_iterations, x.ba_iterations) == \
               (y.is_keyframe, y.pnp_status, y.ba_status, y.n_left, y.n_right, y.pnp_iterations, y.ba_iterations)
        assert np.array_equal(x.T_W_B, y.T_W_B)
    for Ta, Tb in zip(seq.trajectory(), la.trajectory()):
        assert np.array_equal(Ta, Tb)
    ma, mb = seq.window.map_points, la.window.map_points
    assert sorted(ma) == sorted(mb) and all(np.array_equal(ma[i], mb[i]) for i in ma)
    # the look-ahead: submit(0), then per frame t: collect(t), submit(t + 1), [pnp(t)]
    log = [e for e in spy.log]
    assert log[:3] == ["submit", "collect", "submit"]
    first_pnp = log.index("pnp")
    assert log[first_pnp - 2:first_pnp] == ["collect", "submit"]
    assert log.count("submit") == log.count("collect") == len(s.frames)
    # an early stop leaves no frame in flight
    la2 = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=win, backend=OracleBackend(oracle, w, h, cams))
    g = la2.run(s.frames)
    next(g)
    g.close()
    assert la2.backend._submitted is None
