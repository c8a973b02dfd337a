"""GPU parity of the sliding-window BA (HP-B) against the f64 CPU oracle, through the C ABI.

Tolerances (f64; the GPU sums per camera block and per landmark in a fixed tree order, the
oracle sequentially): reduced camera system S, b within 1e-9 of max|S| / max|b|; cost within
1e-10 relative; solved poses within 1e-7 and landmarks within 1e-6 m; identical LM status and
iteration count.
"""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def cfg3():
    from rsvio import synthetic as S
    return S.ba_problem()  # config 3: 10 KF x 2000 landmarks, 24,000 observations


def _adjuster(gpu, prob):
    from rsvio.ba import BundleAdjuster
    ba = BundleAdjuster(max_keyframes=21, max_landmarks=max(prob.n_lm, 1), max_observations=max(prob.n_obs, 1))
    ba.set_problem_from(prob)
    return ba


def test_config3_shape(cfg3):
    assert cfg3.n_kf == 10 and cfg3.n_lm == 2000 and cfg3.n_obs == 24000


@pytest.mark.parametrize("lam", [1e-4, 1.0])
def test_reduced_system_matches_oracle(gpu, oracle, cfg3, lam):
    ba = _adjuster(gpu, cfg3)
    S, b, cost = ba.build_system(lam)
    So, bo, co = oracle.ba_build_system(cfg3, lam)
    assert S.shape == (54, 54)
    assert np.abs(S - So).max() <= 1e-9 * np.abs(So).max()
    assert np.abs(b - bo).max() <= 1e-9 * np.abs(bo).max()
    assert abs(cost - co) <= 1e-10 * abs(co)
    assert np.allclose(S, S.T, rtol=0, atol=1e-12 * np.abs(S).max())


def test_golden_system_and_solve(gpu):
    g = np.load(GOLD / "ba_small.npz", allow_pickle=False)
    from rsvio.ba import BundleAdjuster
    ba = BundleAdjuster(max_keyframes=8, max_landmarks=100, max_observations=1000)
    ba.set_problem(g["pose7"], g["kf_fixed"], g["p_W"], g["obs_lm"], g["obs_kf"], g["obs_cam"], g["obs_uv"], g["T_C_B2"])
    S, b, cost = ba.build_system(1e-4)
    assert np.abs(S - g["S"]).max() <= 1e-9 * np.abs(g["S"]).max()
    assert np.abs(b - g["b"]).max() <= 1e-9 * np.abs(g["b"]).max()
    res = ba.run()
    pose, pw = ba.state()
    assert res.status == int(g["status"]) and res.iterations == int(g["iterations"])
    assert np.abs(pose - g["sol_pose7"]).max() < 1e-7
    assert np.abs(pw - g["sol_p_W"]).max() < 1e-6
    assert abs(res.final_cost - float(g["final_cost"])) <= 1e-6 * float(g["initial_cost"])


def test_solve_matches_oracle_config3(gpu, oracle, cfg3):
    ba = _adjuster(gpu, cfg3)
    res = ba.run()
    pose, pw = ba.state()
    po, pwo, ro = oracle.ba_solve(cfg3)
    assert res.status == ro.status and res.iterations == ro.iterations
    assert res.status > 0
    assert abs(res.initial_cost - ro.initial_cost) <= 1e-10 * ro.initial_cost
    assert abs(res.final_cost - ro.final_cost) <= 1e-8 * ro.initial_cost
    assert np.abs(pose - po).max() < 1e-7
    assert np.abs(pw - pwo).max() < 1e-6
    # and it actually optimised: cost drops and poses approach the truth
    assert res.final_cost < 0.1 * res.initial_cost
    err0 = np.abs(cfg3.pose7[1:, :3] - cfg3.true_pose7[1:, :3]).max()
    err1 = np.abs(pose[1:, :3] - cfg3.true_pose7[1:, :3]).max()
    assert err1 < 0.5 * err0


def test_solve_is_deterministic(gpu, cfg3):
    ba = _adjuster(gpu, cfg3)
    r1 = ba.run()
    s1 = ba.state()
    r2 = ba.run()
    s2 = ba.state()
    assert r1.iterations == r2.iterations and r1.final_cost == r2.final_cost
    assert np.array_equal(s1[0], s2[0]) and np.array_equal(s1[1], s2[1])


def test_noise_free_converges_to_truth(gpu):
    # the reference's only numeric BA assertion (src/optimization/tests.rs:335-379): landmark error < 1e-3
    from rsvio import synthetic as S
    prob = S.ba_problem(n_kf=5, n_lm=60, kf_per_lm=5, seed=21, noise_px=0.0, init_seed=22)
    ba = _adjuster(gpu, prob)
    from rsvio.ba import lm_cfg
    res = ba.run(lm_cfg(max_iterations=50))
    pose, pw = ba.state()
    assert res.status in (1, 2, 3)
    assert np.linalg.norm(pw - prob.true_p_W, axis=1).max() < 1e-3
    assert np.abs(pose[:, :3] - prob.true_pose7[:, :3]).max() < 1e-4


def test_cheirality_and_skip(gpu, oracle):
    from rsvio import synthetic as S
    prob = S.ba_problem(n_kf=3, n_lm=20, kf_per_lm=2, seed=5, init_seed=6)
    prob.p_W[0] = -prob.p_W[0] * 5.0  # push one landmark behind the cameras
    ba = _adjuster(gpu, prob)
    S_, b, cost = ba.build_system(1e-4)
    So, bo, co = oracle.ba_build_system(prob, 1e-4)
    assert abs(cost - co) <= 1e-10 * co and cost > 1e6  # [1e6, 1e6] residuals under Huber(2)
    assert np.abs(S_ - So).max() <= 1e-9 * np.abs(So).max()
    r = ba.run()
    po, pwo, ro = oracle.ba_solve(prob)
    assert r.status == ro.status and r.iterations == ro.iterations
    # sliding_window.rs:309-319: too few residuals -> skipped, state untouched
    tiny = S.ba_problem(n_kf=2, n_lm=1, kf_per_lm=1, seed=1)
    ba2 = _adjuster(gpu, tiny)
    r2 = ba2.run()
    assert r2.status == -2


def test_config5_shape_matches_oracle(gpu, oracle):
    from rsvio import synthetic as S
    prob = S.ba_problem(n_kf=20, n_lm=5000, kf_per_lm=8, seed=55, init_seed=56)
    assert prob.n_obs == 80000
    ba = _adjuster(gpu, prob)
    S_, b, cost = ba.build_system(1e-4)
    So, bo, co = oracle.ba_build_system(prob, 1e-4)
    assert S_.shape == (114, 114)
    assert np.abs(S_ - So).max() <= 1e-9 * np.abs(So).max()
    res = ba.run()
    pose, pw = ba.state()
    po, pwo, ro = oracle.ba_solve(prob)
    assert res.status == ro.status and res.iterations == ro.iterations
    assert np.abs(pose - po).max() < 1e-7 and np.abs(pw - pwo).max() < 1e-6


def test_sliding_window_mirror(gpu, oracle):
    from rsvio import synthetic as S
    from rsvio.ba import Frame, SlidingWindow
    prob = S.ba_problem(n_kf=4, n_lm=50, kf_per_lm=4, seed=8, init_seed=9)
    frames = []
    for k in range(prob.n_kf):
        T_B_W = np.eye(4)
        T_B_W[:3, :3] = S.rot_from_quat(prob.true_pose7[k, 3:])
        T_B_W[:3, 3] = prob.true_pose7[k, :3]
        fr = Frame(frame_id=k, T_W_B=np.linalg.inv(T_B_W), T_B_Cl=S.T_B_CL, T_B_Cr=S.T_B_CR)
        for o in np.nonzero(prob.obs_kf == k)[0]:
            (fr.left_features if prob.obs_cam[o] == 0 else fr.right_features).append(
                (int(prob.obs_lm[o]), tuple(prob.obs_uv[o])))
        frames.append(fr)
    sw = SlidingWindow(4)
    for fr in frames[:3]:
        sw.add_frame(fr)
    with pytest.raises(RuntimeError):
        sw.optimize()
    sw.add_frame(frames[3])
    assert sw.is_full()
    assert sw.optimize()
    assert len(sw.map_points) == 50
    assert sw.last_result.status > 0
    # second solve starts from the f32 map points (sliding_window.rs:249-254)
    assert sw.optimize()


@pytest.mark.parametrize("n_kf", [3, 11, 12, 14, 17, 20, 21])
def test_camera_solve_matches_dense_solve(gpu, n_kf):
    """K5 alone: dc of S dc = b for every solve variant (one row per lane up to 10 free keyframes,
    two rows per lane padded to 13 / 16 / 20 above), repeated (a publication race would show as a
    run-to-run difference), against numpy's dense solve of the same S, b (tolerance 1e-9 relative)."""
    from rsvio import synthetic as S
    prob = S.ba_problem(n_kf=n_kf, n_lm=40 * n_kf, kf_per_lm=min(n_kf, 4), seed=100 + n_kf, init_seed=200 + n_kf)
    ba = _adjuster(gpu, prob)
    S_, b, _ = ba.build_system(1e-4)
    ref = np.linalg.solve(S_, b)
    first = None
    for _ in range(4):
        dc = ba.camera_step(1e-4)
        assert np.abs(dc - ref).max() <= 1e-9 * np.abs(ref).max()
        if first is None:
            first = dc
        assert np.array_equal(dc, first)
    ba.close()


@pytest.mark.parametrize("n_kf", [2, 3, 4, 6, 8, 11, 12, 14, 17, 21])
def test_window_sizes_match_oracle(gpu, oracle, n_kf):
    """Every camera-solve variant: one row per lane for 1..10 free keyframes, two rows per lane
    (padded to 13, 16 or 20 free keyframes) above."""
    from rsvio import synthetic as S
    prob = S.ba_problem(n_kf=n_kf, n_lm=40 * n_kf, kf_per_lm=min(n_kf, 4), seed=100 + n_kf, init_seed=200 + n_kf)
    ba = _adjuster(gpu, prob)
    res = ba.run()
    pose, pw = ba.state()
    po, pwo, ro = oracle.ba_solve(prob)
    assert res.status == ro.status and res.iterations == ro.iterations
    assert np.abs(pose - po).max() < 1e-7
    assert np.abs(pw - pwo).max() < 1e-6
    ba.close()


@pytest.mark.parametrize("variant", ["pipe4", "gj1"])
@pytest.mark.parametrize("n_kf", [2, 3, 4, 5, 7, 8, 10, 11, 14, 21])
def test_camera_solve_variants_match_oracle(gpu, oracle, monkeypatch, variant, n_kf):
    """The K5 A/B variants (RSVIO_K5, read at handle creation): the pipelined VALU LDL^T (one row
    per lane up to 10 free keyframes, two rows per lane past them) and the one-wave Gauss-Jordan
    solve give the oracle's status and iteration count and its state within the stated
    tolerances, and the camera step of one system within 1e-9 of the default MFMA solve (8-column
    panels up to 10 free keyframes, 6x6 block pivots past them)."""
    from rsvio import synthetic as S
    if variant == "gj1" and n_kf > 10:
        pytest.skip("gj1 is instantiated up to 9 free keyframes")
    prob = S.ba_problem(n_kf=n_kf, n_lm=40 * n_kf, kf_per_lm=min(n_kf, 4), seed=300 + n_kf, init_seed=400 + n_kf)
    ref = _adjuster(gpu, prob)
    dc_ref = ref.camera_step(1e-4)
    monkeypatch.setenv("RSVIO_K5", variant)
    ba = _adjuster(gpu, prob)
    monkeypatch.delenv("RSVIO_K5")
    dc = ba.camera_step(1e-4)
    assert np.abs(dc - dc_ref).max() <= 1e-9 * max(np.abs(dc_ref).max(), 1e-12)
    res = ba.run()
    pose, pw = ba.state()
    po, pwo, ro = oracle.ba_solve(prob)
    assert res.status == ro.status and res.iterations == ro.iterations
    assert np.abs(pose - po).max() < 1e-7
    assert np.abs(pw - pwo).max() < 1e-6
    ba.close()
    ref.close()


def test_camera_solve_pipe4_config3(gpu, oracle, cfg3, monkeypatch):
    """Config 3 (9 free keyframes, n = 54) with the pipelined VALU camera solve (RSVIO_K5=pipe4,
    the A/B alternative to the default MFMA solve): oracle parity."""
    monkeypatch.setenv("RSVIO_K5", "pipe4")
    ba = _adjuster(gpu, cfg3)
    monkeypatch.delenv("RSVIO_K5")
    res = ba.run()
    pose, pw = ba.state()
    po, pwo, ro = oracle.ba_solve(cfg3)
    assert res.status == ro.status and res.iterations == ro.iterations
    assert np.abs(pose - po).max() < 1e-7 and np.abs(pw - pwo).max() < 1e-6
    ba.close()


def test_sharded_code_path_single_rank(gpu, cfg3):
    """The sharded path (RCCL all-reduce of sys, per-rank trial scalars + 32-B all-reduce,
    pre-reduced LM decision) on a 1-rank communicator equals the unsharded path bit for bit."""
    from rsvio.ba import BundleAdjuster
    a = _adjuster(gpu, cfg3)
    ra = a.run()
    pa, wa = a.state()
    b = BundleAdjuster(max_keyframes=21, max_landmarks=cfg3.n_lm, max_observations=cfg3.n_obs)
    b.attach_comm(1, 0, BundleAdjuster.rccl_unique_id())
    b.set_problem_from(cfg3)
    rb = b.run()
    pb, wb = b.state()
    assert (ra.status, ra.iterations) == (rb.status, rb.iterations)
    assert ra.final_cost == rb.final_cost
    assert np.array_equal(pa, pb) and np.array_equal(wa, wb)
    a.close()
    b.close()


def test_async_solve_equals_run(gpu, cfg3):
    """rsvio_ba_run_async + rsvio_ba_wait is the same solve as rsvio_ba_run."""
    a = _adjuster(gpu, cfg3)
    ra = a.run()
    pa, wa = a.state()
    a.run_async()
    rb = a.wait()
    pb, wb = a.state()
    assert (ra.status, ra.iterations, ra.final_cost) == (rb.status, rb.iterations, rb.final_cost)
    assert np.array_equal(pa, pb) and np.array_equal(wa, wb)
    with pytest.raises(Exception):
        a.wait()  # nothing in flight
    a.close()


def test_ticket_wait_equals_stream_sync(gpu, cfg3, monkeypatch):
    """rsvio_ba_wait on the decision ticket (default) returns the same solve as the stream-sync
    wait (RSVIO_BA_WAIT=sync, read at handle creation), back-to-back solves included, and the
    state read right after the ticket (get_state settles the stream) is bit-identical."""
    monkeypatch.setenv("RSVIO_BA_WAIT", "sync")
    s = _adjuster(gpu, cfg3)
    monkeypatch.delenv("RSVIO_BA_WAIT")
    t = _adjuster(gpu, cfg3)
    for _ in range(3):
        s.run_async()
        t.run_async()
        rs, rt = s.wait(), t.wait()
        assert (rs.status, rs.iterations, rs.initial_cost, rs.final_cost) == \
            (rt.status, rt.iterations, rt.initial_cost, rt.final_cost)
        assert rt.status > 0 and 0.0 < rt.solve_ms < 100.0
        ps, ws = s.state()
        pt, wt = t.state()
        assert np.array_equal(ps, pt) and np.array_equal(ws, wt)
    s.close()
    t.close()


def test_recapture_after_ticket_wait(gpu, cfg3):
    """A ticket wait returns before the last decision kernel has exited; the next solve with a
    different LM configuration re-captures the graph (the old exec is destroyed only after the
    stream settles).  Each solve equals the same solve on a fresh handle, bit for bit."""
    from rsvio.ba import fallback_cfg, lm_cfg
    cfgs = [lm_cfg(), lm_cfg(max_iterations=7), fallback_cfg(), lm_cfg(lambda_init=1e-3), lm_cfg()]
    a = _adjuster(gpu, cfg3)
    for c in cfgs:
        a.run_async(c)
        ra = a.wait()
        pa, wa = a.state()
        f = _adjuster(gpu, cfg3)
        rf = f.run(c)
        pf, wf = f.state()
        f.close()
        assert (ra.status, ra.iterations, ra.final_cost) == (rf.status, rf.iterations, rf.final_cost)
        assert np.array_equal(pa, pf) and np.array_equal(wa, wf)
    # back to back: the async solve's ticket, then a synchronous run with another config at once
    a.run_async(lm_cfg())
    a.wait()
    r = a.run(lm_cfg(max_iterations=3))
    assert r.iterations <= 3
    a.close()


def test_descriptor_graph_equals_by_value(gpu, cfg3, monkeypatch, capfd):
    """The first solve of a new window runs the descriptor-mode graph (the window's geometry and
    buffers read from its device descriptor, K4 / K6 over a rounded-up wave grid whose spare
    workgroups return at once); a window solved again replays the by-value graph.  Over a sequence
    of windows -- same shape (the exec replayed as it stands, no capture), fewer landmarks within
    the rounded-up grid (replayed, spare workgroups), fewer keyframes (re-captured), a changed LM
    configuration (the descriptor refreshed) -- every solve equals, bit for bit, the same solve on
    a handle with the descriptor mode off (RSVIO_BA_DESC=0: by-value kernels captured per window).
    Replays with a first chunk longer than the solve needs run iterations past convergence that
    return at once."""
    from rsvio import synthetic as S
    from rsvio.ba import BundleAdjuster, fallback_cfg, lm_cfg
    windows = [cfg3, S.ba_problem(seed=17, init_seed=23), S.ba_problem(n_lm=1900, seed=5, init_seed=6),
               S.ba_problem(n_kf=6, n_lm=300, seed=7), cfg3]
    cfgs = [lm_cfg(), lm_cfg(), lm_cfg(), lm_cfg(), fallback_cfg()]

    def mk():
        return BundleAdjuster(max_keyframes=21, max_landmarks=2000, max_observations=24000)

    monkeypatch.setenv("RSVIO_BA_DESC", "0")
    v = mk()
    monkeypatch.delenv("RSVIO_BA_DESC")
    monkeypatch.setenv("RSVIO_BA_PROFILE", "1")
    d = mk()
    monkeypatch.delenv("RSVIO_BA_PROFILE")
    for h in (v, d):  # warm-up: the first chunk of a solve is the previous solve's iteration count,
        h.set_problem_from(cfg3)  # and the state read-back turns the final decision's export on
        h.run()
        h.state()
        last = h.run().iterations

    def n_wave(p):  # set_problem's greedy packing: whole landmarks, <= 64 slots (keyframes) a wave
        keys = np.unique(p.obs_lm.astype(np.int64) * 64 + p.obs_kf)
        slots = np.bincount(keys // 64, minlength=p.n_lm)
        n, fill = 0, 64
        for ns in slots[slots > 0]:
            if fill + ns > 64:
                n, fill = n + 1, 0
            fill += ns
        return n

    captures, expected = [], []
    key, cap, kx = None, 0, 0
    for w, c in zip(windows, cfgs):
        for h in (v, d):
            h.set_problem_from(w)
        capfd.readouterr()
        for rep in range(2):  # the descriptor graph, then the window re-solved by the by-value one
            rv, rd = v.run(c), d.run(c)
            assert (rv.status, rv.iterations, rv.initial_cost, rv.final_cost) == \
                (rd.status, rd.iterations, rd.initial_cost, rd.final_cost)
            assert rd.status > 0
            pv, wv = v.state()
            pd, wd = d.state()
            assert np.array_equal(pv, pd) and np.array_equal(wv, wd)
            if rep == 0:
                captures.append(capfd.readouterr().err.count("graph us (desc)"))
                # replayed iff the shape key agrees, the exec's first chunk is the wanted one or up
                # to 2 longer, and the wave count fits the captured grid's upper half
                nw, k = n_wave(w), min(last, c.max_iterations)
                kk = (int((w.kf_fixed == 0).sum()), c.max_iterations, c.linear_solver)
                hit = kk == key and k <= kx <= k + 2 and nw <= cap and 2 * nw > cap
                expected.append(0 if hit else 1)
                if not hit:
                    key, cap, kx = kk, (nw + nw // 4 + 7) // 8 * 8, k
            last = rd.iterations
    assert captures == expected, (captures, expected)
    assert expected[1] == 0 or expected[2] == 0  # a replay happened (same shape / fewer landmarks)
    v.close()
    d.close()


def test_observation_order_is_irrelevant(gpu, cfg3):
    """set_problem builds the slot layout from per-landmark (keyframe, camera) masks, not from the
    input order: a shuffled observation list gives the same solve, bit for bit."""
    import dataclasses
    rng = np.random.default_rng(3)
    perm = rng.permutation(cfg3.n_obs)
    shuf = dataclasses.replace(cfg3, obs_lm=cfg3.obs_lm[perm], obs_kf=cfg3.obs_kf[perm],
                               obs_cam=cfg3.obs_cam[perm], obs_uv=cfg3.obs_uv[perm])
    a, b = _adjuster(gpu, cfg3), _adjuster(gpu, shuf)
    ra, rb = a.run(), b.run()
    assert (ra.status, ra.iterations, ra.initial_cost, ra.final_cost) == \
        (rb.status, rb.iterations, rb.initial_cost, rb.final_cost)
    for x, y in zip(a.state(), b.state()):
        assert np.array_equal(x, y)
    a.close()
    b.close()


def test_duplicate_observation_refused(gpu, cfg3):
    """Two observations of one landmark by the same camera of one keyframe (feature ids are unique
    per camera and frame in the reference) are refused with RSVIO_ERR_INVALID_ARG."""
    import dataclasses
    i = np.arange(cfg3.n_obs)
    dup = np.concatenate([i, i[:1]])
    bad = dataclasses.replace(cfg3, obs_lm=cfg3.obs_lm[dup], obs_kf=cfg3.obs_kf[dup], obs_cam=cfg3.obs_cam[dup],
                              obs_uv=cfg3.obs_uv[dup])
    from rsvio.ba import BundleAdjuster
    ba = BundleAdjuster(max_keyframes=21, max_landmarks=cfg3.n_lm, max_observations=cfg3.n_obs + 1)
    with pytest.raises(gpu.RsvioError) as e:
        ba.set_problem_from(bad)
    assert e.value.code == -1 and "more than one observation" in str(e.value)
    ba.set_problem_from(cfg3)  # the handle stays usable
    assert ba.run().status > 0
    ba.close()


def test_state_export_equals_device_copy(gpu, cfg3):
    """After the first rsvio_ba_get_state, each solve's final decision kernel publishes the
    optimised state to pinned host memory with its ticket; get_state then copies it from there.
    It equals the device-buffer copy of the same solve on a fresh handle, across a window change,
    and a skipped solve or build_system fall back to the device buffers (never a stale export)."""
    import dataclasses

    from rsvio import synthetic as S
    alt = S.ba_problem(seed=17, init_seed=23)
    a = _adjuster(gpu, cfg3)
    a.run()
    a.state()                                   # device copy; turns the export on
    for prob in (cfg3, alt, cfg3):
        a.set_problem_from(prob)
        ra = a.run()
        pa, wa = a.state()                      # exported
        f = _adjuster(gpu, prob)
        rf = f.run()
        pf, wf = f.state()                      # device copy
        f.close()
        assert (ra.status, ra.iterations, ra.final_cost) == (rf.status, rf.iterations, rf.final_cost)
        assert np.array_equal(pa, pf) and np.array_equal(wa, wf)
    few = dataclasses.replace(cfg3, obs_lm=cfg3.obs_lm[:5], obs_kf=cfg3.obs_kf[:5], obs_cam=cfg3.obs_cam[:5],
                              obs_uv=cfg3.obs_uv[:5])
    a.set_problem_from(few)
    assert a.run().status == -2                 # skipped: the state is the initial one
    p0, w0 = a.state()
    assert np.array_equal(p0, few.pose7) and np.array_equal(w0, few.p_W)
    a.set_problem_from(cfg3)
    a.run()
    a.build_system(1e-4)                        # resets the device state to the initial one
    p1, w1 = a.state()
    assert np.array_equal(p1, cfg3.pose7) and np.array_equal(w1, cfg3.p_W)
    a.close()


def test_skip_guard_counts_every_keyframe(gpu, oracle):
    """sliding_window.rs:304,315: num_variables counts every keyframe variable, the fixed KF_0
    included, so n_obs == n_free + n_lm is underconstrained (skipped) and n_obs == n_kf + n_lm
    is not -- on the device and in the oracle."""
    import dataclasses

    from rsvio import synthetic as S
    prob = S.ba_problem(n_kf=3, n_lm=8, kf_per_lm=3, seed=9, init_seed=10)
    for n_obs, skipped in ((prob.n_kf - 1 + prob.n_lm, True), (prob.n_kf + prob.n_lm, False)):
        cut = dataclasses.replace(prob, obs_lm=prob.obs_lm[:n_obs], obs_kf=prob.obs_kf[:n_obs],
                                  obs_cam=prob.obs_cam[:n_obs], obs_uv=prob.obs_uv[:n_obs])
        assert len(cut.obs_lm) == n_obs and int(cut.kf_fixed.sum()) == 1
        ba = _adjuster(gpu, cut)
        r = ba.run()
        _, _, ro = oracle.ba_solve(cut)
        assert (r.status == -2) == skipped and (ro.status == -2) == skipped, (n_obs, r.status, ro.status)
        ba.close()


def test_async_wrong_call_order_refused(gpu, cfg3):
    """Between rsvio_ba_run_async and rsvio_ba_wait, every entry point that reads or replaces
    what the solve uses is refused with RSVIO_ERR_INVALID_ARG (the in-flight solve is intact)."""
    a = _adjuster(gpu, cfg3)
    ra = a.run()
    pa, wa = a.state()
    a.run_async()
    for call in (lambda: a.state(), lambda: a.set_problem_from(cfg3), lambda: a.run_async(),
                 lambda: a.detach_p2p(), lambda: a.attach_comm(1, 0, a.rccl_unique_id()),
                 lambda: a.attach_p2p(1, 0, [bytes(64)])):
        with pytest.raises(gpu.RsvioError) as e:
            call()
        assert e.value.code == -1
    rb = a.wait()
    pb, wb = a.state()
    assert (ra.status, ra.iterations, ra.final_cost) == (rb.status, rb.iterations, rb.final_cost)
    assert np.array_equal(pa, pb) and np.array_equal(wa, wb)
    a.close()


def _p2p_worker(rank, world, port, out_dir, n_lm=2000, env=None):
    import os

    import torch.distributed as dist
    # ranks share this one GPU: the 4-launch iteration unless a test asks for another (the
    # 3-launch one's K4c waits in hundreds of workgroups for every rank's K6, which on a shared
    # device can starve a peer's K6 -- one rank per GPU never shares)
    os.environ["RSVIO_P2P_FOLD"] = "1"
    os.environ.update(env or {})
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rsvio import synthetic as S
        from rsvio.ba import BundleAdjuster
        full = S.ba_problem(n_lm=n_lm)
        shard = full.shard(rank, world)
        ba = BundleAdjuster(max_keyframes=21, max_landmarks=shard.n_lm, max_observations=shard.n_obs)
        mine = ba.p2p_export(world)
        handles = [None] * world
        dist.all_gather_object(handles, mine)
        ba.attach_p2p(world, rank, handles)
        ba.set_problem_from(shard)
        r = ba.run()
        pose, pw = ba.state()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), pose=pose, pw=pw,
                 res=np.array([r.status, r.iterations, r.final_cost, r.initial_cost]))
        ba.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharded_p2p_two_ranks_match_oracle(gpu, oracle, cfg3, tmp_path):
    """The landmark-sharded BA with the P2P one-shot all-reduce, 2 ranks (2 processes on one
    GPU: the exchange buffers are IPC-shared): both ranks end with the same poses, and the
    gathered solution matches the oracle's single-problem solve within the config-3 tolerances."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_p2p_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    assert np.array_equal(r0["pose"], r1["pose"]) and np.array_equal(r0["res"], r1["res"])
    po, pwo, ro = oracle.ba_solve(cfg3)
    status, iters = int(r0["res"][0]), int(r0["res"][1])
    assert status == ro.status and iters == ro.iterations
    assert abs(r0["res"][2] - ro.final_cost) <= 1e-8 * ro.initial_cost
    assert np.abs(r0["pose"] - po).max() < 1e-7
    pw = np.concatenate([r0["pw"], r1["pw"]])
    assert np.abs(pw - pwo).max() < 1e-6


def test_sharded_p2p_weak_scaling_size_matches_oracle(gpu, oracle, tmp_path):
    """The weak-scaling configuration of the bench at N = 2: 2,000 landmarks per rank (4,000 in
    all, 48,000 observations), the fused P2P path (K4c, K5 with the reduced system's exchange in
    its prologue, K6, X2 with the trial scalars' exchange: 4 launches per LM iteration -- the
    3-launch one is checked bit for bit against it below), against the oracle's single
    4,000-landmark solve within the config-3 tolerances."""
    import socket

    import torch.multiprocessing as mp
    from rsvio import synthetic as S
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_p2p_worker, args=(2, port, str(tmp_path), 4000), nprocs=2, join=True, start_method="spawn")
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    assert np.array_equal(r0["pose"], r1["pose"]) and np.array_equal(r0["res"], r1["res"])
    full = S.ba_problem(n_lm=4000)
    po, pwo, ro = oracle.ba_solve(full)
    assert int(r0["res"][0]) == ro.status and int(r0["res"][1]) == ro.iterations
    assert abs(r0["res"][2] - ro.final_cost) <= 1e-8 * ro.initial_cost
    assert np.abs(r0["pose"] - po).max() < 1e-7
    assert np.abs(np.concatenate([r0["pw"], r1["pw"]]) - pwo).max() < 1e-6


def _small_fallback_problem(seed=3):
    from rsvio import synthetic as S
    return S.ba_problem(n_kf=4, n_lm=40, kf_per_lm=3, seed=seed, init_seed=seed + 1)


def test_cholesky_fallback_matches_oracle(gpu, oracle, cfg3):
    """B3: the device's SparseCholesky fallback (landmarks eliminated first, 3x3 LL^T blocks) vs
    the oracle's dense LL^T of the full damped system: same LM path, tolerance parity; and on
    config 3 it takes the Schur solve's path (the two solvers differ only in rounding)."""
    from rsvio.ba import SOLVER_CHOLESKY, lm_cfg
    for prob in (_small_fallback_problem(), cfg3):
        ba = _adjuster(gpu, prob)
        r = ba.run(lm_cfg(linear_solver=SOLVER_CHOLESKY))
        pose, pw = ba.state()
        rs = ba.run(lm_cfg())
        ps, ws = ba.state()
        assert r.status > 0 and (r.status, r.iterations) == (rs.status, rs.iterations)
        assert np.abs(pose - ps).max() < 1e-9 and np.abs(pw - ws).max() < 1e-8
        if prob.n_lm <= 100:  # the oracle's dense full-system Cholesky is O(N^3)
            po, pwo, ro = oracle.ba_solve(prob, oracle.lm_cfg(linear_solver=1))
            assert (r.status, r.iterations) == (ro.status, ro.iterations)
            assert np.abs(pose - po).max() < 1e-7 and np.abs(pw - pwo).max() < 1e-6
        ba.close()


def test_singular_landmark_block_linear_solve_failed(gpu, oracle):
    """B3: a singular landmark block (lambda_init 0, a landmark behind every camera) fails the
    Schur solve with LinearSolveFailed at iteration 1 and the fallback the same way, as the
    oracle does; the state is left at the initial values (the caller reverts)."""
    import dataclasses

    from rsvio.ba import LINEAR_SOLVE_FAILED, SOLVER_CHOLESKY, lm_cfg
    base = _small_fallback_problem()
    pw = base.p_W.copy()
    pw[5] = 2.0 * base.p_W[0] - pw[5] * np.array([1.0, 1.0, -3.0])
    pw[5, 2] = -abs(pw[5, 2]) - 5.0
    prob = dataclasses.replace(base, p_W=pw)
    ba = _adjuster(gpu, prob)
    for ls in (0, SOLVER_CHOLESKY):
        r = ba.run(lm_cfg(lambda_init=0.0, linear_solver=ls))
        _, _, ro = oracle.ba_solve(prob, oracle.lm_cfg(lambda_init=0.0, linear_solver=ls))
        assert (r.status, r.iterations) == (LINEAR_SOLVE_FAILED, 1) == (ro.status, ro.iterations)
    r = ba.run(lm_cfg())  # default damping: solvable
    _, _, ro = oracle.ba_solve(prob, oracle.lm_cfg())
    assert r.status > 0 and (r.status, r.iterations) == (ro.status, ro.iterations)
    ba.close()


def test_batched_windows_match_single_and_oracle(gpu, oracle):
    """Batched mode (rsvio_ba_batch_*): ragged windows -- 2..11 keyframes, different landmark and
    observation counts, one window the guards skip -- solved by one launch chain; every window
    equals its own single-handle solve (status, iterations, state within 1e-10) and the oracle's
    solve of it within the stated tolerances."""
    from rsvio import synthetic as S
    from rsvio.ba import BundleAdjuster, BundleBatch
    shapes = [(3, 60, 2), (5, 150, 4), (8, 300, 5), (10, 2000, 6), (11, 400, 6), (4, 90, 3), (2, 1, 1)]
    probs = [S.ba_problem(n_kf=k, n_lm=m, kf_per_lm=p, seed=500 + i, init_seed=600 + i)
             for i, (k, m, p) in enumerate(shapes)]
    wins = [_adjuster(gpu, pr) for pr in probs]
    batch = BundleBatch(wins)
    for rep in range(2):                     # twice: the second run re-uses the chunk size
        for w, pr in zip(wins, probs):
            w.set_problem_from(pr)
        res = batch.run()
        for i, (w, pr, r) in enumerate(zip(wins, probs, res)):
            if i == len(probs) - 1:
                assert r.status == -2        # too few residuals: skipped
                continue
            pose, pw = w.state()
            one = _adjuster(gpu, pr)
            r1 = one.run()
            p1, w1 = one.state()
            one.close()
            assert (r.status, r.iterations) == (r1.status, r1.iterations), i
            assert np.abs(pose - p1).max() <= 1e-10 and np.abs(pw - w1).max() <= 1e-10, i
            po, pwo, ro = oracle.ba_solve(pr)
            assert r.status == ro.status and r.iterations == ro.iterations, i
            assert np.abs(pose - po).max() < 1e-7 and np.abs(pw - pwo).max() < 1e-6, i
    batch.close()
    for w in wins:
        w.close()


def test_batched_windows_past_ten_free_keyframes(gpu, oracle):
    """Batched mode with windows of 13, 16 and 20 free keyframes (the batch's K5 is the 6x6-block
    MFMA solver's padded template, bab_camera_solve_blk<20>) next to a 3-free-keyframe window padded
    to the same template: every window equals its own single-handle solve (status, iterations,
    state within 1e-9) and the oracle's solve within the stated tolerances."""
    from rsvio import synthetic as S
    from rsvio.ba import BundleBatch
    shapes = [(4, 90, 3), (14, 300, 5), (17, 200, 4), (21, 400, 6)]
    probs = [S.ba_problem(n_kf=k, n_lm=m, kf_per_lm=p, seed=900 + i, init_seed=950 + i)
             for i, (k, m, p) in enumerate(shapes)]
    wins = [_adjuster(gpu, pr) for pr in probs]
    batch = BundleBatch(wins)
    res = batch.run()
    for i, (w, pr, r) in enumerate(zip(wins, probs, res)):
        pose, pw = w.state()
        one = _adjuster(gpu, pr)
        r1 = one.run()
        p1, w1 = one.state()
        one.close()
        assert (r.status, r.iterations) == (r1.status, r1.iterations), i
        assert np.abs(pose - p1).max() <= 1e-9 and np.abs(pw - w1).max() <= 1e-9, i
        po, pwo, ro = oracle.ba_solve(pr)
        assert r.status == ro.status and r.iterations == ro.iterations, i
        assert np.abs(pose - po).max() < 1e-7 and np.abs(pw - pwo).max() < 1e-6, i
    batch.close()
    for w in wins:
        w.close()


def test_batch_runs_right_after_a_large_upload(gpu, oracle):
    """set_problem is asynchronous (H2D of the arena, ba_build_layout and a memset on
    the window's stream), so the batch stream must be ordered after it.  The largest window
    (config 5's shape, 20 keyframes would exceed the batched K5; 10 x 5,000 here) is uploaded
    LAST and the batch started at once, for several rounds of fresh problems: every window must
    equal the oracle's solve of ITS problem (a batch that read a half-written arena would not)."""
    from rsvio import synthetic as S
    from rsvio.ba import BundleAdjuster, BundleBatch
    shapes = [(4, 80, 3), (6, 200, 4), (10, 5000, 6)]
    wins = [BundleAdjuster(max_keyframes=21, max_landmarks=5000, max_observations=80000) for _ in shapes]
    batch = BundleBatch(wins)
    for rnd in range(3):
        probs = [S.ba_problem(n_kf=k, n_lm=m, kf_per_lm=p, seed=700 + 10 * rnd + i, init_seed=800 + 10 * rnd + i)
                 for i, (k, m, p) in enumerate(shapes)]
        for w, pr in zip(wins, probs):   # the large window goes up last
            w.set_problem_from(pr)
        res = batch.run()
        for i, (w, pr, r) in enumerate(zip(wins, probs, res)):
            pose, pw = w.state()
            po, pwo, ro = oracle.ba_solve(pr)
            assert (r.status, r.iterations) == (ro.status, ro.iterations), (rnd, i)
            assert np.abs(pose - po).max() < 1e-7 and np.abs(pw - pwo).max() < 1e-6, (rnd, i)
    batch.close()
    for w in wins:
        w.close()


def test_batch_refuses_a_handle_twice(gpu, cfg3):
    """two grid rows on one handle's state buffers would race -- refused."""
    from rsvio import RsvioError
    from rsvio.ba import BundleBatch
    a = _adjuster(gpu, cfg3)
    with pytest.raises(RsvioError) as e:
        BundleBatch([a, a])
    assert e.value.code == -1
    a.close()


def _run_p2p(world, n_lm, tmp_path, env=None):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_p2p_worker, args=(world, port, str(tmp_path), n_lm, env), nprocs=world, join=True,
                       start_method="spawn")
    return [np.load(tmp_path / f"r{r}.npz") for r in range(world)]


def test_sharded_p2p_four_ranks_match_oracle(gpu, oracle, tmp_path):
    """Four ranks (four processes on one GPU, IPC-mapped exchange buffers): the 4-rank slot layout,
    generation parity and rank-ordered sums N = 8 uses.  2,000 landmarks per rank = the oracle's
    single 8,000-landmark, 96,000-observation solve; every rank ends with bitwise the same poses and
    LM outcome, and the gathered solution matches the oracle within the config-3 tolerances."""
    from rsvio import synthetic as S
    rs = _run_p2p(4, 8000, tmp_path)
    for r in rs[1:]:
        assert np.array_equal(rs[0]["pose"], r["pose"]) and np.array_equal(rs[0]["res"], r["res"])
    full = S.ba_problem(n_lm=8000)
    po, pwo, ro = oracle.ba_solve(full)
    assert int(rs[0]["res"][0]) == ro.status and int(rs[0]["res"][1]) == ro.iterations
    assert abs(rs[0]["res"][2] - ro.final_cost) <= 1e-8 * ro.initial_cost
    assert np.abs(rs[0]["pose"] - po).max() < 1e-7
    assert np.abs(np.concatenate([r["pw"] for r in rs]) - pwo).max() < 1e-6


def test_sharded_p2p_six_ranks_match_oracle(gpu, oracle, tmp_path):
    """Six ranks (six processes on one GPU): past four ranks K5 reads every peer's slot in one
    group of 8 (the N=8 node's path), the trial exchange spans 6 x 4 words.  2,000 landmarks per
    rank = the oracle's 12,000-landmark solve; every rank ends with bitwise the same poses and LM
    outcome, within the config-3 tolerances of the oracle."""
    from rsvio import synthetic as S
    rs = _run_p2p(6, 12000, tmp_path)
    for r in rs[1:]:
        assert np.array_equal(rs[0]["pose"], r["pose"]) and np.array_equal(rs[0]["res"], r["res"])
    full = S.ba_problem(n_lm=12000)
    po, pwo, ro = oracle.ba_solve(full)
    assert int(rs[0]["res"][0]) == ro.status and int(rs[0]["res"][1]) == ro.iterations
    assert abs(rs[0]["res"][2] - ro.final_cost) <= 1e-8 * ro.initial_cost
    assert np.abs(rs[0]["pose"] - po).max() < 1e-7
    assert np.abs(np.concatenate([r["pw"] for r in rs]) - pwo).max() < 1e-6


def test_sharded_p2p_eight_ranks_match_oracle(gpu, oracle, tmp_path):
    """Eight ranks (eight processes on one GPU), the node's full group: K5 pulls the 7 peers'
    slots in one group of 8, the exchange uses all 8 parity slots per generation and the trial
    exchange spans 8 x 4 flag-in-word scalars.  2,000 landmarks per rank = the oracle's
    16,000-landmark, 192,000-observation solve; every rank ends with bitwise the same poses and LM
    outcome, within the config-3 tolerances of the oracle."""
    from rsvio import synthetic as S
    rs = _run_p2p(8, 16000, tmp_path)
    for r in rs[1:]:
        assert np.array_equal(rs[0]["pose"], r["pose"]) and np.array_equal(rs[0]["res"], r["res"])
    full = S.ba_problem(n_lm=16000)
    po, pwo, ro = oracle.ba_solve(full)
    assert int(rs[0]["res"][0]) == ro.status and int(rs[0]["res"][1]) == ro.iterations
    assert abs(rs[0]["res"][2] - ro.final_cost) <= 1e-8 * ro.initial_cost
    assert np.abs(rs[0]["pose"] - po).max() < 1e-7
    assert np.abs(np.concatenate([r["pw"] for r in rs]) - pwo).max() < 1e-6


@pytest.mark.parametrize("level,world,per_rank", [("3", 8, 2000), ("4", 2, 2000), ("4", 4, 2000), ("3", 2, 2000), ("3", 2, 7000),
                                                  ("2", 2, 2000), ("0", 2, 2000)])
def test_sharded_p2p_fold_equals_separate_exchange(gpu, tmp_path, level, world, per_rank):
    """The 4-launch iteration (RSVIO_P2P_FOLD=1: the reduced system's exchange in K5's prologue,
    the trial scalars through X2's flag-in-word exchange) against the 3-launch ones (4: K6's
    last-arriving wave sums the rank's wave partials and pushes the 4 scalars, the next decision
    polls them; 3: K6's reducer workgroup sums the rank's tagged wave partials and runs the trial
    exchange; 2: the trial scalars pushed by K6's waves and summed by the next decision) and the
    5-launch one (0: X1 as a kernel of its own): the same sums in the same order, so the solves are
    bit-identical on every rank.  7,000 landmarks per rank (> 512 waves) take fold 3's reducer
    through its full-width sweeps and their second chunk (2,000: the half-width one)."""
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    n = per_rank * world
    fold = _run_p2p(world, n, tmp_path / "a", env={"RSVIO_P2P_FOLD": "1"})
    # (on this shared GPU attach_p2p would lower fold 2 to 1; the test keeps it to compare its sums)
    sep = _run_p2p(world, n, tmp_path / "b", env={"RSVIO_P2P_FOLD": level, "RSVIO_P2P_FOLD_SHARED": "1"})
    for a, b in zip(fold, sep):
        for k in ("pose", "pw", "res"):
            assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_p2p_flag_in_word_equals_flag_protocol(gpu, tmp_path, world):
    """K5's system exchange in flag-in-word form (RSVIO_P2P_LL=1: every entry as two tagged 8-byte
    words, the reader polling the words, no fence and no flags) against the data + flags
    protocol: the same sums in the same rank order, so the solves are bit-identical on every
    rank (2 and 4 ranks sharing the GPU)."""
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    ll = _run_p2p(world, 2000 * world, tmp_path / "a", env={"RSVIO_P2P_LL": "1"})
    fl = _run_p2p(world, 2000 * world, tmp_path / "b")
    for a, b in zip(ll, fl):
        for k in ("pose", "pw", "res"):
            assert np.array_equal(a[k], b[k]), k


def _cap_worker(rank, world, port, out_dir, n_cu):
    import os

    import torch.distributed as dist
    os.environ["RSVIO_P2P_FOLD"] = "3"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rsvio import synthetic as S
        from rsvio._lib import CuStream
        from rsvio.ba import BundleAdjuster
        shard = S.ba_problem(n_lm=2000 * world).shard(rank, world)
        ba = BundleAdjuster(max_keyframes=21, max_landmarks=shard.n_lm, max_observations=shard.n_obs)
        # n_cu CUs: mask bits 0 .. n_cu - 1 = CU i // 8 of XCD i % 8 (every XCD keeps a CU)
        st = CuStream(0, list(range(n_cu))) if n_cu else None
        if st:
            ba.set_stream(st.ptr)
        mine = ba.p2p_export(world)
        handles = [None] * world
        dist.all_gather_object(handles, mine)
        ba.attach_p2p(world, rank, handles)
        ba.set_problem_from(shard)
        level = ba.p2p_level()
        r = ba.run()
        pose, pw = ba.state()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), pose=pose, pw=pw, level=level,
                 res=np.array([r.status, r.iterations, r.final_cost, r.initial_cost]))
        ba.close()
        if st:
            st.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_fold3_refused_past_resident_capacity(gpu, tmp_path):
    """ADVICE/verdict r05: fold 3's reducer waits inside K6's grid for the other workgroups, so the
    handle takes fold 3 only while n_wave + 1 <= K6's resident capacity on its stream's CU mask
    (shared among the ranks on the device).  Two ranks on an 8-CU stream (capacity far below a
    2,000-landmark shard's waves) report level 1 and solve bit-identically to two ranks on the
    whole GPU at level 3."""
    import socket

    import torch.multiprocessing as mp
    outs = {}
    for n_cu in (0, 8):
        d = tmp_path / f"cu{n_cu}"
        d.mkdir()
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.start_processes(_cap_worker, args=(2, port, str(d), n_cu), nprocs=2, join=True, start_method="spawn")
        outs[n_cu] = [np.load(d / f"r{r}.npz") for r in range(2)]
    assert [int(r["level"]) for r in outs[0]] == [3, 3]
    assert [int(r["level"]) for r in outs[8]] == [1, 1]
    for a, b in zip(outs[0], outs[8]):
        for k in ("pose", "pw", "res"):
            assert np.array_equal(a[k], b[k]), k


def _mismatch_worker(rank, world, port, out_dir):
    import os

    import torch.distributed as dist
    # the injected fault: rank 1 asks for the flag-in-word system exchange, rank 0 does not
    os.environ["RSVIO_P2P_LL"] = "1" if rank == 1 else "0"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rsvio import synthetic as S
        from rsvio.ba import BundleAdjuster
        shard = S.ba_problem(n_lm=400, seed=5, init_seed=6).shard(rank, world)
        ba = BundleAdjuster(max_keyframes=21, max_landmarks=shard.n_lm, max_observations=shard.n_obs)
        try:
            got = ba.attach_sharded(world, rank, "p2p", rccl_ok=False)
        except RuntimeError as e:
            got = "error: " + str(e)[:60]
        ba.set_problem_from(shard)      # the handle is intact and unsharded: its own shard solves
        r = ba.run()
        with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
            f.write(f"{got}\n{r.status}\n")
        ba.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharded_attach_disagreement_fails_on_every_rank(gpu, tmp_path):
    """Verdict r04 item 5: a fault injected on ONE rank (its exchange settings differ) makes the
    P2P self-test fail on EVERY rank; no RCCL on a shared GPU, so every rank raises RuntimeError
    (none hangs: the test's own timeout) and keeps a working unsharded handle."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_mismatch_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    outs = [(tmp_path / f"r{r}.txt").read_text().split("\n") for r in range(2)]
    for got, status, _ in outs:
        assert got.startswith("error: P2P exchange unavailable"), got
        assert int(status) > 0
