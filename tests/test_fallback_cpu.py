"""B3: the Schur -> SparseCholesky fallback (src/estimator/sliding_window.rs:326-353), on CPU.

* The oracle's two linear solvers: SparseSchurComplement (Schur + dense camera Cholesky) and the
  SparseCholesky fallback (the full damped system, dense LL^T with the landmarks ordered first)
  take the same LM path on a regular window (poses 1e-12, landmarks 1e-10: rounding only).
* A singular landmark block (lambda_init 0 and a landmark behind every camera: J = 0, so
  V + 0 I = 0) makes the Schur solve fail with LinearSolveFailed (status -3) at the first
  iteration, and the fallback fails the same way.
* The SlidingWindow mirror retries with SparseCholesky from the same initial values and, when
  that fails too, reverts (Ok(false), nothing modified); a succeeding retry is applied.
"""
import dataclasses

import numpy as np

from rsvio import synthetic as S
from rsvio.ba import LINEAR_SOLVE_FAILED, SOLVER_CHOLESKY, SOLVER_SCHUR, Frame, SlidingWindow
from rsvio.synthetic import T_B_CL, T_B_CR


def _small(seed=3):
    return S.ba_problem(n_kf=4, n_lm=40, kf_per_lm=3, seed=seed, init_seed=seed + 1)


def _behind(prob, l=5):
    """Landmark l mirrored behind the cameras: every observation fails cheirality (J = 0)."""
    pw = prob.p_W.copy()
    pw[l] = 2.0 * prob.p_W[0] - pw[l] * np.array([1.0, 1.0, -3.0])
    pw[l, 2] = -abs(pw[l, 2]) - 5.0
    return dataclasses.replace(prob, p_W=pw)


def test_oracle_cholesky_fallback_equals_schur(oracle):
    prob = _small()
    p0, w0, r0 = oracle.ba_solve(prob, oracle.lm_cfg(linear_solver=0))
    p1, w1, r1 = oracle.ba_solve(prob, oracle.lm_cfg(linear_solver=1))
    assert r0.status > 0 and (r0.status, r0.iterations) == (r1.status, r1.iterations)
    assert np.abs(p0 - p1).max() < 1e-12 and np.abs(w0 - w1).max() < 1e-10
    assert abs(r0.final_cost - r1.final_cost) <= 1e-12 * r0.initial_cost


def test_oracle_singular_landmark_fails_both_solvers(oracle):
    prob = _behind(_small())
    for ls in (0, 1):
        _, _, r = oracle.ba_solve(prob, oracle.lm_cfg(lambda_init=0.0, linear_solver=ls))
        assert (r.status, r.iterations) == (LINEAR_SOLVE_FAILED, 1)
    # with the default damping the same window solves (V + 1e-4 I is positive definite)
    _, _, r = oracle.ba_solve(prob, oracle.lm_cfg())
    assert r.status > 0


class _ScriptedSolver:
    """Records the linear solver of every call and returns scripted statuses."""

    def __init__(self, statuses):
        self.statuses = list(statuses)
        self.calls = []

    def solve(self, pose7, kf_fixed, p_W, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2, cfg=None):
        self.calls.append(SOLVER_SCHUR if cfg is None else cfg.linear_solver)
        st = self.statuses.pop(0)
        res = type("R", (), {"status": st, "iterations": 1, "initial_cost": 1.0, "final_cost": 0.5})()
        return np.asarray(pose7).copy(), np.asarray(p_W).copy() + 0.25, res


def _window(solver, n_kf=4):
    rng = np.random.default_rng(0)
    sw = SlidingWindow(n_kf, solver=solver)
    for k in range(n_kf):
        T = np.eye(4)
        T[:3, 3] = [0.1 * k, 0.0, 0.0]
        feats = [[(i, tuple(rng.normal(0, 0.2, 2))) for i in range(30)] for _ in range(2)]
        sw.add_frame(Frame(frame_id=k, T_W_B=T, T_B_Cl=T_B_CL, T_B_Cr=T_B_CR, left_features=feats[0],
                           right_features=feats[1]))
    return sw


def test_sliding_window_retries_then_reverts():
    solver = _ScriptedSolver([LINEAR_SOLVE_FAILED, LINEAR_SOLVE_FAILED])
    sw = _window(solver)
    before = [f.T_W_B.copy() for f in sw.keyframes]
    assert sw.optimize() is False
    assert solver.calls == [SOLVER_SCHUR, SOLVER_CHOLESKY] and sw.fallbacks == 1
    assert sw.map_points == {} and all(np.array_equal(a, f.T_W_B) for a, f in zip(before, sw.keyframes))


def test_sliding_window_retry_success_is_applied():
    solver = _ScriptedSolver([LINEAR_SOLVE_FAILED, 1])
    sw = _window(solver)
    assert sw.optimize() is True
    assert solver.calls == [SOLVER_SCHUR, SOLVER_CHOLESKY] and len(sw.map_points) == 30


def test_sliding_window_other_failures_do_not_retry():
    for st in (-1, 4, 1):
        solver = _ScriptedSolver([st])
        sw = _window(solver)
        sw.optimize()
        assert solver.calls == [SOLVER_SCHUR] and sw.fallbacks == 0
