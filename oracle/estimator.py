"""Test infrastructure (tests and bench.py's cpu_baseline leg only): the Estimator's backend
seam filled with the CPU oracle, so the same host logic (rsvio.estimator.Estimator over rsvio.ba.SlidingWindow) runs once over the
device library and once over the restatement.  Nothing in rsvio imports it.

  track       -> oracle.StereoTracker (feature_tracker.rs:116-187) + oracle.unproject (frame.rs:107-134)
  track_motion-> oracle.track_motion (sliding_window.rs:490-587 + estimator.rs:195-234)
  solver      -> oracle.ba_solve (sliding_window.rs:159-381 + apex LM, restated)
"""
from types import SimpleNamespace

import numpy as np

from rsvio.camera import CONVENTIONS


def _orc_cfg(oracle, cfg):
    if cfg is None:
        return None
    return oracle.lm_cfg(cfg.max_iterations, cfg.cost_tolerance, cfg.parameter_tolerance, cfg.huber_delta,
                         cfg.lambda_init, cfg.linear_solver)


class OracleSolver:
    def __init__(self, oracle):
        self.o = oracle

    def solve(self, pose7, kf_fixed, p_W, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2, cfg=None):
        prob = SimpleNamespace(pose7=pose7, kf_fixed=kf_fixed, p_W=p_W, obs_lm=obs_lm, obs_kf=obs_kf,
                               obs_cam=obs_cam, obs_uv=obs_uv, T_C_B2=T_C_B2)
        return self.o.ba_solve(prob, _orc_cfg(self.o, cfg))

    def close(self):
        pass


class OracleBackend:
    def __init__(self, oracle, width, height, cameras, levels=6, grid_size=50, max_iterations=20, thresh=0.01,
                 translation_threshold=0.05, rotation_threshold=0.05, threads=1):
        """threads > 1: the all-cores CPU leg -- the tracker's pyramid levels and features in
        parallel (rayon's par_iter) and the threaded Schur BA (oracle.set_ba_threads, a process-wide
        setting the caller restores)."""
        self.o = oracle
        self.tracker = oracle.StereoTracker(width, height, levels, grid_size, max_iterations, thresh, threads=threads)
        self.cams = [oracle.camera(c.model, c.params, CONVENTIONS[c.convention], c.max_iterations) for c in cameras]
        self.thr = (translation_threshold, rotation_threshold)
        self.solver = OracleSolver(oracle)
        self.map = (np.zeros(0, np.uint64), np.zeros((0, 3), np.float32))

    def submit(self, left, right):
        self._submitted = (left, right)

    def collect(self):
        (left, right), self._submitted = self._submitted, None
        return self.track(left, right)

    def track(self, left, right):
        out = []
        for feats, cam in zip(self.tracker.process_frame(left, right), self.cams):
            ids = np.array([f[0] for f in feats], np.int64)
            px = np.array([[f[1], f[2]] for f in feats], np.float32).reshape(-1, 2)
            uv, _ = self.o.unproject(cam, px)
            out.append((ids, uv))
        self.last = tuple(out)     # track_motion reads them (the device backend keeps them on device)
        return self.last

    def set_map(self, ids, p_W):
        self.map = (np.asarray(ids, np.uint64), np.asarray(p_W, np.float32))

    def track_motion(self, T_W_B_last_kf, T_C_B2):
        (ids_l, uv_l), (ids_r, uv_r) = self.last
        r = self.o.track_motion(ids_l, uv_l, ids_r, uv_r, self.map[0], self.map[1], T_W_B_last_kf, T_C_B2,
                                thr_t=self.thr[0], thr_r=self.thr[1])
        return r.status, bool(r.is_keyframe), np.array(r.T_W_B[:]).reshape(4, 4), r.iterations, r.final_cost

    def close(self):
        pass



def outcome_difference(rd, ro):
    """How the device FrameResult rd differs from the oracle's ro in its integer outcomes: None
    when the keyframe flag, the PnP status + LM iterations and the BA status + LM iterations are
    all equal, else a description of the divergence.  No exception: since round 5 the LM's
    cost-tolerance test takes |change| <= tol * cost whatever the change's sign, before the
    accept test, so a change at rounding level -- where the device's tree
    sums and the oracle's sequential sums round differently -- no longer decides an outcome."""
    if rd.is_keyframe != ro.is_keyframe:
        return f"keyframe flag {rd.is_keyframe} vs {ro.is_keyframe}"
    if (rd.ba_status, rd.ba_iterations) != (ro.ba_status, ro.ba_iterations):
        return f"BA (status, iterations) {(rd.ba_status, rd.ba_iterations)} vs {(ro.ba_status, ro.ba_iterations)}"
    pd, po = (rd.pnp_status, rd.pnp_iterations), (ro.pnp_status, ro.pnp_iterations)
    if pd != po:
        return f"PnP (status, iterations) {pd} vs {po}, final cost {rd.pnp_cost} vs {ro.pnp_cost}"
    return None
