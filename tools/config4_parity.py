"""Config 4 parity over a long stream: the device Estimator and the oracle Estimator side by side,
frame by frame (ids, undistorted f32 bits, keyframe flags, PnP / BA status, pose), reporting the
first divergent frame of each kind and the largest pose difference.  Writes a JSON summary.
  python tools/config4_parity.py [n_frames] [out.json]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]


class Spy:
    def __init__(self, be):
        self.be, self.solver, self.feats = be, be.solver, None

    def track(self, l, r):
        self.feats = self.be.track(l, r)
        return self.feats

    def submit(self, l, r):
        self.be.submit(l, r)

    def collect(self):
        self.feats = self.be.collect()
        return self.feats

    def __getattr__(self, k):
        return getattr(self.be, k)


def compare(n_frames, pipelined=True, log_every=50):
    from oracle import oracle as O
    from oracle.estimator import OracleBackend, outcome_difference
    from rsvio import synthetic as S
    from rsvio.camera import Camera
    from rsvio.estimator import DeviceBackend, Estimator
    s = S.euroc_scene_stream(n_frames)
    h, w = s.frames[0][0].shape
    cams = [Camera.opencv5(*p) for p in s.intrinsics]
    dev = Spy(DeviceBackend(w, h, cams, 6, 50, 20, 0.01, 10, 0.05, 0.05, 0))
    orc = Spy(OracleBackend(O, w, h, cams))
    # the device in the bench's mode (Estimator.run: tracker one frame ahead, pipelined BA); its
    # FrameResults are complete once the next solve is waited for, so they are compared at the end
    ed = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=10, backend=dev, pipelined=pipelined)
    eo = Estimator(w, h, cams, s.T_B_Cl, s.T_B_Cr, window=10, backend=orc)
    dev_frames = ed.run(s.frames) if pipelined else (ed.process_frame(l, r) for l, r in s.frames)
    pairs = []
    first = {"ids": None, "uv_bits": None, "keyframe": None, "status_class": None, "status_exact": None,
             "pose_1e-6": None}
    max_pose = 0.0
    gerr = oerr = 0.0
    n_kf = 0
    t0 = time.time()
    for k, ((l, r), rd) in enumerate(zip(s.frames, dev_frames)):
        ro = eo.process_frame(l, r)
        for (ids_d, uv_d), (ids_o, uv_o) in zip(dev.feats, orc.feats):
            if first["ids"] is None and not np.array_equal(ids_d, ids_o):
                first["ids"] = k
            if first["uv_bits"] is None and not (np.shape(uv_d) == np.shape(uv_o) and np.array_equal(
                    np.asarray(uv_d, np.float32).view(np.uint32), np.asarray(uv_o, np.float32).view(np.uint32))):
                first["uv_bits"] = k
        pairs.append((rd, ro))
        if log_every and (k + 1) % log_every == 0:
            print(f"frame {k + 1}/{n_frames} ({time.time() - t0:.0f} s): first {first}", flush=True)
    ed.flush()
    for k, (rd, ro) in enumerate(pairs):
        if first["keyframe"] is None and rd.is_keyframe != ro.is_keyframe:
            first["keyframe"] = k
        for a, b in ((rd.pnp_status, ro.pnp_status), (rd.ba_status, ro.ba_status)):
            if first["status_class"] is None and not ((a is None) == (b is None) and (a is None or (a > 0) == (b > 0))):
                first["status_class"] = k
        if first["status_exact"] is None and outcome_difference(rd, ro) is not None:
            first["status_exact"] = k
        d = float(np.abs(rd.T_W_B - ro.T_W_B).max())
        max_pose = max(max_pose, d)
        if first["pose_1e-6"] is None and d > 1e-6:
            first["pose_1e-6"] = k
        gerr = max(gerr, float(np.linalg.norm(rd.T_W_B[:3, 3] - s.T_W_B[k][:3, 3])))
        oerr = max(oerr, float(np.linalg.norm(ro.T_W_B[:3, 3] - s.T_W_B[k][:3, 3])))
        n_kf += rd.is_keyframe
    traj = max(float(np.abs(a - b).max()) for a, b in zip(ed.trajectory(), eo.trajectory()))
    md, mo = ed.window.map_points, eo.window.map_points
    dev.be.close()
    return {"frames": n_frames, "mode": "Estimator.run (look-ahead, pipelined)" if pipelined else "sequential",
            "status_exact_means": "keyframe flag, BA status + LM iterations, PnP status + LM iterations "
                                  "(oracle/estimator.py outcome_difference)",
            "keyframes": n_kf, "first_divergent_frame": first,
            "max_pose_diff_vs_oracle": max_pose, "max_trajectory_diff_vs_oracle": traj,
            "map_ids_equal": sorted(md) == sorted(mo),
            "gpu_max_position_error_m": gerr, "oracle_max_position_error_m": oerr}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    res = compare(n)
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")
