"""Regenerate the committed golden vectors (tests/golden/*.npz) from the CPU oracle.

The reference is pure Rust and cannot be built offline, so these vectors come
from the oracle restatement (oracle/) and pin the GPU path and the oracle against drift.
Run from the repo root:  python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

from oracle import oracle as O  # noqa: E402
from rsvio import synthetic as S  # noqa: E402

OUT = Path(__file__).resolve().parent


def small_frames(n, w=160, h=120, seed=99):
    tex = S.make_texture(w, h, n_blobs=400, seed=seed)
    rng = np.random.default_rng(seed + 1)
    frames = []
    for t in range(n):
        left = S._render(tex, w, h, t, False, 2.0 * rng.standard_normal((h, w)))
        right = S._render(tex, w, h, t, True, 2.0 * rng.standard_normal((h, w)))
        frames.append((left, right))
    return frames


def tracker_golden():
    w, h, L = 160, 120, 3
    frames = small_frames(4, w, h)
    left = np.stack([f[0] for f in frames])
    right = np.stack([f[1] for f in frames])
    rng = np.random.default_rng(5)
    noise_img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    pyr_l0 = O.build_pyramid(left[0], L)
    pyr_l1 = O.build_pyramid(left[1], L)
    pyr_r0 = O.build_pyramid(right[0], L)
    pyr_noise6 = O.build_pyramid(noise_img, 5)
    aff = S.track_features(left[0], 24, seed=3, spacing=12.0)
    t_aff, t_valid = O.track_points(pyr_l0, pyr_l1, w, h, L, aff)
    s_aff, s_valid = O.track_points(pyr_l0, pyr_r0, w, h, L, aff)
    det_xy, det_score = O.detect_key_points(left[0], 30, None)
    det2_xy, det2_score = O.detect_key_points(left[0], 30, det_xy[: len(det_xy) // 2].astype(np.float32))
    # full StereoPatchTracker over 4 frames (grid 30, L=3)
    tr = O.StereoTracker(w, h, L, 30, 20, 0.01)
    pipe = []
    for k in range(4):
        fl, fr = tr.process_frame(left[k], right[k])
        pipe.append((fl, fr))
    pipe_l = np.array([(k, f[0], f[1], f[2]) for k, (fl, _) in enumerate(pipe) for f in fl], np.float64)
    pipe_r = np.array([(k, f[0], f[1], f[2]) for k, (_, fr) in enumerate(pipe) for f in fr], np.float64)
    np.savez_compressed(OUT / "tracker_small.npz", w=w, h=h, levels=L, left=left, right=right,
                        noise_img=noise_img, pyr_l0=pyr_l0, pyr_l1=pyr_l1, pyr_r0=pyr_r0, pyr_noise5=pyr_noise6,
                        aff=aff, t_aff=t_aff, t_valid=t_valid, s_aff=s_aff, s_valid=s_valid, det_xy=det_xy, det_score=det_score, det2_xy=det2_xy,
                        det2_score=det2_score, pipe_l=pipe_l, pipe_r=pipe_r)


def ba_golden():
    prob = S.ba_problem(n_kf=4, n_lm=40, kf_per_lm=3, seed=3, init_seed=4)
    S_, b, cost = O.ba_build_system(prob, 1e-4)
    pose, pw, res = O.ba_solve(prob)
    np.savez_compressed(OUT / "ba_small.npz", pose7=prob.pose7, kf_fixed=prob.kf_fixed, p_W=prob.p_W,
                        obs_lm=prob.obs_lm, obs_kf=prob.obs_kf, obs_cam=prob.obs_cam, obs_uv=prob.obs_uv,
                        T_C_B2=prob.T_C_B2, true_pose7=prob.true_pose7, true_p_W=prob.true_p_W, S=S_, b=b,
                        cost=cost, sol_pose7=pose, sol_p_W=pw, status=res.status, iterations=res.iterations,
                        initial_cost=res.initial_cost, final_cost=res.final_cost)


def ft_frames(n, w=160, h=120, seed=31):
    """Noise-free mosaic frames (piecewise constant: the fixture compresses to a few KB)."""
    rects = S.make_mosaic(w, h, n_rects=160, seed=seed, size=(6.0, 28.0))
    return np.stack([S.render_mosaic(rects, w, h, t, np.zeros((h, w))) for t in range(n)])


def sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ft_golden():
    """feature_tracker/ crate variant: 160 x 120 mosaic frames, 3 levels (glibc sinf/cosf, as the
    reference's f32::sin/cos).  Large float outputs are pinned by SHA-256 of their bytes."""
    w, h, L = 160, 120, 3
    frames = ft_frames(4, w, h)
    pyr0 = O.ft_build_pyramid(frames[0], L)
    pyr1 = O.ft_build_pyramid(frames[1], L)
    pyr0_noblur = O.ft_build_pyramid(frames[0], L, blur=False)
    fine0 = pyr0[:w * h].reshape(h, w)
    score0 = O.ft_shi_tomasi_score(fine0)
    new0 = O.ft_add_points(fine0)
    trk_xy = (new0[: len(new0) // 2].astype(np.float32) + np.float32(0.3))
    new0_tr = O.ft_add_points(fine0, trk_xy)
    xy = new0.astype(np.float32)
    iso_ssd, v_ssd = O.ft_track_points(pyr0, pyr1, w, h, xy, nlevels=L, cost=0)
    iso_lssd, v_lssd = O.ft_track_points(pyr0, pyr1, w, h, xy, nlevels=L, cost=1)
    ft = O.FeatureTracker(w, h, O.ft_config(nlevels=L))
    pipe = []
    for k in range(len(frames)):
        ids, fxy = ft.process_frame(frames[k])
        pipe += [(k, int(i), float(p[0]), float(p[1])) for i, p in zip(ids, fxy)]
    np.savez_compressed(OUT / "ft_small.npz", w=w, h=h, levels=L, frames=frames, sha_pyr0=sha(pyr0),
                        sha_pyr1=sha(pyr1), sha_pyr0_noblur=sha(pyr0_noblur), sha_score0=sha(score0), new0=new0,
                        trk_xy=trk_xy, new0_tr=new0_tr, xy=xy, iso_ssd=iso_ssd, v_ssd=v_ssd, iso_lssd=iso_lssd,
                        v_lssd=v_lssd, pipe=np.array(pipe, np.float64))


if __name__ == "__main__":
    which = sys.argv[1:] or ["tracker", "ba", "ft"]
    if "tracker" in which:
        tracker_golden()
    if "ba" in which:
        ba_golden()
    if "ft" in which:
        ft_golden()
    print("wrote", sorted(p.name for p in OUT.glob("*.npz")))
