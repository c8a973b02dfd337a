"""The Estimator's per-keyframe host logic in the library's C++ (csrc/window.hip:
rsvio_window_problem, rsvio_window_apply) against an independent numpy restatement of
sliding_window.rs:174-300 and :418-486 -- host code, no device needed.

Integer outputs (landmark ids and order, observation lists) equal exactly; the floating-point
outputs within 1e-12 relative: the C++ inverts 4x4 transforms by the cofactor form
(nalgebra's try_inverse), numpy by LAPACK's LU, and the two round differently."""
import numpy as np
import pytest


def _feature_arrays(feats):
    ids, uv = feats
    return (np.asarray(ids, np.int64).reshape(-1),
            np.asarray(uv, np.float64).reshape(-1, 2).astype(np.float32).astype(np.float64))


def _numpy_problem(window):
    """The round-3 numpy build (sliding_window.rs:174-300), kept as the independent check."""
    from rsvio.ba import quat_from_matrix
    kfs = list(window.keyframes)
    T_Cl_B, T_Cr_B = np.linalg.inv(np.stack([kfs[0].T_B_Cl, kfs[0].T_B_Cr]))
    ids, uv, kf, cam = [], [], [], []
    for i, f in enumerate(kfs):
        for c, feats in enumerate((f.left_features, f.right_features)):
            fi, fu = _feature_arrays(feats)
            ids.append(fi)
            uv.append(fu)
            kf.append(np.full(len(fi), i, np.int32))
            cam.append(np.full(len(fi), c, np.uint8))
    ids, uv = np.concatenate(ids), np.concatenate(uv)
    kf, cam = np.concatenate(kf), np.concatenate(cam)
    keep = np.isin(ids, ids[cam == 0]) & np.isin(ids, ids[cam == 1])
    ids, uv, kf, cam = ids[keep], uv[keep], kf[keep], cam[keep]
    uniq, first, inv = np.unique(ids, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")
    rank = np.empty(len(uniq), np.int64)
    rank[order] = np.arange(len(uniq))
    obs_lm = rank[inv].astype(np.int32)
    lm_ids = uniq[order]
    p_init = np.zeros((len(lm_ids), 3))
    in_map = np.zeros(len(lm_ids), bool)
    if len(window.map_ids):
        mid, mpw = window.map_ids, window.map_pw.astype(np.float64)
        pos = np.clip(np.searchsorted(mid, lm_ids), 0, len(mid) - 1)
        in_map = mid[pos] == lm_ids
        p_init[in_map] = mpw[pos[in_map]]
    fo = first[order]
    T_B_C = np.linalg.inv(np.stack([T_Cl_B, T_Cr_B]))
    T_W_B = np.stack([f.T_W_B for f in kfs])
    for j in np.nonzero(~in_map)[0]:
        o = fo[j]
        p_C = np.array([uv[o, 0], uv[o, 1], 2.0])
        p_B = T_B_C[cam[o], :3, :3] @ p_C + T_B_C[cam[o], :3, 3]
        p_init[j] = T_W_B[kf[o], :3, :3] @ p_B + T_W_B[kf[o], :3, 3]
    pose7 = np.zeros((len(kfs), 7))
    T_B_W = np.linalg.inv(T_W_B)
    pose7[:, :3] = T_B_W[:, :3, 3]
    pose7[:, 3:] = quat_from_matrix(T_B_W[:, :3, :3])
    fixed = np.zeros(len(kfs), np.uint8)
    fixed[0] = 1
    T_C_B2 = np.stack([T_Cl_B.reshape(16), T_Cr_B.reshape(16)])
    return pose7, fixed, p_init, obs_lm, kf, cam, uv, T_C_B2, lm_ids


def _window(seed, n_kf=10, n_feat=300, n_map=150):
    """A window of keyframes with overlapping feature ids (some only left / only right) and a
    map holding part of them."""
    from rsvio.ba import Frame, SlidingWindow, quat_from_matrix  # noqa: F401
    rng = np.random.default_rng(seed)

    def rigid():
        a = rng.normal(size=3) * 0.3
        R = np.linalg.qr(rng.normal(size=(3, 3)))[0]
        if np.linalg.det(R) < 0:
            R[:, 0] *= -1
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = a
        return T
    w = SlidingWindow.__new__(SlidingWindow)
    from collections import deque
    w.keyframes = deque()
    T_B_Cl, T_B_Cr = rigid(), rigid()
    base = 0
    for k in range(n_kf):
        ids_l = np.sort(rng.choice(np.arange(base, base + 2 * n_feat), n_feat, replace=False))
        ids_r = np.sort(rng.choice(np.arange(base, base + 2 * n_feat), n_feat // 2, replace=False))
        uv_l = rng.normal(size=(len(ids_l), 2)).astype(np.float32)
        uv_r = rng.normal(size=(len(ids_r), 2)).astype(np.float32)
        w.keyframes.append(Frame(frame_id=k, T_W_B=rigid(), T_B_Cl=T_B_Cl, T_B_Cr=T_B_Cr,
                                 left_features=(ids_l, uv_l), right_features=(ids_r, uv_r)))
        base += n_feat // 3
    all_ids = np.unique(np.concatenate([f.left_features[0] for f in w.keyframes]))
    mid = np.sort(rng.choice(all_ids, min(n_map, len(all_ids)), replace=False))
    w.map_ids = mid.astype(np.int64)
    w.map_pw = rng.normal(size=(len(mid), 3)).astype(np.float32)
    w.map_version = 0
    return w


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_window_problem_matches_numpy_restatement(seed):
    from rsvio.ba import SlidingWindow
    w = _window(seed)
    got = SlidingWindow.build_problem(w)
    ref = _numpy_problem(w)
    names = ("pose7", "kf_fixed", "p_init", "obs_lm", "obs_kf", "obs_cam", "obs_uv", "T_C_B2", "lm_ids")
    for name, a, b in zip(names, got, ref):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape, name
        if name in ("kf_fixed", "obs_lm", "obs_kf", "obs_cam", "lm_ids", "obs_uv"):
            assert np.array_equal(a, b), name
        else:
            assert np.allclose(a, b, rtol=1e-12, atol=1e-12), name
    assert len(got[8]) > 100 and len(got[3]) > 1000


def test_window_problem_capacity_and_empty_map():
    import ctypes as C

    from rsvio import _lib
    from rsvio.ba import SlidingWindow
    w = _window(4)
    w.map_ids, w.map_pw = np.zeros(0, np.int64), np.zeros((0, 3), np.float32)
    got, ref = SlidingWindow.build_problem(w), _numpy_problem(w)
    assert np.array_equal(got[8], ref[8]) and np.allclose(got[2], ref[2], rtol=1e-12, atol=1e-12)
    # too small an output capacity -> RSVIO_ERR_CAPACITY (-4)
    lib = _lib.load()
    T = np.stack([np.eye(4)] * 2)
    ids = np.arange(4, dtype=np.uint64)
    uv = np.zeros((4, 2), np.float32)
    ids = np.concatenate([ids, ids])
    uv = np.concatenate([uv, uv])
    P, U = ids.ctypes.data, uv.ctypes.data
    nf = np.array([4, 4], np.int32)
    out = [np.zeros(64) for _ in range(8)]
    nl, no = C.c_int32(0), C.c_int32(0)
    rc = lib.rsvio_window_problem(1, np.eye(4).ctypes.data, T.ctypes.data, P, U, nf.ctypes.data, None, None, 0,
                                  out[0].ctypes.data, out[1].ctypes.data, out[2].ctypes.data, 2, out[3].ctypes.data,
                                  out[4].ctypes.data, C.byref(nl), 8, out[5].ctypes.data, out[6].ctypes.data,
                                  out[7].ctypes.data, out[0].ctypes.data, C.byref(no))
    assert rc == -4


def test_window_apply_matches_numpy():
    from rsvio.ba import SlidingWindow, se3_matrix
    w = _window(5)
    rng = np.random.default_rng(9)
    pose = rng.normal(size=(len(w.keyframes), 7))
    ids = rng.permutation(np.arange(1000, 1300)).astype(np.int64)
    pw = rng.normal(size=(len(ids), 3))
    r = type("R", (), {"status": 1})()
    assert SlidingWindow._apply(w, ids, pose, pw, r)
    srt = np.argsort(ids)
    assert np.array_equal(w.map_ids, ids[srt]) and np.array_equal(w.map_pw, pw.astype(np.float32)[srt])
    T_ref = np.linalg.inv(np.stack([se3_matrix(p) for p in pose]))
    for f, T in zip(w.keyframes, T_ref):
        assert np.allclose(f.T_W_B, T, rtol=1e-12, atol=1e-12)
