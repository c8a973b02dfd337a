"""GPU parity of the patch tracker (HP-T) against the CPU oracle, through the C ABI.

Bars (DESIGN.md "Tracker parity"):
  * pyramid: bit-exact (u8 output of f32 arithmetic in the reference's order);
  * FAST grid detection: bit-exact (integer);
  * track_points: bit-exact against the oracle, whose SE(2) sin/cos are glibc's sinf/cosf (what
    Rust's f32::sin/cos call); the kernel's restatement of them is proven equal over all 2^32
    inputs (test_trig_gpu.py);
  * StereoPatchTracker: identical ids, counts and (bitwise) positions frame by frame.
"""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def _gold(name):
    return np.load(GOLD / name, allow_pickle=False)


@pytest.mark.parametrize("shape,levels", [((480, 752), 3), ((480, 752), 6), ((61, 97), 3), ((120, 160), 5),
                                          ((512, 512), 6), ((33, 40), 2)])
def test_pyramid_bitexact(gpu, oracle, shape, levels):
    rng = np.random.default_rng(shape[0] * 1000 + levels)
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    ref = oracle.build_pyramid(img, levels)
    out = gpu.build_image_pyramid(img, levels)
    assert out.shape == ref.shape
    assert np.array_equal(out, ref)


def test_pyramid_dimensions(gpu):
    # reference KAT (feature_tracker/src/image_operations.rs:84-94): 120x60 -> 60x30 -> 30x15
    img = np.zeros((60, 120), np.uint8)
    pyr = gpu.build_image_pyramid(img, 3)
    lv = gpu.pyramid_levels(pyr, 120, 60, 3)
    assert [x.shape for x in lv] == [(60, 120), (30, 60), (15, 30)]


def test_pyramid_golden(gpu):
    g = _gold("tracker_small.npz")
    assert np.array_equal(gpu.build_image_pyramid(g["left"][0], 3), g["pyr_l0"])
    assert np.array_equal(gpu.build_image_pyramid(g["noise_img"], 5), g["pyr_noise5"])


def test_pyramid_synthetic_frame(gpu, oracle, stereo_frames):
    left, _ = stereo_frames[0]
    for levels in (3, 6):
        assert np.array_equal(gpu.build_image_pyramid(left, levels), oracle.build_pyramid(left, levels))


def test_track_points_golden(gpu):
    g = _gold("tracker_small.npz")
    w, h, L = int(g["w"]), int(g["h"]), int(g["levels"])
    aff, valid = gpu.track_points(g["pyr_l0"], g["pyr_l1"], w, h, L, g["aff"])
    assert np.array_equal(valid, g["t_valid"].astype(bool))
    assert np.array_equal(aff[valid].view(np.uint32), g["t_aff"][valid].view(np.uint32))
    aff, valid = gpu.track_points(g["pyr_l0"], g["pyr_r0"], w, h, L, g["aff"])
    assert np.array_equal(valid, g["s_valid"].astype(bool))
    assert np.array_equal(aff[valid].view(np.uint32), g["s_aff"][valid].view(np.uint32))


@pytest.mark.parametrize("levels", [3, 6])
def test_track_points_bitexact(gpu, oracle, stereo_frames, levels):
    from rsvio import synthetic as S
    (l0, r0), (l1, r1) = stereo_frames[0], stereo_frames[1]
    w, h = 752, 480
    p0 = oracle.build_pyramid(l0, levels)
    p1 = oracle.build_pyramid(l1, levels)
    pr = oracle.build_pyramid(r0, levels)
    aff = S.track_features(l0, 300)
    for a_pyr, b_pyr in ((p0, p1), (p0, pr)):
        ref_aff, ref_valid = oracle.track_points(a_pyr, b_pyr, w, h, levels, aff)
        out_aff, out_valid = gpu.track_points(a_pyr, b_pyr, w, h, levels, aff)
        assert np.array_equal(out_valid, ref_valid)
        assert np.array_equal(out_aff.view(np.uint32), ref_aff.view(np.uint32))
        # L=6 loses tracks whose template leaves the 23x15 top level (reference behaviour)
        assert ref_valid.mean() > (0.8 if levels == 3 else 0.3)


def test_track_points_vs_libm_oracle(gpu, oracle, stereo_frames):
    """Large rotations: states pre-rotated and frames far apart, so the Gauss-Newton increments
    take sin/cos well outside the small-angle path (|theta| up to pi/4 and beyond); the valid
    flags and every output bit equal the libm oracle's."""
    from rsvio import synthetic as S
    (l0, _), (l1, _) = stereo_frames[0], stereo_frames[3]
    p0, p1 = oracle.build_pyramid(l0, 3), oracle.build_pyramid(l1, 3)
    aff = S.track_features(l0, 300)
    rng = np.random.default_rng(11)
    ang = rng.uniform(-0.6, 0.6, len(aff)).astype(np.float32)
    aff[:, 0], aff[:, 1], aff[:, 2], aff[:, 3] = np.cos(ang), -np.sin(ang), np.sin(ang), np.cos(ang)
    ref_aff, ref_valid = oracle.track_points(p0, p1, 752, 480, 3, aff)
    out_aff, out_valid = gpu.track_points(p0, p1, 752, 480, 3, aff)
    assert np.array_equal(out_valid, ref_valid)
    assert np.array_equal(out_aff.view(np.uint32), ref_aff.view(np.uint32))


def test_track_points_edge_cases(gpu, oracle):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (64, 80), dtype=np.uint8)
    black = np.zeros((64, 80), np.uint8)
    p = oracle.build_pyramid(img, 2)
    pb = oracle.build_pyramid(black, 2)
    aff = np.zeros((7, 6), np.float32)
    aff[:, 0] = aff[:, 3] = 1.0
    aff[:, 4:6] = [[1.0, 1.0], [40.0, 30.0], [79.5, 63.5], [-5.0, 10.0], [40.0, 30.0], [2.6, 2.6], [1e9, 5.0]]
    aff[4, 0:4] = [0.0, -1.0, 1.0, 0.0]  # rotated state (rotation is carried, not used)
    for a, b in ((p, p), (p, pb), (pb, p)):
        ra, rv = oracle.track_points(a, b, 80, 64, 2, aff)
        ga, gv = gpu.track_points(a, b, 80, 64, 2, aff)
        assert np.array_equal(gv, rv)
        assert np.array_equal(ga.view(np.uint32), ra.view(np.uint32))
    # empty batch
    ga, gv = gpu.track_points(p, p, 80, 64, 2, np.zeros((0, 6), np.float32))
    assert ga.shape == (0, 6) and gv.shape == (0,)


def test_detect_golden(gpu):
    g = _gold("tracker_small.npz")
    xy, sc = gpu.detect_key_points(g["left"][0], 30, None)
    assert np.array_equal(xy, g["det_xy"]) and np.array_equal(sc, g["det_score"])
    ex = g["det_xy"][: len(g["det_xy"]) // 2].astype(np.float32)
    xy, sc = gpu.detect_key_points(g["left"][0], 30, ex)
    assert np.array_equal(xy, g["det2_xy"]) and np.array_equal(sc, g["det2_score"])


@pytest.mark.parametrize("grid", [30, 50])
def test_detect_bitexact(gpu, oracle, stereo_frames, grid):
    left, _ = stereo_frames[0]
    rng = np.random.default_rng(grid)
    for existing in (None, rng.uniform(-10, 760, (200, 2)).astype(np.float32)):
        ref = oracle.detect_key_points(left, grid, existing)
        out = gpu.detect_key_points(left, grid, existing)
        assert np.array_equal(out[0], ref[0])
        assert np.array_equal(out[1], ref[1])
    noise = rng.integers(0, 256, (480, 752), dtype=np.uint8)
    assert all(np.array_equal(a, b) for a, b in zip(gpu.detect_key_points(noise, grid),
                                                     oracle.detect_key_points(noise, grid)))
    flat = np.full((480, 752), 77, np.uint8)
    assert len(gpu.detect_key_points(flat, grid)[0]) == 0


def _pipeline_compare(gpu, oracle, frames, w, h, levels, grid):
    ref = oracle.StereoTracker(w, h, levels, grid, 20, 0.01)
    trk = gpu.StereoPatchTracker(w, h, levels=levels, grid_size=grid)
    for k, (l, r) in enumerate(frames):
        rl, rr = ref.process_frame(l, r)
        gl, gr = trk.process_frame(l, r)
        for refl, gpul in ((rl, gl), (rr, gr)):
            assert len(refl) == len(gpul), f"frame {k}"
            assert [f[0] for f in refl] == gpul["id"].tolist()
            assert np.array_equal(np.array([f[1] for f in refl], np.float32).view(np.uint32),
                                  gpul["x"].view(np.uint32))
            assert np.array_equal(np.array([f[2] for f in refl], np.float32).view(np.uint32),
                                  gpul["y"].view(np.uint32))
            assert np.array_equal(np.array([f[3][:4] for f in refl], np.float32).reshape(-1, 4).view(np.uint32),
                                  gpul["r"].reshape(-1, 4).view(np.uint32))
    trk.close()


def test_stereo_tracker_golden(gpu):
    g = _gold("tracker_small.npz")
    w, h = int(g["w"]), int(g["h"])
    trk = gpu.StereoPatchTracker(w, h, levels=3, grid_size=30)
    rows_l, rows_r = [], []
    for k in range(4):
        fl, fr = trk.process_frame(g["left"][k], g["right"][k])
        rows_l += [(k, float(f["id"]), float(f["x"]), float(f["y"])) for f in fl]
        rows_r += [(k, float(f["id"]), float(f["x"]), float(f["y"])) for f in fr]
    assert np.array_equal(np.array(rows_l), g["pipe_l"])
    assert np.array_equal(np.array(rows_r), g["pipe_r"])


def test_stereo_tracker_pipeline(gpu, oracle, stereo_frames):
    _pipeline_compare(gpu, oracle, stereo_frames, 752, 480, 6, 50)


def test_stereo_tracker_pipeline_l3(gpu, oracle, stereo_frames):
    _pipeline_compare(gpu, oracle, stereo_frames[:3], 752, 480, 3, 30)


def test_stereo_tracker_remove_ids(gpu, stereo_frames):
    trk = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50)
    l0, r0 = stereo_frames[0]
    fl, fr = trk.process_frame(l0, r0)
    drop = fl["id"][::3]
    trk.remove_id(drop)
    l1, r1 = stereo_frames[1]
    gl, gr = trk.process_frame(l1, r1)
    assert not set(drop.tolist()) & set(gl["id"].tolist())
    assert not set(drop.tolist()) & set(gr["id"].tolist())
    assert np.all(np.diff(gl["id"].astype(np.int64)) > 0)


def test_stereo_tracker_bad_input(gpu):
    trk = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50)
    with pytest.raises(ValueError):
        trk.process_frame(np.zeros((10, 10), np.uint8), np.zeros((10, 10), np.uint8))
    with pytest.raises(gpu.RsvioError):
        gpu.StereoPatchTracker(8, 8, levels=3)


def _batch_table(lib_mod, specs, dev):
    """Device descriptor table (rsvio_track_batch[]) + int32 prefix of the batch sizes."""
    import ctypes as C

    import torch
    tb = (lib_mod.TrackBatch * len(specs))()
    for i, (p0, p1, a, o, v, n) in enumerate(specs):
        tb[i] = lib_mod.TrackBatch(p0, p1, a, o, v, n)
    raw = np.frombuffer(C.string_at(C.addressof(tb), C.sizeof(tb)), np.uint8).copy()
    start = np.concatenate([[0], np.cumsum([s[5] for s in specs])]).astype(np.int32)
    return torch.from_numpy(raw).to(dev), torch.from_numpy(start).to(dev), int(start[-1])


def test_track_points_table_batched(gpu, oracle, stereo_frames):
    """Batched serving mode: 4 stereo streams x 3 batches (cam0 temporal, cam1 temporal, stereo)
    in ONE rsvio_track_points_table_d launch, ragged sizes plus an empty batch; pyramids of 10
    images through the packed path (more than one launch's worth of pointer slots).  Every batch
    is bit-identical to the oracle."""
    import ctypes as C

    import torch

    from rsvio import _lib
    from rsvio import synthetic as S
    lib = _lib.load()
    w, h, L = 752, 480, 3
    dev = torch.device("cuda", 0)
    frames = stereo_frames
    # streams s = 0..3 track frame (s % 3) -> (s % 3) + 1; images of 5 frames (10 images), packed
    imgs = np.stack([np.stack(f) for f in frames[:4]] + [np.stack(frames[0])]).reshape(10, h, w)
    pb = int(lib.rsvio_pyramid_bytes(w, h, L))
    ctx = C.c_void_p()
    _lib.check(lib.rsvio_track_ctx_create(w, h, L, 0, C.byref(ctx)))
    try:
        d_imgs = torch.from_numpy(imgs).to(dev)
        d_pyr = torch.empty((10, pb), dtype=torch.uint8, device=dev)
        _lib.check(lib.rsvio_build_pyramids_d(ctx, d_imgs.data_ptr(), 10, d_pyr.data_ptr(), None))
        torch.cuda.synchronize()
        pyr = d_pyr.cpu().numpy()
        for i in range(10):
            assert np.array_equal(pyr[i], oracle.build_pyramid(imgs[i], L)), i
        sizes = [300, 257, 300, 1, 0, 300, 300, 300, 120, 64, 300, 299]
        specs, keep, ref = [], [], []
        for s in range(4):
            t = s % 3
            a0 = S.track_features(frames[t][0], 300)
            a1 = S.stereo_shift(a0)
            jobs = [(2 * t, 2 * t + 2, a0), (2 * t + 1, 2 * t + 3, a1), (2 * t + 2, 2 * t + 3, a0)]
            for j, (i0, i1, a) in enumerate(jobs):
                n = sizes[3 * s + j]
                a = np.ascontiguousarray(a[:n])
                da = torch.from_numpy(a).to(dev) if n else torch.zeros((1, 6), device=dev)
                do = torch.full((max(n, 1), 6), -7.0, device=dev)
                dv = torch.full((max(n, 1),), 9, dtype=torch.uint8, device=dev)
                keep += [da, do, dv]
                specs.append((d_pyr[i0].data_ptr(), d_pyr[i1].data_ptr(), da.data_ptr(), do.data_ptr(),
                              dv.data_ptr(), n))
                ref.append((i0, i1, a, do, dv))
        table, start, total = _batch_table(_lib, specs, dev)
        assert total == sum(sizes)
        _lib.check(lib.rsvio_track_points_table_d(ctx, table.data_ptr(), start.data_ptr(), len(specs), total,
                                                  20, C.c_float(0.01), None))
        torch.cuda.synchronize()
        for i0, i1, a, do, dv in ref:
            if len(a) == 0:
                assert float(do[0, 0]) == -7.0 and int(dv[0]) == 9  # empty batch untouched
                continue
            ra, rv = oracle.track_points(pyr[i0], pyr[i1], w, h, L, a)
            gv = dv[:len(a)].cpu().numpy().astype(bool)
            ga = do[:len(a)].cpu().numpy()
            assert np.array_equal(gv, rv)
            assert np.array_equal(ga.view(np.uint32), ra.view(np.uint32))
        # zero batches / zero total are no-ops; bad arguments are rejected
        assert lib.rsvio_track_points_table_d(ctx, None, None, 0, 0, 20, C.c_float(0.01), None) == 0
        assert lib.rsvio_track_points_table_d(ctx, None, None, 3, 10, 20, C.c_float(0.01), None) < 0
    finally:
        lib.rsvio_track_ctx_destroy(ctx)


def test_stereo_tracker_capacity_overflow(gpu, oracle, stereo_frames):
    """max_features smaller than one frame's new points: both cameras admit the same leading
    new points (ids consecutive, no unwritten slot counted), the call reports
    RSVIO_ERR_CAPACITY, and the lists equal the first `cap` ids of the uncapped oracle."""
    cap = 20
    trk = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50, max_features=cap)
    try:
        ref = oracle.StereoTracker(752, 480, 3, 50, 20, 0.01)
        l0, r0 = stereo_frames[0]
        rl, _ = ref.process_frame(l0, r0)
        assert len(rl) > cap  # the uncapped tracker would exceed the capacity
        with pytest.raises(gpu.RsvioError) as e:
            trk.process_frame(l0, r0)
        assert e.value.code == -4
        fl, fr = trk.get_track_points()
        assert sorted(fl) == list(range(cap)) and sorted(fr) == list(range(cap))
        for k in range(cap):  # the admitted points are the oracle's first cap points
            assert fl[k] == (rl[k][1], rl[k][2])
        # the next frame continues from a full, consistent state: ids never exceed those issued
        l1, r1 = stereo_frames[1]
        try:
            gl, gr = trk.process_frame(l1, r1)
        except gpu.RsvioError as e2:
            assert e2.code == -4
        gl, gr = trk.get_track_points()
        assert len(gl) <= cap and len(gr) <= cap
        assert max(list(gl) + list(gr)) < 2 * cap
    finally:
        trk.close()


def test_stereo_tracker_remove_ids_undistorted(gpu, stereo_frames):
    """remove_id keeps the fused unprojection aligned with the compacted feature lists."""
    from rsvio.camera import EUROC
    cl, cr = EUROC
    trk = gpu.StereoPatchTracker(752, 480, levels=3, grid_size=50)
    trk.set_cameras(cl, cr)
    l0, r0 = stereo_frames[0]
    l1, r1 = stereo_frames[1]
    trk.process_frame(l0, r0)
    fl, fr = trk.process_frame(l1, r1)
    ul, ur = trk.undistorted()
    drop = fl["id"][1::4]
    trk.remove_id(drop)
    kl, kr = ~np.isin(fl["id"], drop), ~np.isin(fr["id"], drop)
    ul2, ur2 = trk.undistorted()
    assert np.array_equal(ul2, ul[kl]) and np.array_equal(ur2, ur[kr])
    pl, pr = trk.get_track_points()
    assert sorted(pl) == sorted(fl["id"][kl].tolist()) and sorted(pr) == sorted(fr["id"][kr].tolist())
    trk.close()
