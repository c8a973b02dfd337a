"""The LK kernel's exact f32 quotients (csrc/lk_track.hip div_rcp): a / b for f32 a, b is formed
as RN_f32(a * (1/b)) in f64 with a ~2^-52 reciprocal, which equals the correctly rounded f32
division (patch.rs:222 nv v / sum, image_utilities.rs:96-97 sin / theta and (1 - cos) / theta)
because an f32 quotient is never within 2^-49 (relative) of an f32 rounding midpoint.  Checked on
the kernel's operand ranges and on random significands, with the reciprocal perturbed by up to
2 f64 ulps (the device's rcp + Newton is within that of 1/b)."""
import numpy as np


def _check(a, b):
    a, b = a.astype(np.float32), b.astype(np.float32)
    ref = (a / b).astype(np.float32)
    r = 1.0 / b.astype(np.float64)
    for pert in (-2, -1, 0, 1, 2):
        q = (a.astype(np.float64) * (r * (1.0 + pert * 2.0 ** -52))).astype(np.float32)
        assert np.array_equal(q, ref)


def test_div_rcp_kernel_ranges():
    rng = np.random.default_rng(7)
    n = 1_000_000
    th = (np.exp(rng.uniform(np.log(1.2e-7), np.log(3.0), n)) * rng.choice([-1.0, 1.0], n)).astype(np.float32)
    _check(np.sin(th).astype(np.float32), th)
    _check((1.0 - np.cos(th)).astype(np.float32), th)
    nv = rng.integers(27, 53, n).astype(np.float32)
    v = rng.uniform(0.0, 255.0, n).astype(np.float32)
    _check((nv * v).astype(np.float32), rng.uniform(1.0, 13260.0, n).astype(np.float32))


def test_div_rcp_random_significands():
    rng = np.random.default_rng(8)
    n = 1_000_000
    _check(rng.uniform(1.0, 2.0, n), rng.uniform(1.0, 2.0, n))
    _check(rng.uniform(-1e3, 1e3, n), np.exp(rng.uniform(-20, 20, n)))


def _f32_step(t, d):
    return np.frombuffer((np.frombuffer(np.float32(t).tobytes(), np.int32) + d).tobytes(), np.float32)[0]


def test_norm_threshold_without_sqrt():
    """track_at_level's norm tests (feature_tracker.rs:376-384) without the square root: for f32 x
    and a positive normal f32 t, RN(sqrt(x)) < t  <=>  x < m^2 in f64, m the midpoint of t and its
    predecessor; RN(sqrt(x)) > 1e6  <=>  x > m'^2, m' the midpoint of 1e6 and its successor.
    Every f32 x within 2^17 ulps of t^2, and random x over the whole positive range."""
    rng = np.random.default_rng(9)
    rand = np.frombuffer(rng.integers(0, 0x7F800000, 2_000_000, dtype=np.int32).tobytes(), np.float32)
    for t in (np.float32(0.01), np.float32(1e-3), np.float32(0.5), np.float32(3.0), np.float32(4.7e-38)):
        m = 0.5 * (float(_f32_step(t, -1)) + float(t))
        c = np.frombuffer(np.float32(t * t).tobytes(), np.int32)[0]
        xs = np.frombuffer(np.arange(c - 2 ** 17, c + 2 ** 17, dtype=np.int32).tobytes(), np.float32)
        for x in (xs, rand):
            assert np.array_equal(np.sqrt(x) < t, x.astype(np.float64) < m * m)
    t = np.float32(1e6)
    m = 0.5 * (float(t) + float(_f32_step(t, 1)))
    c = np.frombuffer(np.float32(t * t).tobytes(), np.int32)[0]
    xs = np.frombuffer(np.arange(c - 2 ** 17, c + 2 ** 17, dtype=np.int32).tobytes(), np.float32)
    for x in (xs, rand):
        assert np.array_equal(np.sqrt(x) > t, x.astype(np.float64) > m * m)
