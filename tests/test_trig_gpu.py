"""The trackers' f32 sin/cos on the device (rs-vio_amd/csrc/trig.hpp, glibc sinf/cosf restated)
against the host's libm -- the functions Rust's f32::sin/cos call in se2_exp_matrix
(src/feature_tracker/image_utilities.rs:84) and exp_se2 (feature_tracker/src/feature_tracker/
feature_tracking.rs:199-203).  Bar: bit-exact for every f32 input (NaN payloads excepted)."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIBM = C.CDLL("libm.so.6")
LIBM.sinf.restype = LIBM.cosf.restype = C.c_float
LIBM.sinf.argtypes = LIBM.cosf.argtypes = [C.c_float]


def _device_digest(first, count, chunk_log2):
    from rsvio import _lib
    n = (count + (1 << chunk_log2) - 1) >> chunk_log2
    out = np.zeros(n, np.uint64)
    _lib.check(_lib.load().rsvio_sincosf_digest(first, count, chunk_log2, out.ctypes.data))
    return out


def test_sincosf_special_values(gpu):
    from rsvio import _lib
    bits = [0x00000000, 0x80000000, 0x00000001, 0x807fffff, 0x397fffff, 0x39800000, 0xb9800000,
            0x3f490fda, 0x3f490fdb, 0x3f490fdc, 0xbf490fdb, 0x42efffff, 0x42f00000, 0xc2f00000,
            0x4255b0a9, 0xc255b0a9, 0x7f7fffff, 0xff7fffff, 0x7f800000, 0xff800000, 0x7fc00000,
            0x3fc90fdb, 0x40490fdb, 0x40c90fdb, 0x461c4000, 0x4b800000, 0x5a000000]
    rng = np.random.default_rng(7)
    bits = np.concatenate([np.array(bits, np.uint32), rng.integers(0, 2 ** 32, 4096, dtype=np.uint64).astype(np.uint32),
                           np.float32(rng.uniform(-0.8, 0.8, 4096)).view(np.uint32)])
    x = bits.view(np.float32)
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    _lib.check(_lib.load().rsvio_sincosf(x.ctypes.data, len(x), s.ctypes.data, c.ctypes.data))
    for i, v in enumerate(x):
        ls, lc = np.float32(LIBM.sinf(float(v))), np.float32(LIBM.cosf(float(v)))
        for got, want in ((s[i], ls), (c[i], lc)):
            assert (np.isnan(got) and np.isnan(want)) or got.view(np.uint32) == want.view(np.uint32), hex(bits[i])


def test_sincosf_all_f32_inputs(gpu, oracle):
    """All 2^32 bit patterns, 256 chunk digests each side (host libm on <= 16 threads)."""
    threads = min(16, os.cpu_count() or 1)
    dev = _device_digest(0, 1 << 32, 24)
    host = oracle.libm_sincosf_digest(0, 1 << 32, 24, threads)
    assert len(np.unique(host)) == len(host) and (host != 0).all()  # 256 live, distinct digests
    bad = np.nonzero(dev != host)[0]
    assert len(bad) == 0, [hex(int(k) << 24) for k in bad[:8]]
