"""Host side of the trackers' trig parity (no GPU): the restatement in rs-vio_amd/csrc/trig.hpp,
compiled for the host by tools/trig_exhaustive.cpp, equals this machine's libm sinf/cosf, and the
oracle's digest (the checker test_trig_gpu.py compares the device with) follows its definition.
The full 2^32 sweep takes ~1.5 min on 8 cores (profiles/r03_trig_exhaustive.txt); here the
|y| < pi/4 + reduce_fast range of both signs and a stride over everything else."""
import ctypes as C
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def exhaustive_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ absent")
    out = tmp_path_factory.mktemp("trig") / "trig_exhaustive"
    subprocess.run(["g++", "-O2", "-mfma", "-ffp-contract=off", "-fno-builtin", "-I",
                    str(ROOT / "rs-vio_amd" / "csrc"), str(ROOT / "tools" / "trig_exhaustive.cpp"), "-o", str(out),
                    "-lm", "-lpthread"], check=True)
    return out


@pytest.mark.parametrize("lo,hi", [(0x39000000, 0x3f800000), (0xb9000000, 0xbf800000),   # |y| in [2^-13, 1)
                                   (0x3f800000, 0x42f80000), (0xbf800000, 0xc2f80000)])  # 1 <= |y| < 124
def test_restatement_equals_libm(exhaustive_bin, lo, hi):
    r = subprocess.run([str(exhaustive_bin), hex(lo), hex(hi)], capture_output=True, text=True)
    assert r.returncode == 0 and "bit-equal" in r.stdout, r.stdout


def test_oracle_digest_definition(oracle):
    libm = C.CDLL("libm.so.6")
    libm.sinf.restype = libm.cosf.restype = C.c_float
    libm.sinf.argtypes = libm.cosf.argtypes = [C.c_float]
    first, n = 0x3e000000, 1 << 16
    m = (1 << 64) - 1
    acc = 0
    for u in range(first, first + n):
        y = float(np.uint32(u).view(np.float32))
        sb = int(np.float32(libm.sinf(y)).view(np.uint32))
        cb = int(np.float32(libm.cosf(y)).view(np.uint32))
        z = (((sb << 32) | cb) + u * 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        acc = (acc + (z ^ (z >> 31))) & m
    assert int(oracle.libm_sincosf_digest(first, n, 16, 2)[0]) == acc
