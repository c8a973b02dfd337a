"""set_problem's chunked observation pass (rs-vio_amd/csrc/obs_pass.hpp) on the CPU.

The pass is host code of rsvio_ba_set_problem (the window hand-over of
src/estimator/sliding_window.rs:274-300): keys, per-landmark masks and the (u, v) narrowed to
f32, cut into landmark-run-aligned chunks over a helper-thread pool.  tools/obs_pass_bench.cpp
compiles the header with g++ and checks, over many repetitions, that the pooled pass writes exactly
what the single-threaded pass writes, and that a landmark split over two runs and a duplicate
observation are rejected (set_problem then takes its exact pass).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ absent")
    out = str(tmp_path_factory.mktemp("obs") / "obs_pass_bench")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "rs-vio_amd", "csrc"),
                    os.path.join(ROOT, "tools", "obs_pass_bench.cpp"), "-o", out], check=True)
    return out


@pytest.mark.parametrize("threads,n_lm", [("3", "2000"), ("1", "2000"), ("0", "2000"), ("3", "700"),
                                          ("7", "5000")])
def test_pooled_pass_equals_single_pass(bench_bin, threads, n_lm):
    env = dict(os.environ, RSVIO_BA_HOST_THREADS=threads)
    r = subprocess.run([bench_bin, n_lm, "200"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "equal 1; split rejected 1, duplicate rejected 1" in r.stdout, r.stdout
