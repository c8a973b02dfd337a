import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "rs-vio_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and lib/librsvio_gpu.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.load()
    return O


@pytest.fixture(scope="session")
def gpu():
    """The product library on a real device; fails (never skips) when either is missing."""
    import rsvio
    name = rsvio.require_device(int(os.environ.get("RSVIO_DEVICE", "0")))
    assert "gfx950" in name
    return rsvio


@pytest.fixture(scope="session")
def stereo_frames():
    from rsvio import synthetic as S
    return list(S.stereo_sequence(4))


@pytest.fixture(scope="session")
def scene_stream_long():
    """Config 4's rendered stereo stream at the reference window: 72 frames,
    config/euroc_vio.yaml's keyframe_window_size 10 (30 keyframes, 21 full-window solves)."""
    from rsvio import synthetic as S
    return S.euroc_scene_stream(72), 10


@pytest.fixture(scope="session")
def scene_stream(scene_stream_long):
    """The same stream shortened: its first 24 frames, window 5."""
    import dataclasses
    s, _ = scene_stream_long
    return dataclasses.replace(s, frames=s.frames[:24], T_W_B=s.T_W_B[:24]), 5
