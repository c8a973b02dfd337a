"""The C-ABI library builds, loads without a GPU and exports every symbol include/rsvio_gpu.h
declares; argument validation runs before any device call."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "rsvio_gpu.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(rsvio_\w+)\s*\(", text, re.M)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("rsvio_tracker_create", "rsvio_tracker_process_frame", "rsvio_track_points", "rsvio_build_pyramid",
              "rsvio_ba_solve", "rsvio_ba_attach_comm", "rsvio_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from rsvio import _lib
    lib = _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (rsvio_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    for s in declared_symbols():
        assert getattr(lib, s) is not None


def test_ctypes_signatures_cover_header():
    from rsvio import _lib
    assert set(declared_symbols()) <= set(_lib.SIG)


def test_struct_layouts():
    from rsvio import _lib
    assert C.sizeof(_lib.Feature) == 32
    assert C.sizeof(_lib.TrackerParams) == 32
    assert C.sizeof(_lib.TrackBatch) == 48
    assert C.sizeof(_lib.Camera) == 88
    assert C.sizeof(_lib.FtConfig) == 64
    assert C.sizeof(_lib.FtFeature) == 16


def test_camera_struct_matches_oracle_layout():
    from oracle import oracle as O
    from rsvio import _lib
    assert C.sizeof(O.OrcCamera) == C.sizeof(_lib.Camera)
    for (a, ta), (b, tb) in zip(O.OrcCamera._fields_, _lib.Camera._fields_):
        assert a == b and C.sizeof(ta) == C.sizeof(tb)


def test_invalid_arguments_rejected_without_device():
    from rsvio import _lib
    lib = _lib.load()
    assert lib.rsvio_tracker_create(None, None) == -1
    assert lib.rsvio_track_points(None, None, 10, 10, 1, None, 0, 20, C.c_float(0.01), None, None) == -1
    img = np.zeros((10, 10), np.uint8)
    n = C.c_int32()
    assert lib.rsvio_detect_keypoints(img.ctypes.data, 10, 10, 4, None, 0, None, None, 0, C.byref(n)) == -1
    assert lib.rsvio_pyramid_bytes(752, 480, 3) == 752 * 480 + 376 * 240 + 188 * 120
    assert lib.rsvio_ba_solve(None, 0, None, None, 0, None, 0, None, None, None, None, None, None, None) == -1
    cam = _lib.Camera()
    cam.model = 7
    assert lib.rsvio_unproject(C.byref(cam), None, 0, None, None) == -1      # unknown model
    cam.model, cam.params[0], cam.params[1] = 0, 0.0, 1.0
    assert lib.rsvio_unproject(C.byref(cam), None, 0, None, None) == -1      # fx == 0
    assert lib.rsvio_tracker_set_cameras(None, None, None) == -1
    # feature_tracker/ crate variant
    assert lib.rsvio_ft_create(None, None) == -1
    assert lib.rsvio_ft_pyramid_floats(752, 480, 5, 2.0) == 752 * 480 + 376 * 240 + 188 * 120 + 94 * 60 + 47 * 30
    assert lib.rsvio_ft_pyramid_floats(752, 480, 0, 2.0) == 0
    assert lib.rsvio_ft_track_points(None, None, 10, 10, 1, 2.0, None, 0, 25, C.c_float(0.1), 0, None, None) == -1
    n = C.c_int32()
    assert lib.rsvio_ft_add_points(img.ctypes.data, 10, 10, None, 0, C.c_float(2.5), 15, C.c_float(6.0), None, 0,
                                   C.byref(n)) == -1                      # 2 * min_dist >= image size
    assert lib.rsvio_ft_process_frame(None, None, 0, None, 0, None) == -1
