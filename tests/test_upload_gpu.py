"""rsvio_upload_async (rs-vio_amd/csrc/tracker.hip): a host-to-device copy of page-locked memory by a
kernel on the caller's stream, which bench.py's protocol step uses for the frame's two images (the
pyramids then follow without a copy-engine hand-off).  The bar is byte equality: sizes with and
without an 8-byte tail, an empty copy, and the runtime-copy fallbacks (pageable source, unaligned
destination); and a copy into a buffer the stream's next kernel reads."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _stream(torch):
    return torch.cuda.Stream(device=0)


@pytest.mark.parametrize("nbytes", [0, 1, 7, 8, 9, 4096 + 5, 752 * 480 * 2, 3 * 1024 * 1024 + 3])
def test_pinned_source_bytes_equal(gpu, nbytes):
    import torch
    from rsvio import _lib
    lib = _lib.load()
    rng = np.random.default_rng(nbytes)
    src = torch.from_numpy(rng.integers(0, 256, max(nbytes, 1), dtype=np.uint8)).pin_memory()
    dst = torch.full((max(nbytes, 1) + 64,), 0xA5, dtype=torch.uint8, device="cuda:0")
    s = _stream(torch)
    _lib.check(lib.rsvio_upload_async(dst.data_ptr(), src.data_ptr(), nbytes, s.cuda_stream))
    s.synchronize()
    got = dst.cpu().numpy()
    assert np.array_equal(got[:nbytes], src.numpy()[:nbytes])
    assert (got[nbytes:] == 0xA5).all()  # nothing past the end written


def test_pageable_source_and_unaligned_destination_fall_back(gpu):
    import torch
    from rsvio import _lib
    lib = _lib.load()
    rng = np.random.default_rng(3)
    host = rng.integers(0, 256, 100_003, dtype=np.uint8)  # pageable numpy memory
    dst = torch.zeros(100_003 + 64, dtype=torch.uint8, device="cuda:0")
    s = _stream(torch)
    _lib.check(lib.rsvio_upload_async(dst.data_ptr(), host.ctypes.data, host.size, s.cuda_stream))
    s.synchronize()
    assert np.array_equal(dst.cpu().numpy()[:host.size], host)
    pinned = torch.from_numpy(host).pin_memory()
    dst.zero_()
    _lib.check(lib.rsvio_upload_async(dst.data_ptr() + 1, pinned.data_ptr(), host.size, s.cuda_stream))
    s.synchronize()
    got = dst.cpu().numpy()
    assert got[0] == 0 and np.array_equal(got[1:1 + host.size], host)


def test_upload_then_pyramid_matches_host_pyramid(gpu):
    """The copy is ordered before the stream's next kernel: pyramids built from the uploaded images
    equal the pyramids built from the same images uploaded by the runtime."""
    import torch
    from rsvio import _lib
    lib = _lib.load()
    w, h, levels = 752, 480, 3
    rng = np.random.default_rng(11)
    imgs = torch.from_numpy(rng.integers(0, 256, (2, h, w), dtype=np.uint8)).pin_memory()
    ctx = C.c_void_p()
    _lib.check(lib.rsvio_track_ctx_create(w, h, levels, 0, C.byref(ctx)))
    try:
        pb = int(lib.rsvio_pyramid_bytes(w, h, levels))
        s = _stream(torch)
        outs = []
        for use_kernel in (True, False):
            d_img = torch.empty((2, h, w), dtype=torch.uint8, device="cuda:0")
            pyr = torch.empty((2, pb), dtype=torch.uint8, device="cuda:0")
            for _ in range(3):  # back to back on the stream, new contents each time
                if use_kernel:
                    _lib.check(lib.rsvio_upload_async(d_img.data_ptr(), imgs.data_ptr(), imgs.numel(), s.cuda_stream))
                else:
                    with torch.cuda.stream(s):
                        d_img.copy_(imgs, non_blocking=True)
                _lib.check(lib.rsvio_build_pyramids_d(ctx, d_img.data_ptr(), 2, pyr.data_ptr(), s.cuda_stream))
            s.synchronize()
            outs.append(pyr.cpu().numpy())
        assert np.array_equal(outs[0], outs[1])
    finally:
        lib.rsvio_track_ctx_destroy(ctx)
