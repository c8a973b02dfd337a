#!/usr/bin/env python3
"""bench.py -- stereo frames/sec (tracker + BA) on the synthetic EuRoC-shaped stream.

One step = one stereo frame of BASELINE.json config 2 through the patch tracker (2 pyramids,
L=3, + track_points x 3: cam0 temporal, cam1 temporal, cam0->cam1 stereo, 300 features each,
forward + backward) and one full sliding-window BA solve of config 3 (10 keyframes, KF_0 fixed,
2000 landmarks per GPU, 24,000 observations per GPU, LM to convergence, <= 20 iterations) --
every frame is treated as a keyframe (worst case of estimator.rs:243-246).

`value` is BASELINE.md's protocol step, the median of --reps repetitions: the two images go up
from pinned host memory, the three tracked feature lists come back, a NEW keyframe window is
uploaded (rsvio_ba_set_problem; two pre-built windows alternate) and solved, and its optimised
state comes back -- all inside the timed region.  `value_resident` is the device-resident step
(images and the window already in HBM, the same window re-solved from its captured graph).

Multi-GPU (torchrun, one process per GPU): the tracker runs as independent replicas (each rank
its own stream); the BA is ONE problem whose landmarks are sharded 2000 per rank (weak scaling)
with an RCCL all-reduce of the reduced camera system per LM iteration.  value = frames of all
ranks / max-over-ranks time.

Also reported: BA ms per LM iteration, tracker ms per frame, the dominant kernel's roofline
(HIP events on the stream it runs on) and the CPU oracle baseline on the host cores (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import resource
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]

import numpy as np  # noqa: E402

METRIC = "stereo frames/sec (tracker+BA) on 752×480 EuRoC stream; BA ms/iter at window=10"
W, H, LEVELS, NFEAT = 752, 480, 3, 300
MAX_IT, THRESH = 20, 0.01
N_FRAMES = 4                       # palindromic cycle 0,1,2,3,2,1,0,... (one frame of motion per step)
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md: 8 TB/s spec
FP64_PEAK_TFLOPS = 78.6            # MI355X FP64 vector (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------------------
# Algorithmic work per unit, frozen here and in DESIGN.md
# ---------------------------------------------------------------------------------------
def tracker_bytes_per_frame(calls: int) -> int:
    """2 pyramids (source reads + level writes) + 11x11 patch footprint per (call, level) in
    template and target image + 48 B feature state per call."""
    pyr = 2 * ((LEVELS - 1) * W * H + sum((W >> i) * (H >> i) for i in range(1, LEVELS)))
    return pyr + calls * LEVELS * 2 * 121 + calls * 48


def lk_bytes_per_launch(calls: int) -> int:
    return calls * LEVELS * 2 * 121 + calls * 48


def ba_flops_per_iter(n_obs: int, n_lm: int, k_per_lm: int, n_free: int) -> float:
    """F = N_obs (470 + 50) + sum_l [30 + K 108 + K(K+1)/2 216 + K 36 + (K 36 + 18)] + n^3/3 + 2 n^2."""
    K = k_per_lm
    per_lm = 30 + K * 108 + K * (K + 1) / 2 * 216 + K * 36 + (K * 36 + 18)
    n = 6 * n_free
    return n_obs * 520 + n_lm * per_lm + n ** 3 / 3 + 2 * n * n


# ---------------------------------------------------------------------------------------
PNP_FLOP_PER_OBS_PASS = 318   # pnp_linearize (~183) + Huber + 21+6 H/g accumulations (~135), per observation
UNPROJ_BYTES_PER_POINT = 17    # 8 B pixel in, 8 B undistorted out, 1 B valid


def measure_rows(device: int, cpu: bool, reps: int = 200):
    """The §8 rows beside the headline path, each on its own config-shaped input, timed with HIP
    events on the stream its kernel runs on (inputs resident on the device):
      * T12 unprojection: config 5's batch, 80,000 EUCM (TUM-VI cam0) observations;
      * B8 track_motion + keyframe rule: one frame of 300 features per camera (600 mapped
        observations, 40 unmapped per camera) against a 2,000-point map, EuRoC extrinsics.
    The oracle's time on the same inputs (1 host thread) is reported beside each."""
    import torch

    from rsvio import synthetic as S
    from rsvio.camera import TUM_VI
    from rsvio.motion import MotionTracker
    out = {}
    st = torch.cuda.Stream(device)
    # --- T12
    n = 80000
    rng = np.random.default_rng(5)
    px = np.stack([rng.uniform(0, 512, n), rng.uniform(0, 512, n)], 1).astype(np.float32)
    d_px = torch.from_numpy(px).to(f"cuda:{device}")
    d_out = torch.empty_like(d_px)
    d_ok = torch.empty(n, dtype=torch.uint8, device=d_px.device)
    torch.cuda.synchronize()
    cam = TUM_VI[0]
    for _ in range(10):
        cam.unproject_device(d_px.data_ptr(), n, d_out.data_ptr(), d_ok.data_ptr(), st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the reps launches captured once and replayed back to back, so the events time the kernels,
    # not the host's Python + ctypes enqueue rate (on a loaded host that was ~13 us per launch,
    # 3x the kernel); the direct loop if capture is unavailable
    timed_by = "graph"
    try:
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                cam.unproject_device(d_px.data_ptr(), n, d_out.data_ptr(), d_ok.data_ptr(), st.cuda_stream)
        with torch.cuda.stream(st):
            g.replay()
            e0.record(st)
            g.replay()
            e1.record(st)
        st.synchronize()
    except RuntimeError:
        timed_by = "direct launches"
        e0.record(st)
        for _ in range(reps):
            cam.unproject_device(d_px.data_ptr(), n, d_out.data_ptr(), d_ok.data_ptr(), st.cuda_stream)
        e1.record(st)
        st.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = n * UNPROJ_BYTES_PER_POINT / (ms * 1e-3) / 1e9
    row = {"workload": "80,000 EUCM observations (config 5 batch), plane convention",
           "value": round(n / (ms * 1e-3), 1), "unit": "points/s", "kernel": "unproject_kernel",
           "launch_ms": round(ms, 5), "timed_by": timed_by,
           "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 6),
                        "algorithmic_bytes_per_launch": n * UNPROJ_BYTES_PER_POINT,
                        "note": "launch-latency bound at this size (1.36 MB)"}}
    if cpu:
        from oracle import oracle as O
        oc = O.camera(cam.model, cam.params, 0, cam.max_iterations)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 1.0 or k < 3:
            O.unproject(oc, px)
            k += 1
        cms = 1e3 * (time.perf_counter() - t0) / k
        row["cpu_baseline"] = {"value": round(n / (cms * 1e-3), 1), "unit": "points/s", "cores": 1, "kind": "port",
                               "sample": f"{k} x 80,000 points, oracle/camera_oracle.cpp"}
    out["unproject"] = row
    # --- B8
    m = S.motion_frame(seed=3)
    mt = MotionTracker(device)
    mt.set_stream(st.cuda_stream)
    mt.set_map(m.map_ids, m.map_pw)
    for _ in range(5):
        r = mt.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.T_W_B_last_kf, m.T_C_B2)
    evs, kms = [], []
    t0 = time.perf_counter()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        r = mt.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.T_W_B_last_kf, m.T_C_B2)
        b.record(st)
        evs.append((a, b))
        kms.append(r.kernel_ms)
    host_ms = 1e3 * (time.perf_counter() - t0) / reps
    st.synchronize()
    # call_ms: the events around the whole call (feature upload, kernel, the call's own stream
    # synchronisation and the host-side return before the second record); launch_ms: the kernel
    # alone, from the device wall clock the kernel reads at entry and at its result write
    call_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    ms = float(np.mean(kms))
    passes = 1 + r.iterations
    flops = PNP_FLOP_PER_OBS_PASS * r.n_observations * passes
    tf = flops / (ms * 1e-3) / 1e12
    row = {"workload": "1 frame: 300 features/camera (600 mapped observations) vs a 2,000-point map, "
                       "PnP LM <= 10 it + keyframe rule",
           "value": round(1e3 / call_ms, 1), "unit": "frames/s", "kernel": "pnp_track_motion_kernel",
           "launch_ms": round(ms, 5), "call_ms": round(call_ms, 5), "host_inclusive_ms": round(host_ms, 4),
           "lm_iterations": r.iterations, "status": r.status, "observations": r.n_observations,
           "roofline": {"bound": "fp64", "achieved": round(tf, 5), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tf / FP64_PEAK_TFLOPS, 8), "flop_per_launch": flops,
                        "note": "one workgroup by design (a serial LM of <= 10 dependent 6x6 solves)"}}
    if cpu:
        from oracle import oracle as O
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 1.0 or k < 3:
            O.track_motion(m.ids_l, m.uv_l, m.ids_r, m.uv_r, m.map_ids, m.map_pw, m.T_W_B_last_kf, m.T_C_B2)
            k += 1
        cms = 1e3 * (time.perf_counter() - t0) / k
        row["cpu_baseline"] = {"value": round(1e3 / cms, 1), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{k} frames, oracle orc_track_motion"}
    out["track_motion"] = row
    mt.close()
    out["ba_config5"] = measure_config5_row(device, cpu)
    out["ba_batched"] = measure_ba_batched_row(device, 16)
    out["ba_batched_64"] = measure_ba_batched_row(device, 64, reps=5)
    out["ft_tracker"] = measure_ft_row(device, cpu)
    return out


def measure_ba_batched_row(device: int, n_windows: int = 16, reps: int = 10):
    """SURVEY 8d "batched mode" for HP-B: B independent config-3 windows (10 KF x 2,000
    landmarks, distinct seeds) solved by ONE launch chain (rsvio_ba_batch_run: the window is a
    grid dimension of every LM kernel, one camera-solve workgroup per window), every window to
    convergence.  value = solves per second over `reps` batch solves (host wall time around
    rsvio_ba_batch_run); roofline: FP64 work of the LM iterations every window ran / that time,
    and the chain's device time (HIP events on the batch stream, solve_ms)."""
    from rsvio import synthetic as S
    from rsvio.ba import BundleAdjuster, BundleBatch
    probs = [S.ba_problem(seed=7 + 101 * i, init_seed=11 + 101 * i) for i in range(n_windows)]
    bas = [BundleAdjuster(max_keyframes=p.n_kf, max_landmarks=p.n_lm, max_observations=p.n_obs, device=device)
           for p in probs]
    for b, p in zip(bas, probs):
        b.set_problem_from(p)
    batch = BundleBatch(bas)
    for _ in range(2):                                   # warm-up (and sets the chunk size)
        batch.run()
    iters, dev_ms, chain_its = 0, [], []
    t0 = time.perf_counter()
    for _ in range(reps):
        res = batch.run()
        iters += sum(r.iterations for r in res)
        dev_ms.append(res[0].solve_ms)
        chain_its.append(max(r.iterations for r in res))
    el = time.perf_counter() - t0
    p0 = probs[0]
    flops = ba_flops_per_iter(p0.n_obs, p0.n_lm, 6, int((p0.kf_fixed == 0).sum())) * iters
    ach = flops / el / 1e12
    ach_dev = flops / (1e-3 * sum(dev_ms)) / 1e12
    batch.close()
    for b in bas:
        b.close()
    n = n_windows * reps
    return {"workload": f"{n_windows} independent config-3 windows (10 KF x 2,000 landmarks, 24,000 observations "
                        "each) solved by one batched launch chain (rsvio_ba_batch_run)",
            "value": round(n / el, 1), "unit": "solves/s", "windows": n_windows,
            "ms_per_batch": round(1e3 * el / reps, 4), "device_ms_per_batch": round(float(np.median(dev_ms)), 4),
            "lm_iterations_mean": round(iters / n, 2), "chain_iterations_mean": round(float(np.mean(chain_its)), 2),
            "roofline": {"bound": "fp64", "achieved": round(ach, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ach / FP64_PEAK_TFLOPS, 6), "achieved_device_time": round(ach_dev, 4),
                         "frac_device_time": round(ach_dev / FP64_PEAK_TFLOPS, 6),
                         "note": "one launch chain for all windows: K4, then per LM iteration K4c (B x 360 "
                                 "workgroups), K5 (B workgroups), K6 (B x waves), K7 per chunk"}}

def measure_config5_row(device: int, cpu: bool, reps: int = 10):
    """BASELINE config 5: TUM-VI EUCM, window 20 x 5,000 landmarks (80,000 observations).  The
    observations arrive as EUCM pixels and are batch-unprojected on the device (T12, one launch per
    camera), then the sliding-window BA solves from the same initial state `reps` times (solve time
    from the library's HIP events on the BA stream, LM to convergence)."""
    import torch

    from rsvio import synthetic as S
    from rsvio.ba import BundleAdjuster
    from rsvio.camera import TUM_VI
    prob, px = S.config5_problem(TUM_VI)
    dev = f"cuda:{device}"
    st = torch.cuda.Stream(device)
    d_px = torch.from_numpy(px).to(dev)
    d_uv = torch.empty_like(d_px)
    d_ok = torch.empty(prob.n_obs, dtype=torch.uint8, device=dev)
    sel = [torch.from_numpy(np.nonzero(prob.obs_cam == c)[0]).to(dev) for c in range(2)]
    parts = [d_px[i].contiguous() for i in sel]
    outs = [torch.empty_like(p) for p in parts]
    oks = [torch.empty(len(p), dtype=torch.uint8, device=dev) for p in parts]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for c in range(2):
        TUM_VI[c].unproject_device(parts[c].data_ptr(), len(parts[c]), outs[c].data_ptr(), oks[c].data_ptr(),
                                   st.cuda_stream)
    e1.record(st)
    st.synchronize()
    unproj_ms = e0.elapsed_time(e1)
    for c in range(2):
        d_uv[sel[c]] = outs[c]
        d_ok[sel[c]] = oks[c]
    n_valid = int(d_ok.sum().item())
    obs_uv = d_uv.double().cpu().numpy()
    err = float(np.abs(obs_uv - prob.obs_uv).max())
    prob.obs_uv = obs_uv
    ba = BundleAdjuster(max_keyframes=prob.n_kf, max_landmarks=prob.n_lm, max_observations=prob.n_obs, device=device)
    ba.set_problem_from(prob)
    r = ba.run()
    ms, its = [], []
    for _ in range(reps):
        r = ba.run()
        ms.append(r.solve_ms)
        its.append(r.iterations)
    ba.close()
    solve_ms = float(np.median(ms))
    it = float(np.median(its))
    ms_iter = solve_ms / max(it, 1.0)
    flops = ba_flops_per_iter(prob.n_obs, prob.n_lm, 8, int((prob.kf_fixed == 0).sum()))
    tf = flops / (ms_iter * 1e-3) / 1e12
    row = {"workload": "config 5: TUM-VI EUCM, window 20 (19 free KF) x 5,000 landmarks x 8 KF x 2 cams = "
                       "80,000 pixel observations, device unprojection then Schur LM <= 20 it",
           "value": round(ms_iter, 4), "unit": "ms/iter", "higher_is_better": False,
           "ba_ms_per_solve": round(solve_ms, 4), "lm_iterations": it, "status": r.status,
           "unproject_ms": round(unproj_ms, 4), "unprojected_valid": n_valid,
           "unproject_max_err_vs_true_plane": err,
           "roofline": {"bound": "fp64", "achieved": round(tf, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tf / FP64_PEAK_TFLOPS, 6), "flop_per_iter": flops,
                        "note": "latency-bound LM chain (3 kernels per iteration, serial 114x114 solve)"}}
    if cpu:
        legs = [cpu_ba_leg(prob, host_cores(), 3.0, "config-5"), cpu_ba_leg(prob, 1, 2.0, "config-5")]
        row["cpu_baseline"] = dict(legs[0], single_thread=legs[1])
    return row


def cpu_ba_leg(prob, threads: int, budget_s: float, name: str) -> dict:
    """The oracle's BA solve on the host: `threads` = 1 is the sequential reference order, more
    is the threaded Schur variant (landmark ranges in parallel, BASELINE.md's nproc leg)."""
    from oracle import oracle as O
    O.set_ba_threads(threads)
    try:
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < budget_s or k < 2:
            _, _, rr = O.ba_solve(prob)
            k += 1
        cms = 1e3 * (time.perf_counter() - t0) / k
    finally:
        O.set_ba_threads(1)
    return {"value": round(cms / max(rr.iterations, 1), 3), "unit": "ms/iter", "cores": threads, "kind": "port",
            "ms_per_solve": round(cms, 2), "lm_iterations": rr.iterations,
            "sample": f"{k} {name} solves, oracle/ba_oracle.cpp, " +
                      ("1 thread" if threads == 1 else f"{threads} threads (threaded Schur: landmark ranges)")}


class _StageTimer:
    """Wraps an Estimator backend: wall time per stage (track / track_motion / BA solve)."""

    def __init__(self, be):
        self.be, self.t = be, {"track": 0.0, "track_motion": 0.0, "ba": 0.0, "ba_wait": 0.0}
        self.n_solves = 0
        self.ba_iters = 0
        outer = self

        class Solver:
            """Times the solver's host calls: "ba" = problem upload + enqueue (or a synchronous
            solve), "ba_wait" = waiting for an in-flight solve and reading its state back."""

            def solve(self, *a, **k):
                t0 = time.perf_counter()
                r = be.solver.solve(*a, **k)
                outer.t["ba"] += time.perf_counter() - t0
                outer.n_solves += 1
                outer.ba_iters += r[2].iterations
                return r

            def set_problem(self, *a):
                t0 = time.perf_counter()
                be.solver.set_problem(*a)
                outer.t["ba"] += time.perf_counter() - t0

            def run_async(self, cfg=None):
                t0 = time.perf_counter()
                be.solver.run_async(cfg)
                outer.t["ba"] += time.perf_counter() - t0

            def wait(self):
                t0 = time.perf_counter()
                r = be.solver.wait()
                outer.t["ba_wait"] += time.perf_counter() - t0
                outer.n_solves += 1
                outer.ba_iters += r.iterations
                return r

            def state(self):
                t0 = time.perf_counter()
                r = be.solver.state()
                outer.t["ba_wait"] += time.perf_counter() - t0
                return r
        self.solver = Solver()

    def track(self, l, r):
        t0 = time.perf_counter()
        out = self.be.track(l, r)
        self.t["track"] += time.perf_counter() - t0
        return out

    def submit(self, l, r):
        t0 = time.perf_counter()
        self.be.submit(l, r)
        self.t["track"] += time.perf_counter() - t0

    def collect(self):
        """(Estimator.run) the wait for a frame submitted one frame earlier, plus its read-out"""
        t0 = time.perf_counter()
        out = self.be.collect()
        self.t["track"] += time.perf_counter() - t0
        return out

    def track_motion(self, *a):
        t0 = time.perf_counter()
        out = self.be.track_motion(*a)
        self.t["track_motion"] += time.perf_counter() - t0
        return out

    def set_map(self, *a):
        return self.be.set_map(*a)


def measure_pipeline_row(device: int, cpu: bool, n_frames: int = 500, cpu_seconds: float = 40.0,
                         native: bool = True, ba_cus=None):
    """BASELINE config 4 on one GPU: the Estimator (estimator.rs:101-262) over the device backend
    on a rendered stereo stream of textured planes (synthetic.euroc_scene_stream_device, frames
    resident in HBM): per frame the tracker (6 levels, grid 50, fused radtan unprojection), PnP +
    keyframe rule once the window is full, and a window-10 BA per keyframe; host logic in Python
    between the device calls.  Pipelined: a keyframe's BA runs on its own stream while the next
    frame is tracked (Estimator(pipelined=True)), and the tracker runs one frame ahead
    (Estimator.run: frame t + 1 is submitted as soon as frame t's features are back, so frame t's
    host logic, PnP and BA start overlap its tracking); outputs equal the sequential order's
    (tests/test_estimator_*).  value = frames / wall time over the whole stream.  With the CPU
    leg, the row is checked frame by frame against the oracle Estimator (keyframe flags, PnP and
    BA status and iteration counts, pose within 1e-6): a divergent frame FAILS the row (value
    null, "parity": "failed")."""
    import torch

    from rsvio import synthetic as S
    from rsvio.camera import Camera
    from rsvio.estimator import DeviceBackend, Estimator, NativeEstimator
    dev = f"cuda:{device}"
    s = S.euroc_scene_stream_device(n_frames, dev)
    torch.cuda.synchronize()
    cams = [Camera.opencv5(*p) for p in s.intrinsics]

    def run(frames):
        be = _StageTimer(DeviceBackend(W, H, cams, 6, 50, MAX_IT, THRESH, 10, 0.05, 0.05, device, ba_cus=ba_cus))
        if native:  # the host logic in C++ (rsvio.estimator.NativeEstimator): the same calls
            est = NativeEstimator(be.be, s.T_B_Cl, s.T_B_Cr, window=10)
            t0 = time.perf_counter()
            out = est.run(frames)
            el = time.perf_counter() - t0
            st = est.stats
            be.t = {"track": st.track, "track_motion": st.track_motion, "ba": st.ba, "ba_wait": st.ba_wait}
            be.n_solves, be.ba_iters = st.n_solves, st.ba_iterations
        else:
            est = Estimator(W, H, cams, s.T_B_Cl, s.T_B_Cr, window=10, backend=be, pipelined=True)
            t0 = time.perf_counter()
            out = list(est.run(frames))
            est.flush()
            el = time.perf_counter() - t0
        be.be.close()
        return out, el, be

    run(s.frames[:30])                               # warm-up: first launches, allocations
    out, el, be = run(s.frames)
    n_kf = sum(r.is_keyframe for r in out)
    err = max(float(np.linalg.norm(r.T_W_B[:3, 3] - T[:3, 3])) for r, T in zip(out, s.T_W_B))
    row = {"workload": f"config 4: Estimator::process_frame over {n_frames} rendered 752x480 stereo frames "
                       "(textured planes at 3-8 m, EuRoC radtan rig, 0.02 m/frame); tracker L=6 grid 50 + "
                       "unprojection, PnP + keyframe rule, window-10 BA per keyframe (pipelined: the solve overlaps the "
                       "next frame's tracking; the tracker one frame ahead: frame t+1 tracks during frame t's PnP and BA start)",
           "value": round(n_frames / el, 3), "unit": "frames/s", "higher_is_better": True,
           "ms_per_frame": round(1e3 * el / n_frames, 4), "keyframes": n_kf, "ba_solves": be.n_solves,
           "ba_lm_iterations_mean": round(be.ba_iters / max(be.n_solves, 1), 2),
           "features_per_camera_mean": round(float(np.mean([r.n_left for r in out])), 1),
           "stage_ms_per_frame": {k: round(1e3 * v / n_frames, 4) for k, v in be.t.items()},
           "host_ms_per_frame": round(1e3 * (el - sum(be.t.values())) / n_frames, 4),
           "max_position_error_m": round(err, 5),
           "host_logic": "C++ (rsvio.estimator.NativeEstimator, lib/librsvio_host.so)" if native
                         else "Python (rsvio.estimator.Estimator)",
           "note": "frames already in HBM; stage times are host wall time around each device call "
                   "(each returns its results to the host, as the reference API does)"}
    if cpu:
        from oracle import oracle as O
        from oracle.estimator import OracleBackend, outcome_difference
        host = [(l.cpu().numpy(), r.cpu().numpy()) for l, r in s.frames]

        def oracle_leg(threads, budget_s, compare):
            """The same Estimator host logic over the oracle backend: `threads` = 1 sequential,
            more = the tracker's levels / features and the Schur BA threaded (rayon analogue)."""
            ob = _StageTimer(OracleBackend(O, W, H, cams, threads=threads))
            O.set_ba_threads(threads)
            est = Estimator(W, H, cams, s.T_B_Cl, s.T_B_Cr, window=10, backend=ob)
            t0 = time.perf_counter()
            k, oerr, first, maxd = 0, 0.0, None, 0.0
            try:
                # the whole stream when it fits the budget: frame-by-frame parity of the device run
                # (keyframe flags, PnP / BA status, pose) and the oracle's drift on the same frames
                while k < len(host) and (time.perf_counter() - t0 < budget_s or k < 30):
                    ro = est.process_frame(*host[k])
                    oerr = max(oerr, float(np.linalg.norm(ro.T_W_B[:3, 3] - s.T_W_B[k][:3, 3])))
                    if compare:
                        rd = out[k]
                        d = float(np.abs(rd.T_W_B - ro.T_W_B).max())
                        maxd = max(maxd, d)
                        if first is None and (d > 1e-6 or outcome_difference(rd, ro) is not None):
                            first = k
                    k += 1
            finally:
                O.set_ba_threads(1)
            cel = time.perf_counter() - t0
            return k, cel, oerr, first, maxd, ob

        k, cel, oerr, first, maxd, ob = oracle_leg(1, cpu_seconds, True)
        gerr_k = max(float(np.linalg.norm(r.T_W_B[:3, 3] - T[:3, 3])) for r, T in zip(out[:k], s.T_W_B[:k]))
        row["oracle_max_position_error_m"] = round(oerr, 5)
        row["oracle_frames"] = k
        row["gpu_max_position_error_m_same_frames"] = round(gerr_k, 5)
        row["first_divergent_frame"] = first
        row["max_pose_diff_vs_oracle"] = maxd
        row["parity_checks"] = ("per frame: keyframe flag, PnP status + LM iterations and BA status + LM "
                                "iterations exactly (oracle/estimator.py outcome_difference); T_W_B within 1e-6")
        row["parity"] = "ok" if first is None else "failed"
        if first is not None:  # a number whose outputs differ from the reference path's is no result
            row["value_unchecked"] = row["value"]
            row["value"] = None
            print(f"[bench] config-4 row FAILED parity at frame {first}", file=sys.stderr)
        single = {"value": round(k / cel, 3), "unit": "frames/s", "cores": 1, "kind": "port",
                  "sample": f"the first {k} frames of the same stream through the same Estimator "
                            "host logic over the oracle (oracle/estimator.py), 1 thread",
                  "stage_ms_per_frame": {kk: round(1e3 * v / k, 3) for kk, v in ob.t.items()}}
        nt = host_cores()
        k2, cel2, _, _, _, ob2 = oracle_leg(nt, min(cpu_seconds / 2, 20.0), False)
        row["cpu_baseline"] = {"value": round(k2 / cel2, 3), "unit": "frames/s", "cores": nt, "kind": "port",
                               "sample": f"the first {k2} frames through the oracle backend with {nt} threads "
                                         "(tracker levels / features and the Schur BA threaded)",
                               "stage_ms_per_frame": {kk: round(1e3 * v / k2, 3) for kk, v in ob2.t.items()},
                               "single_thread": single}
    return row


FT_LEVELS = 5                  # feature_tracker/config/config.yaml


def ft_bytes_per_frame(n_tracked: int, w: int = W, h: int = H, levels: int = FT_LEVELS) -> int:
    """Algorithmic HBM bytes of one FeatureTracker frame: pyramid (blur:
    read + write the image; each level: read the previous level + write itself), Shi-Tomasi
    (grad: read 1 + write 3 planes; fast_blur: 6 half passes over 3 planes, read + write; score:
    read 3 + write 1; NMS: read 1 -> 45 plane passes) and LK (2 calls per tracked feature, an 18x18
    f32 bicubic footprint of the 52-point pattern in template and target image per (call, level),
    16 B of feature state per call)."""
    dims = [(w, h)] + [(int(w / 2 ** l + 0.5), int(h / 2 ** l + 0.5)) for l in range(1, levels)]
    px = [a * b for a, b in dims]
    pyr = 4 * (2 * px[0] + sum(px[l - 1] + px[l] for l in range(1, levels)))
    det = 4 * 45 * w * h
    calls = 2 * n_tracked
    return pyr + det + calls * levels * 2 * 18 * 18 * 4 + calls * 16


def measure_ft_row(device: int, cpu: bool, reps: int = 60):
    """T-sec: the feature_tracker/ crate's FeatureTracker::process_frame (feature_tracker.rs:77-185)
    on a 752x480 f32 mosaic stream with config.yaml's parameters; frames resident on the device;
    per-frame device time from HIP events on the tracker's stream; the frame list is read back
    every frame (the API returns it)."""
    import torch

    from rsvio import ft
    from rsvio import synthetic as S
    frames = list(S.mono_sequence(6))
    d = torch.from_numpy(np.stack(frames)).to(f"cuda:{device}")
    torch.cuda.synchronize()
    order = [0, 1, 2, 3, 4, 5, 4, 3, 2, 1]          # palindromic: one frame of motion per step
    t = ft.FeatureTracker(W, H, device=device)
    for k in range(10):
        t.process_frame_device(d[order[k % len(order)]].data_ptr())
    st = torch.cuda.ExternalStream(t.stream, device=f"cuda:{device}")
    evs, nfeat = [], []
    t0 = time.perf_counter()
    for k in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        nfeat.append(t.process_frame_device(d[order[k % len(order)]].data_ptr()))
        b.record(st)
        evs.append((a, b))
    wall = (time.perf_counter() - t0) / reps
    st.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
    n = float(np.mean(nfeat))
    byts = ft_bytes_per_frame(int(n))
    gbs = byts / (ms * 1e-3) / 1e9
    t.close()
    row = {"workload": "feature_tracker crate FeatureTracker::process_frame, 752x480 f32 mosaic stream, "
                       "config.yaml (5 levels, blur 2.0, Shi-Tomasi blur 6.0, min_dist 15, LM 25 it, lambda 0.1)",
           "value": round(1.0 / wall, 1), "unit": "frames/s", "features_per_frame": round(n, 1),
           "device_ms_per_frame": round(ms, 4), "host_inclusive_ms": round(wall * 1e3, 4),
           "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 6), "algorithmic_bytes_per_frame": byts,
                        "note": "whole frame (pyramid + LK + Shi-Tomasi); latency-bound: serial LK chains "
                                "(ft_lk_kernel 254 us of 0.56 ms per frame) and fast_blur's sequential running "
                                "sums (ft_boxblur_half 6 x 23 us) -- profiles/r04m_ft_kstats.txt"}}
    if cpu:
        from oracle import oracle as O
        ref = O.FeatureTracker(W, H)
        ref.process_frame(frames[0])
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 3.0 or k < 5:
            ref.process_frame(frames[order[(k + 1) % len(order)]])
            k += 1
        cms = 1e3 * (time.perf_counter() - t0) / k
        row["cpu_baseline"] = {"value": round(1e3 / cms, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{k} frames of the same stream, oracle/ft_oracle.cpp, 1 thread"}
    return row


def pmc_traffic(kernel: str, shape: str = "u8_gath"):
    """HBM bytes per dispatch of `kernel` from the newest committed PMC summary
    profiles/*_pmc_traffic.json (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the
    headline bench command, tools/gpu_round.sh + tools/pmc_summary.py), corrected as the
    MI355X guide's HBM section prescribes: FETCH_SIZE x the multiplier measured for this access
    shape by tools/fetch_calib.hip (profiles/*_fetch_calib.json; the guide's x2 for wide
    16-B-per-lane reads when no calibration is committed), + WRITE_SIZE.  Returns
    (corrected bytes, details) or (None, None)."""
    files = sorted((ROOT / "profiles").glob("*_pmc_traffic.json"))
    if not files:
        return None, None
    ks = json.load(open(files[-1]))["kernels"]
    # summary keys carry the template instantiation ("void lk_track_kernel<3>")
    k = ks.get(kernel) or next((v for n, v in ks.items() if n.split("<")[0].split()[-1] == kernel), None)
    if not k:
        return None, None
    mult, msrc = 2.0, "guide x2 (wide reads)"
    cal = sorted((ROOT / "profiles").glob("*_fetch_calib.json"))
    if cal:
        c = json.load(open(cal[-1]))["kernels"].get(shape)
        # a calibration outside [1/4, 8] is a broken measurement (e.g. loads the compiler
        # deleted), never a counter correction: keep the guide's x2 then
        if c and c.get("multiplier") and 0.25 <= float(c["multiplier"]) <= 8.0:
            mult, msrc = float(c["multiplier"]), f"{cal[-1].name}:{shape}"
    f, w = k["fetch_size_bytes_per_dispatch"], k["write_size_bytes_per_dispatch"]
    return f * mult + w, {"source": files[-1].name, "fetch_raw": round(f), "write_raw": round(w),
                          "fetch_multiplier": round(mult, 4), "multiplier_source": msrc}


def _read_text(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _minor_faults() -> int:
    """This process's minor page faults so far (/proc/self/stat field 10)."""
    t = _read_text("/proc/self/stat")
    return int(t.rsplit(")", 1)[1].split()[7]) if t else -1


def tame_malloc():
    """glibc malloc without trimming and with a fixed 32 MB mmap threshold (mallopt): freed heap
    memory stays mapped, so a later allocation of it does not page-fault again.  Diagnostic A/B
    for the one-rep stall (a ~16 MB burst of the main thread's minor faults inside one
    set_problem, profiles/r06e_*)."""
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    m_trim_threshold, m_mmap_threshold = -1, -3
    ok = libc.mallopt(m_mmap_threshold, 32 << 20) == 1 and libc.mallopt(m_trim_threshold, 1 << 30) == 1
    log(f"[bench] malloc: no trimming, mmap threshold 32 MB ({'ok' if ok else 'mallopt refused'})")


def pin_main_thread(mode: str) -> str:
    """--pin-cpu: keep the calling (main) thread on one CPU -- the one it runs on now ("current"),
    or the given number -- as a real-time caller pins its control thread; the runtime's own threads,
    created earlier, keep their affinity."""
    if mode in ("", "off"):
        return "off"
    try:
        if mode == "current":
            with open("/proc/thread-self/stat") as f:
                cpu = int(f.read().rsplit(")", 1)[1].split()[36])
        else:
            cpu = int(mode)
        os.sched_setaffinity(0, {cpu})
        return f"cpu {cpu}"
    except (OSError, ValueError, IndexError) as e:
        return f"failed ({e})"


def parse_cpulist(text: str) -> set:
    """A Linux CPU list ("0-63,128-191") as a set of CPU numbers."""
    cpus = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def numa_local(device: int) -> str:
    """--numa-local: every thread of the process onto the CPUs of the GPU's NUMA node (those the
    process may use), as a deployment places a GPU's host process -- the pinned staging, the
    caller's arrays and the queue writes then stay on the GPU's side of the socket link."""
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return "off (no PCI bus id)"
        bus = buf.value.decode().lower()
        node = int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
        if node < 0:
            return "off (no NUMA node)"
        cpus = parse_cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read()) & os.sched_getaffinity(0)
        if not cpus:
            return "off (no allowed CPU on the node)"
        for t in os.listdir("/proc/self/task"):
            try:
                os.sched_setaffinity(int(t), cpus)
            except OSError:
                pass
        return f"node {node} ({len(cpus)} CPUs)"
    except (OSError, ValueError) as e:
        return f"off ({e})"


def lock_code() -> str:
    """mlock the executable mappings of the HIP / HSA runtimes and the product library (diagnostic
    of the one-rep stall: if host memory pressure drops their code pages from this process, the
    next call through a cold path re-faults them).  Only when RLIMIT_MEMLOCK covers them."""
    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    libc.mlock.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    names = ("libamdhip64", "libhsa-runtime64", "librsvio", "libhsakmt", "libc.so", "libstdc++")
    spans = []
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and parts[1].startswith("r") and any(n in parts[5] for n in names):
                a, b = (int(x, 16) for x in parts[0].split("-"))
                spans.append((a, b - a))
    total = sum(n for _, n in spans)
    soft, _ = resource.getrlimit(resource.RLIMIT_MEMLOCK)
    if soft != resource.RLIM_INFINITY and total > soft:
        return f"skipped: {total >> 20} MB of mappings > RLIMIT_MEMLOCK {soft >> 10} KB"
    bad = sum(1 for a, n in spans if libc.mlock(a, n) != 0)
    return f"locked {len(spans) - bad}/{len(spans)} mappings, {total >> 20} MB"


def setup_dist(same_device: bool = False):
    """One process per GPU over RCCL.  `same_device` is a rehearsal mode for a one-GPU box: every
    rank on cuda:0 with a gloo control group (RCCL refuses two ranks on one device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if same_device else int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        # the communication libraries' own connection messages (gloo prints "[Gloo] Rank r is
        # connected to ..." on stdout) go to stderr: rank 0's stdout carries the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if same_device:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist.barrier()  # (the mesh is connected here at the latest)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def reduce_scalar(x: float, world: int, op: str = "max") -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN)
    return float(t.item())


def max_over_ranks(x: float, world: int) -> float:
    return reduce_scalar(x, world, "max")


def cu_partition(device: int, frac: float, layout: str):
    """CU sets for the tracker and the BA streams (hipExtStreamCreateWithCUMask): the tracker's
    900 latency-bound one-wave workgroups otherwise share SIMDs with the BA's serial kernels.
    layout "block": mask bits 0..k-1 -- bit i is CU i // 8 of XCD i % 8, so the tracker gets k / 8 CUs
    on every XCD; "stride": every (n / k)-th bit, which for k = n / 4 names XCDs 0 and 4 only -- a
    mask that leaves an XCD empty is not honoured, and both streams then run on every CU
    (tools/xcd_map.hip)."""
    import ctypes as C

    from rsvio import _lib
    n = C.c_int(0)
    _lib.check(_lib.load().rsvio_device_info(device, None, 0, C.byref(n)))
    n = n.value
    k = max(1, min(n - 1, int(round(frac * n))))
    if layout == "block":
        trk = list(range(k))
    else:
        step = n / k
        trk = sorted({int(i * step) for i in range(k)})
    ba = [c for c in range(n) if c not in set(trk)]
    return trk, ba


class TrackerWorkload:
    """Config 2 on device: per-frame pyramids (left, right) + 3 track_points batches."""

    upload_kernel = False  # bench.py --upload: the pcie image upload by rsvio_upload_async

    def __init__(self, device: int, stream_ptr=None):
        import ctypes as C

        import torch

        from rsvio import _lib
        from rsvio import synthetic as S
        self.C, self.torch, self.L = C, torch, _lib
        lib = _lib.load()
        t0 = time.time()
        frames = list(S.stereo_sequence(N_FRAMES, W, H))
        log(f"[bench] rendered {N_FRAMES} stereo frames in {time.time() - t0:.1f}s")
        # true feature positions per frame: cam0 = FAST corners of frame 0 moved by the synthetic motion
        aff0 = S.track_features(frames[0][0], NFEAT)
        ang = math.radians(0.2)
        c = np.array([W / 2.0, H / 2.0])
        affs0, affs1 = [], []
        for t in range(N_FRAMES):
            R = np.array([[math.cos(ang * t), -math.sin(ang * t)], [math.sin(ang * t), math.cos(ang * t)]])
            a = aff0.copy()
            a[:, 4:6] = ((R @ (aff0[:, 4:6] - c).T).T + c + np.array([1.7, -0.9]) * t).astype(np.float32)
            affs0.append(a)
            affs1.append(S.stereo_shift(a))
        dev = torch.device("cuda", device)
        self.imgs = torch.from_numpy(np.stack([np.stack(f) for f in frames])).to(dev)       # F x 2 x H x W
        self.aff0 = torch.from_numpy(np.stack(affs0)).to(dev)                               # F x N x 6
        self.aff1 = torch.from_numpy(np.stack(affs1)).to(dev)
        self.pyr_bytes = int(lib.rsvio_pyramid_bytes(W, H, LEVELS))
        self.pyr = torch.empty((2, 2, self.pyr_bytes), dtype=torch.uint8, device=dev)      # slot x cam
        self.out = torch.empty((3, NFEAT, 6), dtype=torch.float32, device=dev)
        self.valid = torch.empty((3, NFEAT), dtype=torch.uint8, device=dev)
        ctx = C.c_void_p()
        _lib.check(lib.rsvio_track_ctx_create(W, H, LEVELS, device, C.byref(ctx)))
        self.ctx = ctx
        self.lib = lib
        self.seq = [0, 1, 2, 3, 2, 1]
        self.k = 0
        self.slot = 0
        self.stream = (torch.cuda.ExternalStream(stream_ptr, device=dev) if stream_ptr
                       else torch.cuda.current_stream(dev))
        self.ev = []
        # per-frame enqueue as captured graphs (_capture; --tracker-graphs), built on first use
        self.graphs = False
        self._graphs, self._graph_objs = {}, []
        # prime: pyramids of the first frame
        self._pyramids(self.seq[0], self.slot)

    def _pyramids(self, t, slot, src=None):
        s = self.stream.cuda_stream
        src = self.imgs[t] if src is None else src
        self.L.check(self.lib.rsvio_build_pyramids_d(self.ctx, src.data_ptr(), 2, self.pyr[slot].data_ptr(), s))

    def enable_pcie(self):
        """Host-side buffers of the PCIe-inclusive step (GPU frames/sec includes the
        image upload and the feature-list download): the frames in pinned host memory, a device
        staging pair, pinned outputs."""
        torch = self.torch
        self.h_imgs = self.imgs.cpu().pin_memory()
        self.d_stage = torch.empty_like(self.imgs[0])
        self.h_out = torch.empty(self.out.shape, dtype=self.out.dtype).pin_memory()
        self.h_valid = torch.empty(self.valid.shape, dtype=self.valid.dtype).pin_memory()

    def _plan(self, phase: int, pcie: bool):
        """The C arguments of one step, built once per (phase of the frame sequence, pcie): the
        sequence has period len(seq) (even, so the pyramid slot parity repeats with it).  A Rust
        caller passes these as they are; building ctypes structures and taking tensor pointers
        costs tens of microseconds of Python per step, which is harness overhead, not tracker
        work.  The copies go through the HIP runtime the library is bound to (hipMemcpyAsync on
        the tracker stream)."""
        key = (phase, pcie)
        plan = self._plans.get(key) if hasattr(self, "_plans") else None
        if plan is not None:
            return plan
        if not hasattr(self, "_plans"):
            self._plans = {}
            C = self.C
            self._memcpy = self.lib.hipMemcpyAsync
            self._memcpy.restype = C.c_int
            self._memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
            # the frame's completion: an event after the D2H copies, polled (hipEventQuery) --
            # a blocking stream sync may put the thread to sleep and add its wake-up latency
            self._ev_record = self.lib.hipEventRecord
            self._ev_record.restype = C.c_int
            self._ev_record.argtypes = [C.c_void_p, C.c_void_p]
            self._ev_query = self.lib.hipEventQuery
            self._ev_query.restype = C.c_int
            self._ev_query.argtypes = [C.c_void_p]
            ev = C.c_void_p()
            create = self.lib.hipEventCreateWithFlags
            create.restype = C.c_int
            create.argtypes = [C.c_void_p, C.c_uint]
            self.L.check(create(C.byref(ev), 2))  # hipEventDisableTiming
            self._done_ev = ev.value
        t = self.seq[phase]
        t2 = self.seq[(phase + 1) % len(self.seq)]
        prev, cur = phase % 2, 1 - phase % 2
        b = (self.L.TrackBatch * 3)()
        spec = [(self.pyr[prev, 0], self.pyr[cur, 0], self.aff0[t]),
                (self.pyr[prev, 1], self.pyr[cur, 1], self.aff1[t]),
                (self.pyr[cur, 0], self.pyr[cur, 1], self.aff0[t2])]
        for i, (p0, p1, a) in enumerate(spec):
            b[i] = self.L.TrackBatch(p0.data_ptr(), p1.data_ptr(), a.data_ptr(), self.out[i].data_ptr(),
                                     self.valid[i].data_ptr(), NFEAT)
        src = self.d_stage if pcie else self.imgs[t2]
        plan = {"batches": b, "src": src.data_ptr(), "dst": self.pyr[cur].data_ptr(),
                "h_img": self.h_imgs[t2].data_ptr() if pcie else None, "img_bytes": src.numel()}
        self._plans[key] = plan
        return plan

    def upload(self):
        """The next frame's two images up from pinned host memory (the first part of a pcie step:
        issued as soon as the frame is there; step(..., uploaded=True) enqueues the rest)."""
        plan = self._plan(self.k % len(self.seq), True)
        if self.upload_kernel:  # a kernel on the tracker stream reads the pinned images (no copy engine)
            self.L.check(self.lib.rsvio_upload_async(plan["src"], plan["h_img"], plan["img_bytes"],
                                                     self.stream.cuda_stream))
        else:
            self.L.check(self._memcpy(plan["src"], plan["h_img"], plan["img_bytes"], 1, self.stream.cuda_stream))

    def step(self, timed: bool, pcie: bool = False, wait: bool = True, uploaded: bool = False):
        """Frame t -> t': 2 pyramids of t', then cam0 / cam1 temporal + stereo batches.  pcie:
        the two images are uploaded from pinned host memory first (unless upload() already did)
        and the three tracked feature lists (+ valid flags) are downloaded before the step
        returns (wait=False: they are enqueued and sync() completes the frame)."""
        C = self.C
        phase = self.k % len(self.seq)
        assert self.slot == phase % 2
        plan = self._plan(phase, pcie)
        s = self.stream.cuda_stream
        timed = timed and self.k % 4 == 0  # LK launch time sampled on every 4th frame (event overhead)
        if self.graphs and not timed:
            # the frame's copies and kernels as one captured graph per (phase, pcie, uploaded):
            # one hipGraphLaunch instead of up to five enqueue calls (the same work, the same order)
            key = (phase, pcie, uploaded)
            ex = self._graphs.get(key)
            if ex is None:
                ex = self._capture(plan, pcie, uploaded, s)
                self._graphs[key] = ex
            self.L.check(self._graph_launch(ex, s))
            if pcie:
                self.L.check(self._ev_record(self._done_ev, s))
                self._pending = True
                if wait:
                    self.sync()
            self.slot = 1 - self.slot
            self.k += 1
            return
        if pcie and not uploaded:
            self.L.check(self._memcpy(plan["src"], plan["h_img"], plan["img_bytes"], 1, s))
        self.L.check(self.lib.rsvio_build_pyramids_d(self.ctx, plan["src"], 2, plan["dst"], s))
        if timed:
            e0 = self.torch.cuda.Event(enable_timing=True)
            e1 = self.torch.cuda.Event(enable_timing=True)
            e0.record(self.stream)
        self.L.check(self.lib.rsvio_track_points_d(self.ctx, plan["batches"], 3, MAX_IT, C.c_float(THRESH), s))
        if timed:
            e1.record(self.stream)
            self.ev.append((e0, e1))
        if pcie:
            self.L.check(self._memcpy(self.h_out.data_ptr(), self.out.data_ptr(), self.out.numel() * 4, 2, s))
            self.L.check(self._memcpy(self.h_valid.data_ptr(), self.valid.data_ptr(), self.valid.numel(), 2, s))
            self.L.check(self._ev_record(self._done_ev, s))
            self._pending = True
            if wait:
                self.sync()
        self.slot = 1 - self.slot
        self.k += 1

    def precapture(self, pcie: bool, uploaded: bool):
        """Capture every phase's frame graph up front (a caller captures at start-up, not in its
        first timed frames): hipGraphInstantiate costs ~1 ms of host time, which a first use
        inside a timed repetition would add to that repetition alone."""
        if not self.graphs:
            return
        s = self.stream.cuda_stream
        for phase in range(len(self.seq)):
            key = (phase, pcie, uploaded)
            if key not in self._graphs:
                self._graphs[key] = self._capture(self._plan(phase, pcie), pcie, uploaded, s)

    def _capture(self, plan, pcie, uploaded, s):
        """Capture the frame's enqueue sequence on the tracker stream (relaxed mode) into an
        instantiated graph executable."""
        C = self.C
        lib = self.lib
        if not hasattr(self, "_graph_launch"):
            for name, res, args in (("hipStreamBeginCapture", C.c_int, [C.c_void_p, C.c_int]),
                                    ("hipStreamEndCapture", C.c_int, [C.c_void_p, C.c_void_p]),
                                    ("hipGraphInstantiate", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                                      C.c_size_t]),
                                    ("hipGraphLaunch", C.c_int, [C.c_void_p, C.c_void_p])):
                f = getattr(lib, name)
                f.restype, f.argtypes = res, args
            self._graph_launch = lib.hipGraphLaunch
        self.L.check(lib.hipStreamBeginCapture(s, 2))  # hipStreamCaptureModeRelaxed
        if pcie and not uploaded:
            self.L.check(self._memcpy(plan["src"], plan["h_img"], plan["img_bytes"], 1, s))
        self.L.check(lib.rsvio_build_pyramids_d(self.ctx, plan["src"], 2, plan["dst"], s))
        self.L.check(lib.rsvio_track_points_d(self.ctx, plan["batches"], 3, MAX_IT, C.c_float(THRESH), s))
        if pcie:
            self.L.check(self._memcpy(self.h_out.data_ptr(), self.out.data_ptr(), self.out.numel() * 4, 2, s))
            self.L.check(self._memcpy(self.h_valid.data_ptr(), self.valid.data_ptr(), self.valid.numel(), 2, s))
        g = C.c_void_p()
        self.L.check(lib.hipStreamEndCapture(s, C.byref(g)))
        ex = C.c_void_p()
        self.L.check(lib.hipGraphInstantiate(C.byref(ex), g, None, None, 0))
        self._graph_objs.append(g)
        return ex

    def sync(self):
        if getattr(self, "_pending", False):
            while True:
                rc = self._ev_query(self._done_ev)
                if rc != 600:  # hipErrorNotReady
                    if rc:
                        raise RuntimeError(f"hipEventQuery failed with HIP error {rc}")
                    break
            self._pending = False
        else:
            self.stream.synchronize()

    def close(self):
        # pinned blocks carry events recorded on the tracker stream: drain and release them while
        # that stream exists (it is destroyed with the CU-mask streams after this)
        self.torch.cuda.synchronize()
        for k in ("h_imgs", "h_out", "h_valid", "d_stage"):
            self.__dict__.pop(k, None)
        host_empty = getattr(self.torch._C, "_host_emptyCache", None)
        if host_empty:
            host_empty()
        if getattr(self, "_done_ev", None):
            destroy = self.lib.hipEventDestroy
            destroy.restype = self.C.c_int
            destroy.argtypes = [self.C.c_void_p]
            destroy(self._done_ev)
            self._done_ev = None
        if self._graphs or self._graph_objs:
            C = self.C
            for name in ("hipGraphExecDestroy", "hipGraphDestroy"):
                f = getattr(self.lib, name)
                f.restype, f.argtypes = C.c_int, [C.c_void_p]
            for ex in self._graphs.values():
                self.lib.hipGraphExecDestroy(ex)
            for g in self._graph_objs:
                self.lib.hipGraphDestroy(g)
            self._graphs, self._graph_objs = {}, []
        if self.ctx:
            self.lib.rsvio_track_ctx_destroy(self.ctx)
            self.ctx = None

    def lk_ms(self):
        if not self.ev:
            return float("nan")
        return float(np.mean([a.elapsed_time(b) for a, b in self.ev]))


def measure_tracker_batched_row(trk: "TrackerWorkload", device: int, n_streams: int = 64, steps: int = 30,
                                warmup: int = 3):
    """SURVEY 8d "batched mode": config 2's per-frame tracker work for B independent stereo
    streams per step -- one packed pyramid launch (2B images) and ONE rsvio_track_points_table_d
    launch of 3B batches (cam0 temporal, cam1 temporal, stereo; 300 features each, fwd+bwd) --
    so the 900 chains of one frame become 900 B and the roofline fraction is meaningful.  Stream s
    sees the config-2 sequence translated by (s % 8, s // 8) px (distinct images and pyramids per
    stream; its features translated with it).  value = B frames per step / step time (HIP events on
    the launch stream)."""
    import ctypes as C

    import torch

    from rsvio import _lib
    dev = torch.device("cuda", device)
    B, F = n_streams, trk.imgs.shape[0]
    lib, L = trk.lib, _lib
    imgs = torch.empty((F, B, 2, H, W), dtype=torch.uint8, device=dev)
    aff0 = torch.empty((F, B, NFEAT, 6), dtype=torch.float32, device=dev)
    aff1 = torch.empty_like(aff0)
    for s_ in range(B):
        dx, dy = s_ % 8, s_ // 8
        imgs[:, s_] = torch.roll(trk.imgs, shifts=(dy, dx), dims=(-2, -1))
        aff0[:, s_] = trk.aff0
        aff1[:, s_] = trk.aff1
        aff0[:, s_, :, 4] += dx
        aff0[:, s_, :, 5] += dy
        aff1[:, s_, :, 4] += dx
        aff1[:, s_, :, 5] += dy
    pyr = torch.empty((2, B, 2, trk.pyr_bytes), dtype=torch.uint8, device=dev)
    out = torch.empty((3 * B, NFEAT, 6), dtype=torch.float32, device=dev)
    valid = torch.empty((3 * B, NFEAT), dtype=torch.uint8, device=dev)
    seq = trk.seq
    tables = []
    for k in range(len(seq)):        # the (frame, slot) pattern repeats every len(seq) steps
        t, t2 = seq[k % len(seq)], seq[(k + 1) % len(seq)]
        prev, cur = k % 2, 1 - k % 2
        tb = (L.TrackBatch * (3 * B))()
        for s_ in range(B):
            spec = [(pyr[prev, s_, 0], pyr[cur, s_, 0], aff0[t, s_]), (pyr[prev, s_, 1], pyr[cur, s_, 1], aff1[t, s_]),
                    (pyr[cur, s_, 0], pyr[cur, s_, 1], aff0[t2, s_])]
            for j, (p0, p1, a) in enumerate(spec):
                i = 3 * s_ + j
                tb[i] = L.TrackBatch(p0.data_ptr(), p1.data_ptr(), a.data_ptr(), out[i].data_ptr(),
                                     valid[i].data_ptr(), NFEAT)
        raw = np.frombuffer(C.string_at(C.addressof(tb), C.sizeof(tb)), np.uint8).copy()
        tables.append((t2, cur, torch.from_numpy(raw).to(dev)))
    start = torch.arange(0, 3 * B * NFEAT + 1, NFEAT, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    L.check(lib.rsvio_build_pyramids_d(trk.ctx, imgs[seq[0]].data_ptr(), 2 * B, pyr[0].data_ptr(), sp))

    def step(k, evs=None):
        t2, cur, tab = tables[k % len(tables)]
        if evs:
            evs[0].record(stream)
        L.check(lib.rsvio_build_pyramids_d(trk.ctx, imgs[t2].data_ptr(), 2 * B, pyr[cur].data_ptr(), sp))
        if evs:
            evs[1].record(stream)
        L.check(lib.rsvio_track_points_table_d(trk.ctx, tab.data_ptr(), start.data_ptr(), 3 * B, 3 * B * NFEAT,
                                               MAX_IT, C.c_float(THRESH), sp))
        if evs:
            evs[2].record(stream)

    for k in range(warmup):
        step(k)
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for k in range(steps):
        step(warmup + k, evs[k])
    torch.cuda.synchronize()
    pyr_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    lk_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    total_ms = evs[0][0].elapsed_time(evs[-1][2]) / steps
    calls = 3 * NFEAT * 2
    lk_bytes = B * lk_bytes_per_launch(calls)
    frame_bytes = B * tracker_bytes_per_frame(calls)
    ach = lk_bytes / (lk_ms * 1e-3) / 1e9
    row = {"workload": f"config 2 tracker work of {B} independent 752x480 stereo streams per step: one packed "
                       f"pyramid launch ({2 * B} images, L=3) + one table-mode LK launch ({3 * B} batches x 300 "
                       f"features, fwd+bwd = {B * calls} track_one_point calls)",
           "value": round(B / (total_ms * 1e-3), 1), "unit": "frames/s", "streams": B,
           "ms_per_step": round(total_ms, 4), "pyramid_ms": round(pyr_ms, 4), "lk_ms": round(lk_ms, 4),
           "valid_fraction": round(float(valid.float().mean()), 4),
           "roofline": {"kernel": "lk_track_kernel", "bound": "hbm", "achieved": round(ach, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 6),
                        "algorithmic_bytes_per_launch": lk_bytes, "launch_ms": round(lk_ms, 4),
                        "whole_step_achieved_gbs": round(frame_bytes / (total_ms * 1e-3) / 1e9, 2),
                        "note": "still chain-latency-bound: 6 waves per SIMD resident, each a serial "
                                "Gauss-Newton chain; batching raises occupancy, not per-chain latency"}}
    del imgs, pyr, out, valid, tables
    return row


class BAWorkload:
    def __init__(self, device: int, world: int, rank: int, stream_ptr=None, collective: str = "auto",
                 rccl_ok: bool = True):
        from rsvio import synthetic as S
        from rsvio.ba import BundleAdjuster
        t0 = time.time()
        full = S.ba_problem(n_lm=2000 * world)
        self.full = full
        self.prob = full.shard(rank, world) if world > 1 else full
        log(f"[bench] rank {rank}: BA shard {self.prob.n_lm} landmarks / {self.prob.n_obs} obs "
            f"(global {full.n_lm}/{full.n_obs}) built in {time.time() - t0:.1f}s")
        self.ba = BundleAdjuster(max_keyframes=full.n_kf, max_landmarks=self.prob.n_lm,
                                 max_observations=self.prob.n_obs, device=device)
        self.collective = "none"
        if world > 1:
            self.collective = self._attach(world, rank, collective, rccl_ok)
            log(f"[bench] rank {rank}: BA exchange = {self.collective}")
        self.p2p_us = None
        if self.collective == "p2p":
            # the exchange's own latency (max over ranks): the 4 trial scalars and a reduced
            # system of W=10 (1,600 doubles, 12.5 KB), 200 back-to-back exchanges each
            self.p2p_us = {f"{n}_doubles": round(reduce_scalar(self.ba.p2p_latency_us(200, n), world, "max"), 2)
                           for n in (4, 1600)}
            log(f"[bench] rank {rank}: P2P exchange latency {self.p2p_us} us")
        self.stream_ptr = stream_ptr
        if stream_ptr:
            self.ba.set_stream(stream_ptr)
        self.ba.set_problem_from(self.prob)
        self.iters = []
        self.solve_ms = []
        # the protocol step uploads a new window every frame (every frame a keyframe): two
        # pre-built config-3 windows of distinct seeds, alternating (same shapes, different data)
        alt = S.ba_problem(n_lm=2000 * world, seed=17, init_seed=23)
        self.windows = [self.prob, alt.shard(rank, world) if world > 1 else alt]
        self.k = 0
        self._pinned = []

    def pin_windows(self):
        """The windows' host arrays in page-locked memory (diagnostic, --pin-windows 1): the stall
        it was meant to remove turned out to be trimmed heap memory re-faulted inside one
        set_problem (--tame-malloc), not the caller's arrays (profiles/r06c_*, r06i_*)."""
        import dataclasses

        import torch
        out = []
        for w in self.windows:
            repl = {}
            for f in ("pose7", "kf_fixed", "p_W", "obs_lm", "obs_kf", "obs_cam", "obs_uv", "T_C_B2"):
                a = np.ascontiguousarray(getattr(w, f))
                t = torch.empty(a.shape, dtype=getattr(torch, str(a.dtype)), pin_memory=True)
                t.numpy()[...] = a
                self._pinned.append(t)
                repl[f] = t.numpy()
            out.append(dataclasses.replace(w, **repl))
        self.windows = out

    def next_window(self):
        """Upload the next keyframe window (rsvio_ba_set_problem through the handle's pinned
        staging); the solve's graph is re-captured by the following start()."""
        self.k += 1
        self.ba.set_problem_from(self.windows[self.k % len(self.windows)])

    def _attach(self, world, rank, collective, rccl_ok):
        """RCCL communicator first (the fallback), then the P2P one-shot all-reduce when every rank
        can map every peer's exchange buffer; all ranks agree on the outcome."""
        return self.ba.attach_sharded(world, rank, collective, rccl_ok, log=lambda m: log(f"[bench] {m}"))

    def start(self):
        self.ba.run_async()

    def finish(self, timed: bool):
        r = self.ba.wait()
        if r.status <= 0:
            raise RuntimeError(f"BA solve failed with status {r.status}")
        if timed:
            self.iters.append(r.iterations)
            self.solve_ms.append(r.solve_ms)
        return r


class NativeProtocol:
    """bench.py's protocol step driven from C++ (lib/librsvio_host.so, rs-vio_amd/driver/
    protocol.cpp): the same calls on the same buffers as protocol_step's split order -- image
    upload, rsvio_ba_set_problem of the next window, rsvio_ba_run_async, the frame's captured
    tracker graph (every 4th frame enqueued directly with LK timing events, as trk.step does),
    the frame's event polled, rsvio_ba_wait, rsvio_ba_get_state -- without Python between them,
    as the reference's Rust caller runs them.  The library's entry points are passed as the
    function pointers of the library rsvio already loaded."""

    class Window(ctypes.Structure):
        _fields_ = [("n_kf", ctypes.c_int32), ("pose7", ctypes.c_void_p), ("kf_fixed", ctypes.c_void_p),
                    ("n_lm", ctypes.c_int32), ("p_W", ctypes.c_void_p), ("n_obs", ctypes.c_int32),
                    ("obs_lm", ctypes.c_void_p), ("obs_kf", ctypes.c_void_p), ("obs_cam", ctypes.c_void_p),
                    ("obs_uv", ctypes.c_void_p), ("T_C_B2", ctypes.c_void_p)]

    class Frame(ctypes.Structure):
        _fields_ = [("upload_dst", ctypes.c_void_p), ("upload_src", ctypes.c_void_p), ("upload_bytes", ctypes.c_size_t),
                    ("graph_exec", ctypes.c_void_p), ("pyr_dst", ctypes.c_void_p), ("batches", ctypes.c_void_p)]

    class Api(ctypes.Structure):
        _fields_ = [(n, ctypes.c_void_p) for n in ("set_problem", "run_async", "wait", "get_state",
                                                   "build_pyramids_d", "track_points_d", "upload")]

    class Setup(ctypes.Structure):
        _fields_ = [("api", ctypes.c_void_p), ("ba", ctypes.c_void_p), ("cfg", ctypes.c_void_p),
                    ("trk_stream", ctypes.c_void_p), ("done_event", ctypes.c_void_p),
                    ("n_windows", ctypes.c_int32), ("windows", ctypes.c_void_p),
                    ("n_phases", ctypes.c_int32), ("frames", ctypes.c_void_p),
                    ("pose_out", ctypes.c_void_p), ("pw_out", ctypes.c_void_p),
                    ("first_phase", ctypes.c_int32), ("first_window", ctypes.c_int32),
                    ("track_ctx", ctypes.c_void_p), ("max_iterations", ctypes.c_int32), ("thresh", ctypes.c_float),
                    ("d_out", ctypes.c_void_p), ("h_out", ctypes.c_void_p), ("out_bytes", ctypes.c_size_t),
                    ("d_valid", ctypes.c_void_p), ("h_valid", ctypes.c_void_p), ("valid_bytes", ctypes.c_size_t),
                    ("first_step", ctypes.c_int32), ("lk_events", ctypes.c_void_p), ("n_lk_events", ctypes.c_int32),
                    ("order", ctypes.c_int32), ("phase_us", ctypes.c_void_p), ("ba_stream", ctypes.c_void_p),
                    ("tl_events", ctypes.c_void_p), ("n_tl", ctypes.c_int32)]

    def __init__(self, trk: "TrackerWorkload", ba: "BAWorkload", state_out, max_steps: int, order: int = 0):
        from rsvio import _lib
        from rsvio.ba import BundleAdjuster, _DEFAULT_CFG
        lib = _lib.load()
        path = _lib.LIB_PATH.parent / "librsvio_host.so"
        self.drv = ctypes.CDLL(str(path))
        self.drv.rsvio_protocol_run.restype = ctypes.c_int
        self.drv.rsvio_protocol_run.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p]
        fp = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
        self.api = self.Api(fp(lib.rsvio_ba_set_problem), fp(lib.rsvio_ba_run_async), fp(lib.rsvio_ba_wait),
                            fp(lib.rsvio_ba_get_state), fp(lib.rsvio_build_pyramids_d), fp(lib.rsvio_track_points_d),
                            fp(lib.rsvio_upload_async) if trk.upload_kernel else None)
        self.keep = []
        wins = (self.Window * len(ba.windows))()
        for i, w in enumerate(ba.windows):
            keep, args = BundleAdjuster._marshal(*(getattr(w, f) for f in BundleAdjuster._FIELDS))
            self.keep.append(keep)
            wins[i] = self.Window(*args)
        nph = len(trk.seq)
        frames = (self.Frame * nph)()
        for ph in range(nph):
            plan = trk._plan(ph, True)
            ex = trk._graphs.get((ph, True, True))
            if ex is None:
                ex = trk._capture(plan, True, True, trk.stream.cuda_stream)
                trk._graphs[(ph, True, True)] = ex
            frames[ph] = self.Frame(plan["src"], plan["h_img"], plan["img_bytes"], ex, plan["dst"],
                                    ctypes.addressof(plan["batches"]))
        self.wins, self.frames = wins, frames
        n_ev = max_steps // 4 + 2
        create = lib.hipEventCreateWithFlags
        create.restype, create.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint]
        self._elapsed = lib.hipEventElapsedTime
        self._elapsed.restype = ctypes.c_int
        self._elapsed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        self._destroy = lib.hipEventDestroy
        self._destroy.restype, self._destroy.argtypes = ctypes.c_int, [ctypes.c_void_p]
        self.ev_ptrs = (ctypes.c_void_p * (2 * n_ev))()
        for i in range(2 * n_ev):
            e = ctypes.c_void_p()
            _lib.check(create(ctypes.byref(e), 0))  # hipEventDefault: timing
            self.ev_ptrs[i] = e.value
        self.cfg = _DEFAULT_CFG
        self.trk, self.ba, self.state_out = trk, ba, state_out
        self.n_ev = n_ev
        self.order = order
        self.phases = None  # a list: each run appends its steps' 7 host phase times (us)
        self.timeline = None  # a list: each run appends its steps' (window laid out, solve end) (us)
        self.ba_stream = ba.stream_ptr
        self._create = create

    def run(self, steps: int):
        """`steps` protocol steps from the workloads' current phase and window; advances them."""
        trk, ba = self.trk, self.ba
        setup = self.Setup(ctypes.addressof(self.api), ba.ba._h.value, ctypes.addressof(self.cfg),
                           trk.stream.cuda_stream, trk._done_ev, len(ba.windows), ctypes.addressof(self.wins),
                           len(trk.seq), ctypes.addressof(self.frames),
                           self.state_out[0].ctypes.data, self.state_out[1].ctypes.data,
                           trk.k % len(trk.seq), (ba.k + 1) % len(ba.windows),
                           trk.ctx.value, MAX_IT, THRESH,
                           trk.out.data_ptr(), trk.h_out.data_ptr(), trk.out.numel() * 4,
                           trk.valid.data_ptr(), trk.h_valid.data_ptr(), trk.valid.numel(),
                           trk.k, ctypes.addressof(self.ev_ptrs), self.n_ev, self.order, None)
        ph = (ctypes.c_double * (7 * steps))() if self.phases is not None else None
        setup.phase_us = ctypes.addressof(ph) if ph is not None else None
        tl = None
        if self.timeline is not None and self.ba_stream:
            from rsvio import _lib
            tl = (ctypes.c_void_p * (3 * steps))()
            for i in range(3 * steps):
                e = ctypes.c_void_p()
                _lib.check(self._create(ctypes.byref(e), 0))  # timing events
                tl[i] = e.value
            setup.ba_stream = self.ba_stream
            setup.tl_events = ctypes.addressof(tl)
            setup.n_tl = steps
        iters = (ctypes.c_int32 * steps)()
        sms = (ctypes.c_double * steps)()
        sec, npair = ctypes.c_double(0.0), ctypes.c_int32(0)
        rc = self.drv.rsvio_protocol_run(ctypes.addressof(setup), steps, iters, sms, ctypes.byref(sec),
                                         ctypes.byref(npair))
        if rc:
            raise RuntimeError(f"rsvio_protocol_run failed: {rc}")
        if ph is not None:
            self.phases += [list(ph[7 * i:7 * i + 7]) for i in range(steps)]
        if tl is not None:
            for i in range(steps):
                w, e = ctypes.c_float(0.0), ctypes.c_float(0.0)
                self._elapsed(ctypes.byref(w), tl[3 * i], tl[3 * i + 1])
                self._elapsed(ctypes.byref(e), tl[3 * i], tl[3 * i + 2])
                self.timeline.append((1e3 * w.value, 1e3 * e.value))
            for i in range(3 * steps):
                self._destroy(tl[i])
        trk.k += steps
        trk.slot ^= steps & 1
        ba.k += steps
        lk = []
        for i in range(npair.value):
            ms = ctypes.c_float(0.0)
            _ = self._elapsed(ctypes.byref(ms), self.ev_ptrs[2 * i], self.ev_ptrs[2 * i + 1])
            lk.append(ms.value)
        return list(iters), list(sms), lk

    def close(self):
        for e in self.ev_ptrs:
            if e:
                self._destroy(e)
        self.ev_ptrs = (ctypes.c_void_p * 0)()


def host_cores() -> int:
    """Host threads this process may use: the box's CPU share (OMP_NUM_THREADS, set per GPU on
    the pool) or the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(frames_budget_s: float, threads: int = 1):
    """The oracle (C++ restatement of the reference) on the host: same tracker frame + BA solve.
    threads > 1 mirrors the reference's rayon parallelism: per-level pyramids
    (feature_tracker.rs:213) and per-feature track_points (:260) over `threads` threads; the BA
    solve runs the threaded Schur variant (landmark ranges in parallel) on the all-cores leg."""
    from oracle import oracle as O
    from rsvio import synthetic as S
    frames = list(S.stereo_sequence(2, W, H))
    aff0 = S.track_features(frames[0][0], NFEAT)
    aff1 = S.stereo_shift(aff0)
    affn = aff0.copy()
    affn[:, 4:6] += np.array([1.7, -0.9], np.float32)
    prob = S.ba_problem()
    pyr_prev = [O.build_pyramid(frames[0][c], LEVELS) for c in range(2)]
    n, t_track, t_ba, t_pyr = 0, 0.0, 0.0, 0.0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < frames_budget_s or n < 2:
        t0 = time.perf_counter()
        pc = [O.build_pyramid(frames[1][c], LEVELS, threads) for c in range(2)]
        t_pyr += time.perf_counter() - t0
        O.track_points(pyr_prev[0], pc[0], W, H, LEVELS, aff0, MAX_IT, THRESH, threads)
        O.track_points(pyr_prev[1], pc[1], W, H, LEVELS, aff1, MAX_IT, THRESH, threads)
        O.track_points(pc[0], pc[1], W, H, LEVELS, affn, MAX_IT, THRESH, threads)
        t1 = time.perf_counter()
        O.set_ba_threads(threads)   # the threaded Schur variant on the all-cores leg
        try:
            _, _, r = O.ba_solve(prob)
        finally:
            O.set_ba_threads(1)
        t2 = time.perf_counter()
        t_track += t1 - t0
        t_ba += t2 - t1
        n += 1
    fps = n / (t_track + t_ba)
    return {"value": round(fps, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames of config 2 (2 pyramids + 3x300 track_points) each followed by one config-3 "
                      f"BA solve ({r.iterations} LM iterations), oracle/ C++ restatement, "
                      + ("1 thread" if threads == 1 else
                         f"{threads} threads of one persistent pool (oracle/pool.hpp: pyramid levels and grains of "
                         "2 feature tracks claimed dynamically, as rayon's par_iter; threaded Schur BA)"),
            "tracker_ms_per_frame": round(1e3 * t_track / n, 3),
            "stage_ms_per_frame": {"pyramids": round(1e3 * t_pyr / n, 3),
                                   "track_points_900": round(1e3 * (t_track - t_pyr) / n, 3),
                                   "ba_solve": round(1e3 * t_ba / n, 3)},
            "ba_ms_per_solve": round(1e3 * t_ba / n, 3),
            "ba_ms_per_iter": round(1e3 * t_ba / n / max(r.iterations, 1), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5, help="timed repetitions of --steps steps; value = median")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-rows", action="store_true", help="skip the unprojection / track_motion row measurements")
    ap.add_argument("--pipeline-frames", type=int, default=500,
                    help="config-4 Estimator row: rendered frames (0: skip)")
    ap.add_argument("--batch-streams", type=int, default=64,
                    help="batched tracker row: independent stereo streams per launch (0: skip)")
    ap.add_argument("--cu-split", type=float, default=0.25,
                    help="fraction of CUs given to the tracker stream (0: no CU partition); 0.25 measured "
                         "best (round 2 sweep: K4c's 360 two-wave-per-SIMD workgroups fit the BA's 192 CUs "
                         "in one round)")
    ap.add_argument("--cu-layout", default="block", choices=["stride", "block"])
    ap.add_argument("--order", default="split", choices=["frame-first", "ba-first", "split", "window-first"],
                    help="protocol step: the frame's image upload first, then the keyframe window's upload + "
                         "solve start, then the frame's kernels and downloads (split, the default: 4.16-4.35k vs "
                         "3.98-4.08k frames/s for ba-first and 3.74-3.96k for frame-first on one box, "
                         "profiles/r05h_order_ab.txt -- the image and window uploads share the copy engine, and "
                         "the image then lands first without holding the window back behind the frame's kernels "
                         "enqueue); both paths run concurrently either way (the tracker does not depend on the solve); "
                         "window-first: the window's upload, then the image upload, then the solve start and the "
                         "frame (the window's copy ahead of the image's)")
    ap.add_argument("--upload", default="kernel", choices=["kernel", "sdma"],
                    help="the protocol step's image upload: kernel (default, rsvio_upload_async: a kernel on the "
                         "tracker stream reads the pinned images, so the pyramids follow it without a copy-engine "
                         "hand-off) or sdma (hipMemcpyAsync)")
    ap.add_argument("--tracker-graphs", type=int, default=1,
                    help="1: the frame's copies + pyramid + LK launches replayed as one captured HIP graph per "
                         "frame phase (one hipGraphLaunch instead of up to five enqueue calls); 0: direct enqueue")
    ap.add_argument("--driver", default="native", choices=["native", "python"],
                    help="who runs the protocol step's calls: native (default) -- lib/librsvio_host.so, the same "
                         "C ABI calls from C++ as the reference's Rust caller makes them; python -- this loop "
                         "(ctypes; ~1-5 us of interpreter per call; --trace-steps uses it)")
    ap.add_argument("--numa-local", type=int, default=1,
                    help="1 (default): every thread onto the CPUs of the GPU's NUMA node, as a deployment places "
                         "a GPU's host process (4,799-4,854 frames/s vs 4,121-4,821 unplaced, 3 alternating pairs, "
                         "profiles/r06z3_numa_local_ab.txt); 0: wherever the scheduler puts it")
    ap.add_argument("--pin-cpu", default="off",
                    help="pin the main thread: off (default), current (the CPU it runs on), or a CPU number")
    ap.add_argument("--lock-code", type=int, default=0,
                    help="1: mlock the runtimes' and the library's mapped pages (stall diagnostic)")
    ap.add_argument("--tame-malloc", type=int, default=1,
                    help="1 (default): glibc malloc without trimming and with a fixed mmap threshold (mallopt, as "
                         "a real-time caller configures its process): otherwise about every other run one "
                         "set_problem re-faults ~14-16 MB of trimmed heap (3.5-4.1k minor faults, 6-10 ms) -- "
                         "the one slow repetition of rounds 4-5 (profiles/r06i_malloc_ab.txt); 0: glibc defaults")
    ap.add_argument("--pin-windows", type=int, default=0,
                    help="1: the keyframe windows' host arrays in page-locked memory (diagnostic of the stall; it "
                         "did not remove it); 0 (default): ordinary numpy arrays, as a caller's Vecs")
    ap.add_argument("--precapture-graphs", type=int, default=1,
                    help="1: capture the tracker's per-phase frame graphs before the timed region (0: on first "
                         "use, as rounds 4-5 did -- one repetition then pays the instantiations)")
    ap.add_argument("--collective", default="auto", choices=["auto", "rccl", "p2p"],
                    help="BA exchange for N>1: P2P one-shot all-reduce (auto: if every rank attaches) or RCCL")
    ap.add_argument("--trace-steps", default="",
                    help="write every timed protocol step's host phase times (upload, set_problem, solve start, "
                         "frame enqueue, frame wait, solve wait, state read-back) to this JSON file")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a one-GPU box: all ranks on cuda:0, gloo control group, P2P exchange")
    args = ap.parse_args()
    if args.same_device:
        args.collective = "p2p"
        # (ranks sharing one GPU never take the iterations whose next decision waits in K4c,
        # RSVIO_P2P_FOLD=2 and 4: attach_p2p sees the shared device and lowers them to 1 and 3,
        # DESIGN.md section 8)

    if args.tame_malloc:
        tame_malloc()
    world, rank, local = setup_dist(args.same_device)
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    import torch

    import rsvio
    arch = rsvio.require_device(local)
    if args.lock_code:
        log(f"[bench] lock-code: {lock_code()}")
    pin_state = pin_main_thread(args.pin_cpu)
    if args.numa_local:
        pin_state += "; process: " + numa_local(local)
    log(f"[bench] main thread: {pin_state}")
    log(f"[bench] rank {rank}/{world} on cuda:{local} ({arch})")
    streams = []
    if args.cu_split > 0:
        from rsvio._lib import CuStream
        cu_trk, cu_ba = cu_partition(local, args.cu_split, args.cu_layout)
        streams = [CuStream(local, cu_trk), CuStream(local, cu_ba)]
        log(f"[bench] CU partition ({args.cu_layout}): tracker {len(cu_trk)} CUs, BA {len(cu_ba)} CUs")
    trk = TrackerWorkload(local, streams[0].ptr if streams else None)
    trk.graphs = bool(args.tracker_graphs)
    trk.upload_kernel = args.upload == "kernel"
    ba = BAWorkload(local, world, rank, streams[1].ptr if streams else None, args.collective,
                    rccl_ok=not args.same_device)

    barrier(world)

    def resident_step(timed):
        """Device-resident step: the window already on the device is solved again (its captured
        graph replayed); the frame's tracking is enqueued while the solve runs."""
        ba.start()
        trk.step(timed)
        ba.finish(timed)

    def protocol_step(timed):
        """BASELINE.md protocol step, pipelined as the config-4 Estimator is (a keyframe's solve
        overlaps the next frame's tracking): the frame's 2 images go up from pinned host memory
        and the tracker is enqueued (pyramids, LK, the three feature lists + valid flags back to
        pinned host memory); the host uploads a new keyframe window (rsvio_ba_set_problem:
        validation, per-landmark masks, wave packing, pinned staging, H2D copies, slot headers and
        pair lists built on the device) and starts its solve (the descriptor-mode graph: one
        launch); then the frame's features, the solve and its optimised state (48.6 KB, published
        to pinned host memory with the solve's last decision) are waited for.  Default order
        (split): the frame's image upload first (as soon as the frame is there), then the window
        and the solve, then the frame's kernels and downloads; --order ba-first: the window and
        the solve before the whole frame; --order frame-first the other way round."""
        tr = trace is not None and timed
        if tr:
            f0 = (resource.getrusage(resource.RUSAGE_SELF).ru_minflt, resource.getrusage(1).ru_minflt)
            m = [time.perf_counter()]
        if args.order == "frame-first":
            trk.step(timed, pcie=True, wait=False)
        elif args.order == "split":
            trk.upload()
        if tr:
            m.append(time.perf_counter())
        ba.next_window()
        if args.order == "window-first":
            trk.upload()
        if tr:
            m.append(time.perf_counter())
        ba.start()
        if tr:
            m.append(time.perf_counter())
        if args.order != "frame-first":
            trk.step(timed, pcie=True, wait=False, uploaded=args.order in ("split", "window-first"))
        if tr:
            m.append(time.perf_counter())
        trk.sync()
        if tr:
            m.append(time.perf_counter())
        ba.finish(timed)
        if tr:
            m.append(time.perf_counter())
        ba.ba.state(state_out)
        if tr:
            m.append(time.perf_counter())
            trace.append(m)
            trace_flt.append((resource.getrusage(resource.RUSAGE_SELF).ru_minflt - f0[0],
                              resource.getrusage(1).ru_minflt - f0[1]))  # 1: RUSAGE_THREAD

    trace = [] if args.trace_steps else None
    trace_flt = []
    # the optimised state comes back into reused host arrays, as a Rust caller would keep them
    state_out = (np.empty((ba.prob.n_kf, 7)), np.empty((ba.prob.n_lm, 3)))

    def timed_reps(step, reps):
        import gc
        out = []
        for _ in range(reps):
            barrier(world)
            gc.disable()  # no collector pauses inside a timed repetition (the harness is Python)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(True)
            barrier(world)
            out.append(max_over_ranks(time.perf_counter() - t0, world))
            gc.enable()
        return out

    if args.precapture_graphs:
        trk.precapture(False, False)
    for _ in range(args.warmup):
        resident_step(False)
    el_res = timed_reps(resident_step, args.reps)
    lk_ms_resident = trk.lk_ms()
    trk.ev.clear()
    ba_iters_res, ba_solve_ms_res = float(np.mean(ba.iters)), float(np.mean(ba.solve_ms))
    ba.iters.clear()
    ba.solve_ms.clear()
    trk.enable_pcie()
    if args.pin_windows:
        ba.pin_windows()
    if args.precapture_graphs:
        trk.precapture(True, args.order in ("split", "window-first"))
    native = None
    if args.driver == "native" and args.order in ("split", "window-first"):
        native = NativeProtocol(trk, ba, state_out, max(args.steps, args.warmup, 2),
                                order=1 if args.order == "window-first" else 0)
        native.run(max(args.warmup, 2))
        if trace is not None:
            native.phases = []
            native.timeline = []
    else:
        for _ in range(max(args.warmup, 2)):
            protocol_step(False)
    minflt0 = _minor_faults()
    if native is None:
        el_pro = timed_reps(protocol_step, args.reps)
        lk_pro = None
    else:
        import gc
        el_pro, lk_pro = [], []
        for _ in range(args.reps):
            barrier(world)
            gc.disable()
            t0 = time.perf_counter()
            its, sms, lk = native.run(args.steps)
            barrier(world)
            el_pro.append(max_over_ranks(time.perf_counter() - t0, world))
            gc.enable()
            ba.iters += its
            ba.solve_ms += sms
            lk_pro += lk
    minflt = _minor_faults() - minflt0
    if native is not None and native.phases is not None:  # the native driver's own host phase times
        names = ["upload", "set_problem", "start", "frame_enqueue", "frame_wait", "solve_wait", "state"]
        ph = np.array(native.phases)
        with open(args.trace_steps, "w") as f:
            tlv = np.array(native.timeline) if native.timeline else None
            json.dump({"driver": "native", "phases": names, "steps_per_rep": args.steps,
                       "timeline_median_us": ({"window_laid_out": round(float(np.median(tlv[:, 0])), 1),
                                               "solve_end": round(float(np.median(tlv[:, 1])), 1)}
                                              if tlv is not None else None),
                       "median_us": [round(float(x), 2) for x in np.median(ph, axis=0)],
                       "p90_us": [round(float(x), 2) for x in np.percentile(ph, 90, axis=0)],
                       "us": [[round(float(x), 1) for x in r] for r in ph]}, f)
    elif trace is not None:
        names = ["upload", "set_problem", "start", "frame_enqueue", "frame_wait", "solve_wait", "state"]
        with open(args.trace_steps, "w") as f:
            json.dump({"phases": names, "steps_per_rep": args.steps,
                       "us": [[round(1e6 * (b - a), 1) for a, b in zip(m, m[1:])] for m in trace],
                       "t0_us": [round(1e6 * (m[0] - trace[0][0]), 1) for m in trace],
                       "minor_faults_process_thread": trace_flt,
                       "thp": _read_text("/sys/kernel/mm/transparent_hugepage/enabled"),
                       "thp_defrag": _read_text("/sys/kernel/mm/transparent_hugepage/defrag")}, f)
    elapsed = float(np.median(el_pro))
    elapsed_res = float(np.median(el_res))

    frames = world * args.steps
    value = frames / elapsed
    value_res = frames / elapsed_res
    lk_ms = trk.lk_ms() if lk_pro is None else (float(np.mean(lk_pro)) if lk_pro else float("nan"))
    ba_iters = float(np.mean(ba.iters))
    ba_solve_ms = float(np.mean(ba.solve_ms))
    ba_ms_iter = ba_solve_ms / ba_iters
    ba_ms_iter_res = ba_solve_ms_res / ba_iters_res
    calls = 3 * NFEAT * 2
    lk_bytes = lk_bytes_per_launch(calls)
    achieved = lk_bytes / (lk_ms * 1e-3) / 1e9
    prob = ba.prob
    flops = ba_flops_per_iter(prob.n_obs, prob.n_lm, 6, int((prob.kf_fixed == 0).sum()))
    traffic, traffic_src = pmc_traffic("lk_track_kernel")
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "reps": args.reps,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "value_note": "BASELINE.md protocol, median of reps: per frame the 2 x 361 KB images up from "
                      "pinned host memory (--upload kernel: rsvio_upload_async, a kernel reads them over "
                      "PCIe), pyramids + LK, 3 x 300 feature states + valid flags D2H; a NEW keyframe window "
                      "uploaded (rsvio_ba_set_problem: validation, masks, waves and tables into pinned "
                      "staging, ba_stage_in reading it over PCIe, the slot layout built on the device; two "
                      "windows alternate) and solved (the descriptor-mode graph), its state (48.6 KB) "
                      "published to pinned host memory by the final decision and read back",
        "main_thread": pin_state,
        "value_reps": [round(frames / e, 3) for e in el_pro],
        "driver": "native (lib/librsvio_host.so: the step's C ABI calls from C++)" if native is not None
                  else "python (ctypes)",
        "value_reps_min": round(frames / max(el_pro), 3),
        "protocol_minor_faults": minflt,
        "host_numa_balancing": _read_text("/proc/sys/kernel/numa_balancing"),
        "value_reps_max": round(frames / min(el_pro), 3),
        "value_resident": round(value_res, 3),
        "ms_per_step_resident": round(1e3 * elapsed_res / args.steps, 4),
        "value_resident_note": "inputs resident in HBM, the same window re-solved each step (its graph "
                               "replayed), nothing crosses PCIe but the LM status reads",
        "value_resident_reps": [round(frames / e, 3) for e in el_res],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (tracker) / f64 (BA)",
        "data": "synthetic (procedural EuRoC-shaped stereo texture + synthetic 10-KF landmark window; "
                "no dataset offline)",
        "config": {"workload": "config 2 + config 3 per frame: 752x480 stereo, 300 feats, 52-pt pattern, L=3, "
                               "track_points x3 fwd+bwd; then one BA solve 10 KF x 2000 landmarks/GPU "
                               "(24,000 obs/GPU), Schur LM <= 20 it; every frame a keyframe",
                   "image": "752x480", "features": NFEAT, "levels": LEVELS, "keyframes": 10,
                   "landmarks_per_gpu": prob.n_lm, "observations_per_gpu": prob.n_obs,
                   "parallelism": f"tracker replicas x{world}, BA landmark-sharded over {world} GPU(s)"
                                   + (f" ({ba.collective} all-reduce)" if world > 1 else ""),
                   "order": args.order,
                   "cu_partition": (f"{args.cu_layout} {args.cu_split:g} of CUs to the tracker stream"
                                    if args.cu_split > 0 else "none")},
        "ba_ms_per_iter": round(ba_ms_iter, 4),
        "ba_iterations": ba_iters,
        "ba_ms_per_solve": round(ba_solve_ms, 4),
        "ba_ms_per_iter_resident": round(ba_ms_iter_res, 4),
        "ba_ms_per_solve_resident": round(ba_solve_ms_res, 4),
        "tracker_lk_ms_per_frame_resident": round(lk_ms_resident, 4),
        "tracker_lk_ms_per_frame": round(lk_ms, 4),
        "roofline": {"kernel": "lk_track_kernel", "bound": "hbm", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": None if traffic is None else round(traffic),
                     "traffic_detail": traffic_src,
                     "algorithmic_bytes_per_launch": lk_bytes, "launch_ms": round(lk_ms, 4),
                     "note": "the step's longest single kernel; latency-bound: 900 one-wave workgroups "
                             "(fwd+bwd chains) on the tracker's CUs",
                     "step_bound": {"by": "BA LM chain (K4c -> K5 -> K6 per iteration, one stream)",
                                    "bound": "fp64", "unit": "TFLOP/s", "flop_per_iter": flops,
                                    "achieved": round(flops / (ba_ms_iter * 1e-3) / 1e12, 4),
                                    "peak": FP64_PEAK_TFLOPS,
                                    "frac": round(flops / (ba_ms_iter * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 6),
                                    "ba_ms_per_solve": round(ba_solve_ms, 4),
                                    "share_of_step": round(ba_solve_ms / (1e3 * elapsed / args.steps), 3)}},
        "ba_roofline": {"bound": "fp64", "flop_per_iter": flops,
                        "achieved_tflops": round(flops / (ba_ms_iter * 1e-3) / 1e12, 4),
                        "peak_tflops": FP64_PEAK_TFLOPS},
    }
    if world > 1:
        out["ba_exchange"] = {"collective": ba.collective, "p2p_latency_us": ba.p2p_us,
                              "fold": os.environ.get("RSVIO_P2P_FOLD", "3") if ba.collective == "p2p" else None,
                              "flag_in_word_system": os.environ.get("RSVIO_P2P_LL", "0") == "1"
                              if ba.collective == "p2p" else None}
    if rank == 0 and not args.no_rows:
        out["rows"] = measure_rows(local, cpu=(world == 1 and not args.no_cpu))
    if rank == 0 and not args.no_rows and args.batch_streams > 0:
        out.setdefault("rows", {})["tracker_batched"] = measure_tracker_batched_row(trk, local, args.batch_streams)
    if rank == 0 and not args.no_rows and args.pipeline_frames > 0:
        out.setdefault("rows", {})["pipeline_config4"] = measure_pipeline_row(
            local, cpu=(world == 1 and not args.no_cpu), n_frames=args.pipeline_frames,
            native=args.driver == "native")
    if rank == 0 and world == 1 and not args.no_cpu:
        # two legs -- all host cores (the reported baseline, rayon's parallelism) and
        # one thread -- each a bounded sample of the same per-frame work
        cores = host_cores()
        cb = cpu_baseline(args.cpu_seconds, cores)
        cb1 = cpu_baseline(args.cpu_seconds / 2, 1)
        cb["single_thread"] = {k: cb1[k] for k in ("value", "cores", "sample", "tracker_ms_per_frame",
                                                   "stage_ms_per_frame", "ba_ms_per_solve", "ba_ms_per_iter")}
        cb["stage_speedup_all_cores_vs_1"] = {k: round(cb1["stage_ms_per_frame"][k] / max(v, 1e-9), 2)
                                              for k, v in cb["stage_ms_per_frame"].items()}
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu_baseline"] = round(value / cb["value"], 2)
        out["speedup_vs_cpu_single_thread"] = round(value / cb1["value"], 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    # release device objects before interpreter teardown (the CU-mask streams last)
    torch.cuda.synchronize()
    if native is not None:
        native.close()
    ba.ba.close()
    trk.close()
    for st in streams:
        st.close()


if __name__ == "__main__":
    main()
