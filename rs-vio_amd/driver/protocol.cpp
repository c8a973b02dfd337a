// protocol.cpp -- the BASELINE.md protocol step driven the way a compiled caller drives it.
//
// The reference's host code is Rust (src/estimator/estimator.rs:101-262 calls the tracker, then
// SlidingWindow::optimize, sliding_window.rs:159-381, once per keyframe): a handful of FFI calls
// per frame, each ~0.1 us.  bench.py's Python loop pays ~1-5 us of interpreter and ctypes time
// per call, and six of those calls sit on the step's critical path (the BA path: image upload,
// set_problem, the solve's start before it; the wait and the state read-back after it).  This
// driver runs the same calls, in the same order, on the same buffers, from C++ -- nothing in it
// is device work of its own, and nothing of the step is skipped:
//
//   per step k (split order, bench.py protocol_step; order 1 swaps steps 1 and 2):
//     1. the next frame's two images up from pinned host memory (rsvio_upload_async: a kernel on the
//        tracker stream reads them over PCIe; or hipMemcpyAsync when the api's upload is null);
//     2. a NEW keyframe window: rsvio_ba_set_problem (two pre-built windows alternate);
//     3. rsvio_ba_run_async (the solve's captured graph);
//     4. the frame's captured tracker graph (pyramids, LK, the feature lists down) + an event --
//        on every 4th step enqueued directly instead, with HIP events around the LK launch (the
//        kernel's time for bench.py's roofline, as its Python loop samples it);
//     5. wait for the frame (the event polled), then rsvio_ba_wait (status must be > 0);
//     6. rsvio_ba_get_state into the caller's reused arrays.
//
// It reaches the product library only through its C ABI (include/rsvio_gpu.h), as a Rust caller
// would: the four entry points come in as function pointers of the library the caller already
// loaded (bench.py passes those of rsvio._lib, so an A/B build loaded through RSVIO_LIB is the one
// driven).  Not part of the product ABI: lib/librsvio_host.so is loaded by bench.py.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstddef>
#include <cstdint>

#include "rsvio_gpu.h"

extern "C" {

struct rsvio_protocol_window {  // rsvio_ba_set_problem's arguments for one keyframe window
    int32_t n_kf;
    const double* pose7;
    const uint8_t* kf_fixed;
    int32_t n_lm;
    const double* p_W;
    int32_t n_obs;
    const int32_t* obs_lm;
    const int32_t* obs_kf;
    const uint8_t* obs_cam;
    const double* obs_uv;
    const double* T_C_B2;
};

struct rsvio_protocol_frame {  // one phase of the frame sequence
    void* upload_dst;          // device staging of the two images
    const void* upload_src;    // pinned host images
    size_t upload_bytes;
    void* graph_exec;          // hipGraphExec_t: pyramids + track_points + the lists' D2H copies
    uint8_t* pyr_dst;          // the direct path's pyramids (the new frame's slot, both cameras)
    const rsvio_track_batch* batches;  // its 3 track_points batches
};

struct rsvio_protocol_api {  // the product library's entry points (its C ABI)
    decltype(&rsvio_ba_set_problem) set_problem;
    decltype(&rsvio_ba_run_async) run_async;
    decltype(&rsvio_ba_wait) wait;
    decltype(&rsvio_ba_get_state) get_state;
    decltype(&rsvio_build_pyramids_d) build_pyramids_d;
    decltype(&rsvio_track_points_d) track_points_d;
    decltype(&rsvio_upload_async) upload;  // null: the image upload by hipMemcpyAsync (copy engine)
};

struct rsvio_protocol {
    const rsvio_protocol_api* api;
    rsvio_ba* ba;
    const rsvio_lm_cfg* cfg;
    void* trk_stream;          // hipStream_t of the tracker
    void* done_event;          // hipEvent_t recorded after the frame's graph
    int32_t n_windows;
    const rsvio_protocol_window* windows;
    int32_t n_phases;
    const rsvio_protocol_frame* frames;
    double* pose_out;          // rsvio_ba_get_state's destination (reused every step)
    double* pw_out;
    int32_t first_phase;       // the phase of step 0
    int32_t first_window;      // the window of step 0
    // the direct path of every 4th step (step k with (first_step + k) % 4 == 0)
    rsvio_track_ctx* track_ctx;
    int32_t max_iterations;
    float thresh;
    void* d_out;               // the 3 x n feature states and valid flags, and their pinned copies
    void* h_out;
    size_t out_bytes;
    void* d_valid;
    void* h_valid;
    size_t valid_bytes;
    int32_t first_step;
    void** lk_events;          // 2 hipEvent_t (timing) per sampled step, in order; null: no sampling
    int32_t n_lk_events;       // pairs available
    int32_t order;             // 0: split (image upload, window, solve start, frame); 1: window first
                               // (window, image upload, solve start, frame: the window's copy ahead of
                               // the image's on the copy engine)
    double* phase_us;          // null, or 7 host phase times per step (us): image upload, set_problem,
                               // run_async, frame enqueue, frame wait, rsvio_ba_wait, get_state (order
                               // 1 counts the image upload after set_problem into its first entry)
    void* ba_stream;           // hipStream_t of the BA handle (for the timeline events)
    void** tl_events;          // null, or 3 timing hipEvent_t per step for the first n_tl steps: the
    int32_t n_tl;              // step's start (tracker stream, before the image upload), the window
                               // laid out (BA stream, after set_problem), the solve's end (BA stream,
                               // after run_async: the stream's position past the solve's graph)
};

// Runs `steps` protocol steps; per step the solve's LM iterations and device solve time into
// iters_out / solve_ms_out (may be null); the wall time of the whole loop into seconds_out and the
// LK timing event pairs used into lk_pairs_out.  Returns 0, a negative RSVIO_ERR_* from a library
// call, or -100 - status for a failed solve.
int rsvio_protocol_run(const rsvio_protocol* P, int32_t steps, int32_t* iters_out, double* solve_ms_out,
                       double* seconds_out, int32_t* lk_pairs_out) {
    if (!P || !P->api || !P->ba || !P->cfg || !P->windows || !P->frames || P->n_windows < 1 || P->n_phases < 1 ||
        steps < 0)
        return RSVIO_ERR_INVALID_ARG;
    const rsvio_protocol_api& A = *P->api;
    const hipStream_t ts = static_cast<hipStream_t>(P->trk_stream);
    const hipEvent_t done = static_cast<hipEvent_t>(P->done_event);
    int32_t n_lk = 0;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    clk::time_point tp[8];
    double* ph = P->phase_us;
    auto mark = [&](int i) {
        if (ph) tp[i] = clk::now();
    };
    const bool tl = P->tl_events && P->ba_stream;
    const hipStream_t bs = static_cast<hipStream_t>(P->ba_stream);
    for (int32_t k = 0; k < steps; ++k) {
        mark(0);
        const bool tk = tl && k < P->n_tl;
        if (tk && hipEventRecord(static_cast<hipEvent_t>(P->tl_events[3 * k]), ts) != hipSuccess) return RSVIO_ERR_HIP;
        const rsvio_protocol_frame& f = P->frames[(P->first_phase + k) % P->n_phases];
        const rsvio_protocol_window& w = P->windows[(P->first_window + k) % P->n_windows];
        auto up = [&]() -> int {
            if (A.upload) return A.upload(f.upload_dst, f.upload_src, f.upload_bytes, P->trk_stream);
            return hipMemcpyAsync(f.upload_dst, f.upload_src, f.upload_bytes, hipMemcpyHostToDevice, ts) == hipSuccess
                       ? 0
                       : RSVIO_ERR_HIP;
        };
        if (P->order == 0 && up()) return RSVIO_ERR_HIP;
        mark(1);
        int rc = A.set_problem(P->ba, w.n_kf, w.pose7, w.kf_fixed, w.n_lm, w.p_W, w.n_obs, w.obs_lm, w.obs_kf,
                               w.obs_cam, w.obs_uv, w.T_C_B2);
        if (rc) return rc;
        if (tk && hipEventRecord(static_cast<hipEvent_t>(P->tl_events[3 * k + 1]), bs) != hipSuccess)
            return RSVIO_ERR_HIP;
        mark(2);
        if (P->order == 1) {
            if (up()) return RSVIO_ERR_HIP;
            if (ph) {  // (the image upload's time goes to the first phase)
                const auto t = clk::now();
                tp[1] += t - tp[2];
                tp[2] = t;
            }
        }
        if ((rc = A.run_async(P->ba, P->cfg))) return rc;
        if (tk && hipEventRecord(static_cast<hipEvent_t>(P->tl_events[3 * k + 2]), bs) != hipSuccess)
            return RSVIO_ERR_HIP;
        mark(3);
        if (P->lk_events && (P->first_step + k) % 4 == 0 && n_lk < P->n_lk_events) {
            // the frame enqueued directly, the LK launch between two timing events
            if ((rc = A.build_pyramids_d(P->track_ctx, static_cast<const uint8_t*>(f.upload_dst), 2, f.pyr_dst, ts)))
                return rc;
            if (hipEventRecord(static_cast<hipEvent_t>(P->lk_events[2 * n_lk]), ts) != hipSuccess) return RSVIO_ERR_HIP;
            if ((rc = A.track_points_d(P->track_ctx, f.batches, 3, P->max_iterations, P->thresh, ts))) return rc;
            if (hipEventRecord(static_cast<hipEvent_t>(P->lk_events[2 * n_lk + 1]), ts) != hipSuccess)
                return RSVIO_ERR_HIP;
            ++n_lk;
            if (hipMemcpyAsync(P->h_out, P->d_out, P->out_bytes, hipMemcpyDeviceToHost, ts) != hipSuccess ||
                hipMemcpyAsync(P->h_valid, P->d_valid, P->valid_bytes, hipMemcpyDeviceToHost, ts) != hipSuccess)
                return RSVIO_ERR_HIP;
        } else if (hipGraphLaunch(static_cast<hipGraphExec_t>(f.graph_exec), ts) != hipSuccess) {
            return RSVIO_ERR_HIP;
        }
        if (hipEventRecord(done, ts) != hipSuccess) return RSVIO_ERR_HIP;
        mark(4);
        hipError_t q;
        while ((q = hipEventQuery(done)) == hipErrorNotReady) {
        }
        if (q != hipSuccess) return RSVIO_ERR_HIP;
        mark(5);
        rsvio_ba_result r{};
        if ((rc = A.wait(P->ba, &r))) return rc;
        mark(6);
        if (r.status <= 0) return -100 - r.status;
        if (iters_out) iters_out[k] = r.iterations;
        if (solve_ms_out) solve_ms_out[k] = r.solve_ms;
        if ((rc = A.get_state(P->ba, P->pose_out, P->pw_out))) return rc;
        if (ph) {
            tp[7] = clk::now();
            for (int i = 0; i < 7; ++i)
                ph[7 * k + i] = std::chrono::duration<double, std::micro>(tp[i + 1] - tp[i]).count();
        }
    }
    if (seconds_out)
        *seconds_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (lk_pairs_out) *lk_pairs_out = n_lk;
    return 0;
}

// Layout check for the caller's mirror of these structs (bench.py's ctypes; a CPU test compares):
// the sizes of the four structs, then the offsets of their last fields.
int rsvio_protocol_layout(int64_t* out, int32_t n) {
    const int64_t v[] = {(int64_t)sizeof(rsvio_protocol_window), (int64_t)sizeof(rsvio_protocol_frame),
                         (int64_t)sizeof(rsvio_protocol_api), (int64_t)sizeof(rsvio_protocol),
                         (int64_t)offsetof(rsvio_protocol_window, T_C_B2), (int64_t)offsetof(rsvio_protocol_frame, batches),
                         (int64_t)offsetof(rsvio_protocol, first_step), (int64_t)offsetof(rsvio_protocol, lk_events),
                         (int64_t)offsetof(rsvio_protocol, n_lk_events), (int64_t)offsetof(rsvio_protocol, thresh),
                         (int64_t)offsetof(rsvio_protocol, valid_bytes), (int64_t)offsetof(rsvio_protocol, order), (int64_t)offsetof(rsvio_protocol, phase_us),
                         (int64_t)offsetof(rsvio_protocol, n_tl)};
    const int32_t m = (int32_t)(sizeof v / sizeof v[0]);
    for (int32_t i = 0; i < n && i < m; ++i) out[i] = v[i];
    return m;
}

}  // extern "C"
