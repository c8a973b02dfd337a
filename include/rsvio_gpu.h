/*
 * rsvio_gpu.h -- C ABI of the MI355X (gfx950) implementation of RS-VIO's two hot paths.
 *
 * The reference (EthanD11/RS-VIO) is a pure-Rust crate with no FFI layer; its drop-in
 * boundary is the Rust API the estimator calls.  Every entry point below names the
 * reference item it replaces (file:line under the reference root).  INTEGRATION.md
 * shows the `extern "C"` block and safe wrapper a Rust maintainer binds to it.
 *
 * Conventions
 *  - Every function returns int: RSVIO_OK (0) or a negative RSVIO_ERR_* code;
 *    rsvio_last_error() returns a thread-local message.  Nothing aborts or unwinds.
 *  - Per-feature failure is valid = 0 (the reference's Option::None / false).
 *  - Host buffers are borrowed for the duration of the call only.  Device memory is
 *    owned by the handle and released by *_destroy.
 *  - A handle is single-threaded (mirrors `&mut self`); distinct handles may run
 *    concurrently on distinct HIP streams.
 *  - Affine2<f32> state is float[6] = {m11, m12, m21, m22, m13, m23}.
 *  - Pyramids are packed: level i is (w >> i) x (h >> i) u8, levels back to back.
 *  - SE3 poses are 7-vectors {tx, ty, tz, qw, qx, qy, qz} of T_B_W
 *    (src/estimator/sliding_window.rs:222-224).
 */
#ifndef RSVIO_GPU_H
#define RSVIO_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    RSVIO_OK = 0,
    RSVIO_ERR_INVALID_ARG = -1,
    RSVIO_ERR_HIP = -2,
    RSVIO_ERR_NOMEM = -3,
    RSVIO_ERR_CAPACITY = -4,
    RSVIO_ERR_NO_DEVICE = -5,
    RSVIO_ERR_INTERNAL = -6,
    RSVIO_ERR_RCCL = -7
};

/* Thread-local message for the last failing call on this thread. */
const char* rsvio_last_error(void);
/* Library / device identification; returns RSVIO_ERR_NO_DEVICE if no gfx950 is visible. */
int rsvio_device_info(int device, char* name_out, size_t cap, int* n_cus);

/* HIP stream (hipStream_t) for the device-pointer entry points and rsvio_ba_set_stream.
 * cu_mask (mask_words x 32 bits, bit i = CU i; NULL = all CUs) restricts the stream's kernels
 * to a CU subset, so the tracker and the BA of one process can run side by side on disjoint
 * CUs (hipExtStreamCreateWithCUMask).  No reference counterpart (the reference is CPU-only). */
int rsvio_stream_create(int32_t device, const uint32_t* cu_mask, uint32_t mask_words, void** out);
int rsvio_stream_destroy(void* stream);
/* Host-to-device copy of page-locked host memory (hipHostMalloc / hipHostRegister) by a kernel on
 * `stream` instead of a copy engine: the next kernel on the stream starts without the copy-engine ->
 * compute-queue hand-off (how bench.py's protocol step uploads the frame's images).  A pageable or
 * non-16-byte-aligned source or destination takes hipMemcpyAsync.  As with hipMemcpyAsync, the source
 * must stay valid and unchanged until the stream has passed the copy.  No reference counterpart. */
int rsvio_upload_async(void* d_dst, const void* h_src, size_t bytes, void* stream);

/* =============================== HP-T: patch tracker =============================== */

typedef struct {
    int32_t width, height;
    int32_t levels;                 /* StereoPatchTracker<LEVELS> (estimator.rs:27 uses 6) */
    int32_t grid_size;              /* config/euroc_vio.yaml:42 */
    int32_t max_iterations;         /* optical_flow_max_iterations (:44) */
    float convergence_threshold;    /* optical_flow_convergence_threshold (:45), f64->f32 (feature_tracker.rs:112) */
    int32_t device;
    int32_t max_features;           /* per-camera capacity of the track maps (0 -> 4096) */
} rsvio_tracker_params;

/* One tracked point: id + Affine2 state (pixel position = m13, m23). */
typedef struct {
    uint64_t id;
    float x, y;       /* m13, m23 */
    float r[4];       /* m11, m12, m21, m22 */
} rsvio_feature;

typedef struct rsvio_tracker rsvio_tracker;

/* StereoPatchTracker::<N>::new(grid_size, max_iters, thresh)  (src/feature_tracker/feature_tracker.rs:103-114) */
int rsvio_tracker_create(const rsvio_tracker_params* params, rsvio_tracker** out);
void rsvio_tracker_destroy(rsvio_tracker* t);

/* StereoPatchTracker::process_frame(&mut self, &GrayImage, &GrayImage, &mut Frame) (:116-187)
 * followed by get_track_points (:188-200).  Images are u8, row stride `stride` bytes.
 * Outputs are sorted by ascending id (canonical order; the reference iterates HashMaps).
 * New ids are assigned in detection scan order (image_utilities.rs:141-142).
 * RSVIO_ERR_CAPACITY (lists still consistent and returned) when the frame's new points exceed
 * max_features -- both cameras then admit the same leading new points and the rest are dropped
 * -- or when cap_l / cap_r truncated a list. */
int rsvio_tracker_process_frame(rsvio_tracker* t, const uint8_t* left, const uint8_t* right,
                                size_t stride, rsvio_feature* out_l, size_t cap_l, size_t* n_l,
                                rsvio_feature* out_r, size_t cap_r, size_t* n_r);
/* Same, with both images already in device memory (tightly packed w x h). */
int rsvio_tracker_process_frame_device(rsvio_tracker* t, const uint8_t* d_left,
                                       const uint8_t* d_right, rsvio_feature* out_l,
                                       size_t cap_l, size_t* n_l, rsvio_feature* out_r,
                                       size_t cap_r, size_t* n_r);
/* process_frame in two halves, for a caller that runs one frame ahead (the Estimator's look-ahead:
 * estimator.rs:190 passes the tracker only the two images, so frame t+1 can be tracked while frame
 * t's motion tracking and BA run).  submit enqueues the frame (pyramids, LK, FAST, packing and the
 * read-back of its lists) and returns at once; collect waits for it and fills the lists exactly as
 * process_frame does.  One frame in flight per handle: process_frame*, submit*, remove_ids and
 * set_cameras refuse (RSVIO_ERR_INVALID_ARG) while one is, collect refuses when none is.  Host
 * images (rsvio_tracker_submit) are borrowed until collect returns.  Consumers of the last
 * collected frame (rsvio_tracker_undistorted, rsvio_track_motion_tracker) keep reading THAT frame
 * after a later submit: frames alternate between two device output slots. */
int rsvio_tracker_submit(rsvio_tracker* t, const uint8_t* left, const uint8_t* right, size_t stride);
int rsvio_tracker_submit_device(rsvio_tracker* t, const uint8_t* d_left, const uint8_t* d_right);
int rsvio_tracker_collect(rsvio_tracker* t, rsvio_feature* out_l, size_t cap_l, size_t* n_l,
                          rsvio_feature* out_r, size_t cap_r, size_t* n_r);
/* StereoPatchTracker::remove_id (:201-206) */
int rsvio_tracker_remove_ids(rsvio_tracker* t, const uint64_t* ids, size_t n);
/* HIP stream the tracker enqueues on (hipStream_t) */
void* rsvio_tracker_stream(rsvio_tracker* t);

/* ---- parity-level entry points (host buffers in/out) ---- */

size_t rsvio_pyramid_bytes(int32_t w, int32_t h, int32_t levels);
/* build_image_pyramid (feature_tracker.rs:209-220): imageops::resize Triangle per level */
int rsvio_build_pyramid(const uint8_t* img, int32_t w, int32_t h, int32_t levels, uint8_t* out);
/* track_points (feature_tracker.rs:252-291): forward, backward and ||dt||^2 < 0.4 per feature.
 * aff_out receives the forward result for valid features (aff_in copied otherwise). */
int rsvio_track_points(const uint8_t* pyr0, const uint8_t* pyr1, int32_t w, int32_t h,
                       int32_t levels, const float* aff_in, int32_t n, int32_t max_iterations,
                       float thresh, float* aff_out, uint8_t* valid_out);
/* detect_key_points(img, grid, current, 1) (image_utilities.rs:108-175) with the existing
 * tracks' positions (rounded as feature_tracker.rs:232-233).  out_xy: u32 (x, y) pairs. */
int rsvio_detect_keypoints(const uint8_t* img, int32_t w, int32_t h, int32_t grid,
                           const float* existing_xy, int32_t n_existing, uint32_t* out_xy,
                           float* out_score, int32_t cap, int32_t* n_out);

/* ---- device-pointer entry points (enqueue on `stream`, no synchronisation) ---- */
typedef struct rsvio_track_ctx rsvio_track_ctx;
/* Holds the per-(w,h,levels) resampling tables on device. */
int rsvio_track_ctx_create(int32_t w, int32_t h, int32_t levels, int32_t device, rsvio_track_ctx** out);
void rsvio_track_ctx_destroy(rsvio_track_ctx* c);
/* n_img images (each w x h, packed) -> n_img pyramids (each rsvio_pyramid_bytes, packed) */
int rsvio_build_pyramids_d(rsvio_track_ctx* c, const uint8_t* d_imgs, int32_t n_img,
                           uint8_t* d_pyrs, void* stream);
/* Up to 4 independent track_points batches in one launch. */
typedef struct {
    const uint8_t* d_pyr0;
    const uint8_t* d_pyr1;
    const float* d_aff_in;
    float* d_aff_out;
    uint8_t* d_valid;
    int32_t n;
} rsvio_track_batch;
int rsvio_track_points_d(rsvio_track_ctx* c, const rsvio_track_batch* batches, int32_t n_batches,
                         int32_t max_iterations, float thresh, void* stream);
/* Batched serving mode: any number of independent track_points batches (e.g. 3 per stereo
 * stream for many streams) in one launch.  d_table: n_batches descriptors in DEVICE memory;
 * d_start: n_batches + 1 int32 prefix sums of their sizes in device memory (d_start[0] = 0);
 * total = d_start[n_batches], given on the host for the grid size.  Same per-feature results as
 * rsvio_track_points_d (feature_tracker.rs:252-291). */
int rsvio_track_points_table_d(rsvio_track_ctx* c, const rsvio_track_batch* d_table, const int32_t* d_start,
                               int32_t n_batches, int32_t total, int32_t max_iterations, float thresh,
                               void* stream);

/* ====== T-sec: the feature_tracker/ crate (FeatureTracker, bicubic LK + Shi-Tomasi) ====== */

/* FeatureTrackingConfig (feature_tracker/src/feature_tracker.rs:25-38; defaults
 * feature_tracker/config/config.yaml) + image size, matching cost, device and capacity. */
enum { RSVIO_FT_SSD = 0, RSVIO_FT_LSSD = 1 };   /* MatchingCost (patch.rs:6-9) */
typedef struct {
    int32_t width, height;
    int32_t nlevels;                  /* 5 */
    int32_t preprocessing_blur;       /* 1 */
    double ratio;                     /* 2.0 */
    float preprocessing_blur_sigma;   /* 2.0 */
    float detection_threshold;        /* 2.5 */
    uint32_t detection_min_dist;      /* 15 */
    float detection_blur;             /* 6.0 */
    int32_t optical_flow_max_iter;    /* 25 */
    float optical_flow_lm_lambda;     /* 0.1 */
    int32_t matching_cost;            /* RSVIO_FT_SSD: what process_frame uses (feature_tracker.rs:125) */
    int32_t device;
    int32_t max_features;             /* capacity of the frame's feature list (0 -> 8192) */
    int32_t reserved;
} rsvio_ft_config;                    /* 64 bytes */

/* Feature (feature_tracker.rs:41-48): id + central point */
typedef struct {
    uint64_t feature_id;
    float x, y;
} rsvio_ft_feature;                   /* 16 bytes */

typedef struct rsvio_ft rsvio_ft;

/* FeatureTracker::new(config, None) (feature_tracker.rs:59-69) */
int rsvio_ft_create(const rsvio_ft_config* cfg, rsvio_ft** out);
void rsvio_ft_destroy(rsvio_ft* t);
/* FeatureTracker::process_frame(&FloatGrayImage, Frame) (:77-185): img is f32 luma in [0, 1]
 * (to_luma32f), row stride in floats (0 = width).  out receives frame.features: the previous
 * frame's features that track (previous order, positions transform * centre), then the new
 * Shi-Tomasi corners in (y, x) order with consecutive ids.  RSVIO_ERR_CAPACITY when the list
 * exceeds max_features (the list is truncated). */
int rsvio_ft_process_frame(rsvio_ft* t, const float* img, size_t stride, rsvio_ft_feature* out, size_t cap,
                           size_t* n);
/* Same with the image already in device memory (tightly packed). */
int rsvio_ft_process_frame_device(rsvio_ft* t, const float* d_img, rsvio_ft_feature* out, size_t cap, size_t* n);
/* FeatureTracker::get_pyramid (:190-193): the last frame's packed pyramid (rsvio_ft_pyramid_floats) */
int rsvio_ft_get_pyramid(rsvio_ft* t, float* out, size_t cap_floats);
void* rsvio_ft_stream(rsvio_ft* t);

/* ---- parity-level entry points (host buffers in/out, current device) ---- */
/* packed size of build_image_pyramid's output: level l = round(w / ratio^l) x round(h / ratio^l) */
size_t rsvio_ft_pyramid_floats(int32_t w, int32_t h, int32_t nlevels, double ratio);
/* build_image_pyramid (image_operations.rs:47-78) */
int rsvio_ft_build_pyramid(const float* img, int32_t w, int32_t h, int32_t nlevels, double ratio, int32_t blur,
                           float sigma, float* out);
/* feature_tracking::track_points (feature_tracking.rs:16-61) on packed pyramids: per feature the
 * forward transform {cos, sin, tx, ty} (identity when lost) and the keep flag. */
int rsvio_ft_track_points(const float* pyr0, const float* pyr1, int32_t w, int32_t h, int32_t nlevels,
                          double ratio, const float* xy, int32_t n, int32_t max_iter, float lm_lambda,
                          int32_t matching_cost, float* iso_out, uint8_t* valid_out);
/* shi_tomasi_score (feature_detection.rs:82-164) */
int rsvio_ft_shi_tomasi_score(const float* img, int32_t w, int32_t h, float detection_blur, float* score);
/* feature_detection::add_points (feature_detection.rs:47-80) on the fine level with the tracked
 * features' centres: new corners (u32 x, y) in (y, x) order. */
int rsvio_ft_add_points(const float* fine, int32_t w, int32_t h, const float* tracked_xy, int32_t n_tracked,
                        float threshold, int32_t min_dist, float detection_blur, uint32_t* out_xy, int32_t cap,
                        int32_t* n_out);

/* ============ T11: the trackers' f32 sin/cos (glibc sinf/cosf restated, trig.hpp) ============ */

/* Rust's f32::sin/cos as se2_exp_matrix reaches them through nalgebra's Rotation2::new
 * (src/feature_tracker/image_utilities.rs:84,93-94) and the crate's exp_se2
 * (feature_tracker/src/feature_tracker/feature_tracking.rs:199-203): glibc sinf/cosf on x86-64
 * Linux.  Parity entry points for the device restatement the LK kernels use:
 * rsvio_sincosf evaluates it on n host values; rsvio_sincosf_digest evaluates it on the f32 bit
 * patterns [first, first + count) and returns one 64-bit digest per 2^chunk_log2 inputs (the sum
 * mod 2^64 of splitmix64(((sin bits << 32) | cos bits) + u * 0x9E3779B97F4A7C15) over inputs u,
 * NaNs as 0x7fc00000), so all 2^32 inputs can be compared with the host's libm.  first must be
 * chunk-aligned, first + count <= 2^32, 16 <= chunk_log2 <= 32. */
int rsvio_sincosf(const float* x, size_t n, float* sin_out, float* cos_out);
int rsvio_sincosf_digest(uint64_t first, uint64_t count, uint32_t chunk_log2, uint64_t* digests_out);

/* ================= T12: camera unprojection (Frame::add_*_feature) ================= */

/* Camera models of src/datasets/mod.rs:93-163 (camera-intrinsic-model 0.7.2):
 *   RSVIO_CAM_OPENCV5  OpenCVModel5, params {fx, fy, cx, cy, k1, k2, p1, p2, k3} (pinhole-radtan)
 *   RSVIO_CAM_EUCM     EUCM,         params {fx, fy, cx, cy, alpha, beta}
 * unproject_one's return convention is not verifiable offline, so it is
 * a parameter: RSVIO_UNPROJ_PLANE gives (x/z, y/z), RSVIO_UNPROJ_RAY the first two components
 * of the unit ray.  frame.rs:118-119,131-132 keep components [0..2] as f32. */
enum { RSVIO_CAM_OPENCV5 = 0, RSVIO_CAM_EUCM = 1 };
enum { RSVIO_UNPROJ_PLANE = 0, RSVIO_UNPROJ_RAY = 1 };

typedef struct {
    int32_t model;           /* RSVIO_CAM_* */
    int32_t convention;      /* RSVIO_UNPROJ_* */
    int32_t max_iterations;  /* radtan Newton cap; <= 0 means 20 */
    int32_t reserved;
    double params[9];
} rsvio_camera;              /* 88 bytes */

/* Batched unproject_one (frame.rs:107-134): pixels (n x 2 f32, cast to f64 as frame.rs:118)
 * -> undistorted (n x 2 f32).  Failure of one point (EUCM outside its valid cone, radtan
 * Newton not converging, non-finite) gives NaN coordinates and valid_out = 0 (valid_out may be
 * NULL).  Host buffers, current device. */
int rsvio_unproject(const rsvio_camera* cam, const float* px, size_t n, float* out_xy,
                    uint8_t* valid_out);
/* Same on device pointers, enqueued on `stream` (hipStream_t; NULL = legacy stream). */
int rsvio_unproject_d(const rsvio_camera* cam, const float* d_px, size_t n, float* d_out_xy,
                      uint8_t* d_valid_out, void* stream);
/* Frame::add_left_feature / add_right_feature on the tracker's output: after this call every
 * process_frame also unprojects both cameras' features on device (fused into the output
 * packing) and rsvio_tracker_undistorted returns them in feature order.  NULL, NULL turns it
 * off. */
int rsvio_tracker_set_cameras(rsvio_tracker* t, const rsvio_camera* left, const rsvio_camera* right);
int rsvio_tracker_undistorted(rsvio_tracker* t, float* out_l, size_t cap_l, float* out_r, size_t cap_r);

/* =========================== HP-B: sliding-window BA =========================== */

enum {
    RSVIO_LM_COST_TOLERANCE = 1,      /* OptimizationStatus::CostToleranceReached */
    RSVIO_LM_PARAMETER_TOLERANCE = 2, /* ::ParameterToleranceReached */
    RSVIO_LM_MAX_ITERATIONS = 3,      /* ::MaxIterationsReached (counts as success, sliding_window.rs:393) */
    RSVIO_LM_TRUST_REGION = 4,        /* ::TrustRegionRadiusTooSmall */
    RSVIO_LM_NUMERICAL_FAILURE = -1,  /* ::NumericalFailure -> caller reverts (:354-359) */
    RSVIO_LM_SKIPPED = -2,            /* too few residuals (:309-319) -> Ok(false) */
    RSVIO_LM_LINEAR_SOLVE_FAILED = -3 /* Err(LinearSolveFailed / "Singular matrix"): the caller retries
                                       * with RSVIO_SOLVER_CHOLESKY, then reverts (:326-353) */
};

enum {
    RSVIO_SOLVER_SCHUR = 0,     /* LinearSolverType::SparseSchurComplement (sliding_window.rs:126-135) */
    RSVIO_SOLVER_CHOLESKY = 1   /* LinearSolverType::SparseCholesky, the fallback (:334-341): the full
                                 * damped system, landmarks eliminated first (3x3 LL^T blocks) */
};

typedef struct {
    int32_t max_iterations;       /* 20  (sliding_window.rs:131) */
    double cost_tolerance;        /* 1e-6 (:132) */
    double parameter_tolerance;   /* 1e-9 (:133) */
    double huber_delta;           /* 2.0 (:295) */
    double lambda_init;           /* 1e-4 (build's LM) */
    int32_t linear_solver;        /* RSVIO_SOLVER_* (BA only; PnP always solves its 6x6 by Cholesky) */
} rsvio_lm_cfg;

typedef struct {
    int32_t status;               /* RSVIO_LM_* ; success iff > 0 (is_optimization_successful :384-395) */
    int32_t iterations;
    double initial_cost;
    double final_cost;
    double solve_ms;              /* device time of the solve (HIP events) */
} rsvio_ba_result;

typedef struct {
    int32_t max_keyframes;        /* window size (config/euroc_vio.yaml:35) */
    int32_t max_landmarks;
    int32_t max_observations;
    int32_t device;
} rsvio_ba_params;

typedef struct rsvio_ba rsvio_ba;

int rsvio_ba_create(const rsvio_ba_params* params, rsvio_ba** out);
void rsvio_ba_destroy(rsvio_ba* ba);

/* SlidingWindow::optimize's solver call (sliding_window.rs:325): LM with Schur elimination of
 * the landmarks on BundleAdjustmentFactor residuals (factors.rs:350-447) + Huber.
 * Observations: landmark index, keyframe index, camera (0 = left, 1 = right), normalised
 * undistorted coordinates (frame.rs:118-119).  T_C_B2: two row-major 4x4 (T_Cl_B, T_Cr_B).
 * pose7 and p_W are updated in place on success (status > 0). */
int rsvio_ba_solve(rsvio_ba* ba, int32_t n_kf, double* pose7, const uint8_t* kf_fixed,
                   int32_t n_lm, double* p_W, int32_t n_obs, const int32_t* obs_lm,
                   const int32_t* obs_kf, const uint8_t* obs_cam, const double* obs_uv,
                   const double* T_C_B2, const rsvio_lm_cfg* cfg, rsvio_ba_result* res);

/* Split form: upload a window, solve it (possibly many times from the uploaded initial state;
 * nothing crosses PCIe inside rsvio_ba_run except the status).  Observations may come in any
 * order; one per (landmark, keyframe, camera) -- a second is RSVIO_ERR_INVALID_ARG, as is an
 * index out of range.  The host validates the observations and packs per-landmark (keyframe,
 * camera) masks into pinned staging; the slot layout and Schur pair lists are built on the
 * device after one H2D copy.  Does not wait for the previous solve's stream tail.  The window's
 * geometry and buffer addresses also go up as a device descriptor: the first solve of a window
 * replays a launch graph keyed only by the window's shape (free keyframes, LM configuration, wave
 * count within a band), so a new keyframe window costs one graph launch, no capture. */
int rsvio_ba_set_problem(rsvio_ba* ba, int32_t n_kf, const double* pose7, const uint8_t* kf_fixed,
                         int32_t n_lm, const double* p_W, int32_t n_obs, const int32_t* obs_lm,
                         const int32_t* obs_kf, const uint8_t* obs_cam, const double* obs_uv,
                         const double* T_C_B2);
int rsvio_ba_run(rsvio_ba* ba, const rsvio_lm_cfg* cfg, rsvio_ba_result* res);
/* rsvio_ba_run split in two so the host can overlap other work (e.g. the next frame's
 * tracking) with the solve: _run_async enqueues the first chunk of LM iterations and returns;
 * _wait completes the solve and fills res.  One solve in flight per handle.  Single rank, _wait
 * returns when the final LM state has landed in host memory (a ticket the last decision kernel
 * publishes); the stream may still be draining that kernel's exit, and the handle synchronises
 * it before any later call copies to or from its buffers.  res->solve_ms: device wall clock
 * from the solve's first kernel to its last decision. */
int rsvio_ba_run_async(rsvio_ba* ba, const rsvio_lm_cfg* cfg);
/* Enqueue the handle's work on a caller-owned stream (NULL: back to the handle's own stream). */
int rsvio_ba_set_stream(rsvio_ba* ba, void* stream);
int rsvio_ba_wait(rsvio_ba* ba, rsvio_ba_result* res);
/* The current state (n_kf x 7 poses, n_lm x 3 points).  After the first call on a handle, each
 * later solve's final decision kernel also publishes the optimised state to pinned host memory
 * (one slice per workgroup, each with its own flag), and get_state copies it from there without
 * a stream synchronisation; otherwise (or after rsvio_ba_build_system, a skipped solve, a batch
 * run) it is copied from the device buffers. */
int rsvio_ba_get_state(rsvio_ba* ba, double* pose7, double* p_W);
/* Reduced camera system at `lambda` for the uploaded state (parity tests):
 * S is n x n row-major (n = 6 * free keyframes, ascending keyframe order), b is n. */
int rsvio_ba_build_system(rsvio_ba* ba, double lambda, double huber_delta, double* S, double* b,
                          double* cost);

/* Batched mode: n independent windows -- each a handle whose problem was
 * uploaded by rsvio_ba_set_problem -- solved by ONE launch chain (the window is a grid dimension
 * of every LM kernel; one camera-solve workgroup per window), each window exactly as its own
 * rsvio_ba_run would solve it (SlidingWindow::optimize, sliding_window.rs:159-381, per window).
 * Windows may differ in keyframes (<= 10 free each), landmarks and observations; a window the
 * guards of sliding_window.rs:303-319 skip reports RSVIO_LM_SKIPPED.  results[i] is window i's;
 * solve_ms is the whole batch's.  rsvio_ba_get_state on a window handle reads its solution.  The
 * batch borrows the handles (they must outlive it) and runs on its own stream. */
typedef struct rsvio_ba_batch rsvio_ba_batch;
int rsvio_ba_batch_create(rsvio_ba* const* windows, int32_t n, rsvio_ba_batch** out);
int rsvio_ba_batch_run(rsvio_ba_batch* batch, const rsvio_lm_cfg* cfg, rsvio_ba_result* results);
void rsvio_ba_batch_destroy(rsvio_ba_batch* batch);

/* Landmark sharding over ranks: each rank uploads only its own
 * landmarks/observations; the reduced system and costs are summed with RCCL over xGMI. */
int rsvio_rccl_unique_id(uint8_t* out, size_t cap);   /* cap >= 128 */
int rsvio_ba_attach_comm(rsvio_ba* ba, int32_t nranks, int32_t rank, const uint8_t* unique_id);
/* Peer-to-peer one-shot all-reduce for the same exchanges (latency-bound small messages over
 * xGMI): each rank exports its exchange buffer (64-byte IPC handle), the handles of all ranks
 * are exchanged by the caller, then every rank attaches; attach runs a self-test and fails
 * (the handle keeps RCCL / its previous collective) if any peer is unreachable.  All ranks
 * must end in the same mode: on any rank's failure every rank calls rsvio_ba_detach_p2p. */
int rsvio_ba_p2p_export(rsvio_ba* ba, int32_t nranks, uint8_t* handle_out, size_t cap);
int rsvio_ba_attach_p2p(rsvio_ba* ba, int32_t nranks, int32_t rank, const uint8_t* handles);
int rsvio_ba_detach_p2p(rsvio_ba* ba);
/* Diagnostics (no reference counterpart): average device microseconds of one P2P exchange of n
 * doubles (1 <= n <= 8192) over reps back-to-back exchanges after one warm-up; collective --
 * every attached rank makes the same call.  Reported by bench.py at N > 1. */
int rsvio_ba_p2p_latency(rsvio_ba* ba, int32_t reps, int32_t n, double* us_out);
/* Diagnostics (no reference counterpart): the exchange form the current problem's LM iterations
 * take -- -1 not P2P-sharded; 0 five launches (X1, X2); 1 four (K5 exchanges the system, X2 the
 * trial scalars); 2, 3, 4 three (the trial exchange folded into K6 / the next decision).  Level 3
 * (the default) needs K6's whole grid resident on the stream's CUs at once (its reducer workgroup
 * waits inside the grid); a problem past that capacity takes level 1, bit-identically. */
int rsvio_ba_p2p_level(rsvio_ba* ba, int32_t* level_out);

/* ===== B8: motion tracking (PnP) + keyframe rule (SlidingWindow::track_motion) ===== */

/* One SE3 pose (T_B_W) against the fixed map: PnPFactor (src/optimization/factors.rs:455-583,
 * no cheirality guard, J = [dt | dw]) with Huber(2.0), the build's LM with
 * max 10 iterations (sliding_window.rs:494-501), initialised from the last keyframe
 * (:506-517); then the keyframe rule of estimator.rs:195-226.  The whole sequence -- map join,
 * LM, T_W_B = inverse(SE3), T_rel, euler angles, thresholds -- is one single-workgroup kernel. */
typedef struct rsvio_pnp rsvio_pnp;

typedef struct {
    double translation_threshold;  /* keyframe_management.translation_threshold (euroc 0.05) */
    double rotation_threshold;     /* keyframe_management.rotation_threshold    (euroc 0.05) */
} rsvio_keyframe_rule;

typedef struct {
    int32_t status;            /* RSVIO_LM_*; > 0 or TRUST_REGION is success (:384-395) */
    int32_t iterations;
    int32_t is_keyframe;       /* estimator.rs:216-225; 1 on failure (frame keeps is_keyframe) */
    int32_t n_observations;    /* features with a map point (:521-547) */
    double initial_cost;
    double final_cost;
    double translation_norm;   /* ||t_rel|| (estimator.rs:206) */
    double rotation_norm;      /* ||euler(R_rel)|| (:207-212) */
    double T_W_B[16];          /* row-major; identity on failure (frame.rs:95, state.rs:26) */
    double kernel_ms;          /* device time of the launch: its first wave's entry to the result
                                  write (the device wall clock; no host or copy time) */
} rsvio_motion_result;        /* 184 bytes */

int rsvio_pnp_create(int32_t device, rsvio_pnp** out);
void rsvio_pnp_destroy(rsvio_pnp* p);
/* UnitQuaternion::from_matrix (sliding_window.rs:221,511; estimator.rs:209-211): nalgebra's
 * iterative Rotation3::from_matrix_eps(m, f64::EPSILON, 0, identity) then from_rotation_matrix,
 * for n row-major 3x3 matrices -> n quaternions (w, i, j, k).  Host only (no device needed). */
int rsvio_quat_from_matrix(const double* R, size_t n, double* q);
/* ---- the Estimator's per-keyframe host logic (host only, no device needed) ---- */

/* SlidingWindow::optimize's problem assembly (sliding_window.rs:174-300) for a window of n_kf
 * keyframes: T_W_B (n_kf row-major 4x4), T_B_C2 (the FRONT keyframe's T_B_Cl, T_B_Cr; :180-181),
 * per keyframe k and camera c (list 2k + c, the 2 n_kf lists back to back in ids / uv, n_feat[i]
 * entries each) the features' ids and undistorted coordinates (frame.rs:107-134, f32), the map (ids strictly ascending, p_W as f32; :466-475).  Out: pose7
 * (T_B_W as [t; w, i, j, k], :214-226), kf_fixed (KF_0), T_C_B2 (T_Cl_B, T_Cr_B), the landmarks
 * -- features seen at least once in each camera across the window (:183-209, :238-240), indexed
 * by first appearance -- with their ids and initial values (map point, else depth 2.0 along the
 * first observation's ray, :241-262), and one observation per factor in window order (keyframe,
 * left then right, feature order).  RSVIO_ERR_CAPACITY when cap_lm / cap_obs are too small. */
int rsvio_window_problem(int32_t n_kf, const double* T_W_B, const double* T_B_C2, const uint64_t* ids,
                         const float* uv, const int32_t* n_feat, const uint64_t* map_ids,
                         const float* map_pw, int32_t n_map, double* pose7, uint8_t* kf_fixed, double* T_C_B2,
                         int32_t cap_lm, uint64_t* lm_ids, double* p_init, int32_t* n_lm, int32_t cap_obs,
                         int32_t* obs_lm, int32_t* obs_kf, uint8_t* obs_cam, double* obs_uv, int32_t* n_obs);
/* process_optimization_result (sliding_window.rs:418-486): keyframe T_W_B = inverse(SE3(pose7))
 * (n_kf row-major 4x4) and the map = the optimised landmarks as f32, by ascending id. */
int rsvio_window_apply(int32_t n_kf, const double* pose7, int32_t n_lm, const uint64_t* lm_ids, const double* p_W,
                       double* T_W_B, uint64_t* map_ids, float* map_pw);

/* Launch rsvio_track_motion on a caller-owned stream (hipStream_t; NULL: the handle's own). */
int rsvio_pnp_set_stream(rsvio_pnp* p, void* stream);
/* SlidingWindow::map_points after optimize (sliding_window.rs:466-475): feature ids strictly
 * ascending, p_W as f32 triples. */
int rsvio_pnp_set_map(rsvio_pnp* p, const uint64_t* ids, const float* p_W, int32_t n);
/* track_motion(&Frame) + keyframe rule for a frame given as host arrays (feature ids and
 * undistorted coordinates per camera, frame.rs:107-134).  T_W_B_last_kf: keyframes.back()
 * (:506); T_C_B2: T_Cl_B, T_Cr_B of keyframes.front() (:520-521), row-major 4x4 each. */
int rsvio_track_motion(rsvio_pnp* p, const uint64_t* ids_l, const float* uv_l, size_t n_l,
                       const uint64_t* ids_r, const float* uv_r, size_t n_r,
                       const double* T_W_B_last_kf, const double* T_C_B2, const rsvio_lm_cfg* cfg,
                       const rsvio_keyframe_rule* rule, rsvio_motion_result* res);
/* Same for the tracker's last COLLECTED frame, read in place on the device (ids and the fused
 * undistorted coordinates; needs rsvio_tracker_set_cameras): no host round trip between
 * tracking and motion tracking.  Runs on the pnp handle's stream, so it may run while the next
 * frame (rsvio_tracker_submit*) is being tracked: that frame writes the other output slot. */
int rsvio_track_motion_tracker(rsvio_pnp* p, rsvio_tracker* t, const double* T_W_B_last_kf,
                               const double* T_C_B2, const rsvio_lm_cfg* cfg,
                               const rsvio_keyframe_rule* rule, rsvio_motion_result* res);

#ifdef __cplusplus
}
#endif
#endif
