/*
 * rsvio_oracle.h -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * CPU restatement of the two RS-VIO hot paths (EthanD11/RS-VIO, snapshot 2026-03-20),
 * used only as the parity checker by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  The product library (rs-vio_amd/lib/librsvio_gpu.so)
 * never links or loads it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - Reference is pure Rust; no cargo/rustc here => the reference cannot be built.
 *     No golden vectors exist upstream for either path.
 *   - The oracle is pinned only by the reference's own known-answer tests that apply
 *     (exp_se2 KATs, feature_tracker/src/feature_tracker/feature_tracking.rs:264-291;
 *     pyramid dimensions, feature_tracker/src/image_operations.rs:84-94; the
 *     translation-only BA convergence property, src/optimization/tests.rs:135-380).
 *     Third-party arithmetic (image::imageops::resize Triangle, imageproc corners_fast9,
 *     apex-solver LM) is restated from the crates' published algorithms and is
 *     "parity unpinned".
 *
 * Conventions
 *   Affine2 (nalgebra Affine2<f32>) is passed as float[6] = {m11, m12, m21, m22, m13, m23}.
 *   Pyramid levels are packed back to back: level i (width w>>i... see orc_pyramid_offset)
 *   starts at orc_pyramid_offset(w, h, i).
 *   Poses are 7-vectors [tx, ty, tz, qw, qx, qy, qz] of T_B_W (sliding_window.rs:222-224).
 */
#ifndef RSVIO_ORACLE_H
#define RSVIO_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- tracker (src/feature_tracker/) ---------------- */

/* The trackers' trig is glibc sinf/cosf (what Rust f32::sin/cos call on linux-gnu).  Per-chunk
 * digests of libm over f32 bit patterns, as rsvio_sincosf_digest defines them (the checker of
 * the device restatement). */
void orc_libm_sincosf_digest(uint64_t first, uint64_t count, uint32_t chunk_log2, int nthreads,
                             uint64_t* digests);

/* se2_exp_matrix (image_utilities.rs:82-106), twist [vx, vy, theta] -> row-major 3x3 */
void orc_se2_exp(const float* twist, float* out9);

size_t orc_pyramid_offset(int w, int h, int level);
size_t orc_pyramid_bytes(int w, int h, int levels);

/* feature_tracker.rs:209-220 (imageops::resize Triangle from full resolution per level) */
void orc_build_pyramid_mt(const uint8_t* img, int w, int h, int levels, uint8_t* out, int n_threads);
void orc_build_pyramid(const uint8_t* img, int w, int h, int levels, uint8_t* out);

/* image 0.25 imageops::resize(.., FilterType::Triangle), u8 luma */
void orc_resize_triangle(const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh);

/* patch.rs:124-162 -- exposes the template for white-box parity tests.
 * out_data[52], out_hinvjt[3*52] (row-major 3x52); returns valid flag. */
int orc_pattern52_new(const uint8_t* img, int w, int h, float px, float py,
                      float* out_data, float* out_hinvjt, float* out_mean);

/* feature_tracker.rs:344-395; aff in/out float[6]; returns success flag */
int orc_track_point_at_level(const uint8_t* img, int w, int h, const uint8_t* tmpl_img,
                             float px, float py, float* aff, int max_iter, float thresh);

/* feature_tracker.rs:292-342; returns 1 and writes aff_out on success */
int orc_track_one_point(const uint8_t* pyr0, const uint8_t* pyr1, int w, int h, int levels,
                        const float* aff_in, int max_iter, float thresh, float* aff_out);

/* feature_tracker.rs:252-291 (forward + backward + ||dt||^2 < 0.4 check), per feature */
void orc_track_points(const uint8_t* pyr0, const uint8_t* pyr1, int w, int h, int levels,
                      const float* aff_in, int n, int max_iter, float thresh,
                      float* aff_out, uint8_t* valid_out, int n_threads);

/* imageproc corners_fast9 restatement on a full image: writes score per pixel
 * (0 = not a corner at `threshold`), returns corner count. */
int orc_fast9_scores(const uint8_t* img, int w, int h, int threshold, uint8_t* score_out);

/* image_utilities.rs:108-175 with num_points_in_cell = 1.
 * existing_xy: n_existing x 2 float tracked positions (rounded like feature_tracker.rs:232-233).
 * out_xy: corner positions (u32 pairs), returns count (<= cap). */
int orc_detect_keypoints(const uint8_t* img, int w, int h, int grid, const float* existing_xy,
                         int n_existing, uint32_t* out_xy, float* out_score, int cap);

/* StereoPatchTracker (feature_tracker.rs:91-207) with canonical (ascending id) ordering */
typedef struct orc_tracker orc_tracker;
typedef struct {
    uint64_t id;
    float x, y;
    float aff[6];
} orc_feature;
orc_tracker* orc_tracker_create(int w, int h, int levels, int grid, int max_iter, float thresh);
void orc_tracker_destroy(orc_tracker* t);
void orc_tracker_set_threads(orc_tracker* t, int threads);  /* all-cores CPU leg; 1 = sequential */
/* returns 0; fills up to cap features per camera, counts in n_l/n_r */
int orc_tracker_process_frame(orc_tracker* t, const uint8_t* left, const uint8_t* right,
                              orc_feature* out_l, int cap_l, int* n_l,
                              orc_feature* out_r, int cap_r, int* n_r);
void orc_tracker_remove_ids(orc_tracker* t, const uint64_t* ids, int n);

/* ---------------- feature_tracker/ crate (secondary tracker variant, SURVEY T-sec) ----------------
 * f32 images in [0, 1] (image::DynamicImage::to_luma32f, players/tartanair_player.rs:53); pyramid
 * levels packed back to back, level l = round(w / ratio^l) x round(h / ratio^l)
 * (image_operations.rs:69-70).  SE(2) results as float[4] = {cos, sin, tx, ty} (Isometry2). */
typedef struct {
    int32_t nlevels;                  /* config.yaml:1  -> 5 */
    double ratio;                     /* :2  -> 2.0 */
    int32_t preprocessing_blur;       /* :4  -> true */
    float preprocessing_blur_sigma;   /* :5  -> 2.0 */
    float detection_threshold;        /* :8  -> 2.5 */
    uint32_t detection_min_dist;      /* :7  -> 15 */
    float detection_blur;             /* :9  -> 6.0 */
    int32_t optical_flow_max_iter;    /* :11 -> 25 */
    float optical_flow_lm_lambda;     /* :12 -> 0.1 */
    int32_t matching_cost;            /* 0 = SSD (feature_tracker.rs:125), 1 = LSSD */
} orc_ft_config;

void orc_ft_level_dims(int w, int h, int nlevels, double ratio, int* dims);
size_t orc_ft_pyramid_floats(int w, int h, int nlevels, double ratio);
void orc_ft_resize_triangle(const float* src, int w, int h, float* dst, int nw, int nh);
void orc_ft_gaussian_blur(const float* src, int w, int h, float sigma, float* dst);
void orc_ft_fast_blur(const float* src, int w, int h, float sigma, float* dst);
void orc_ft_boxes_for_gauss(float sigma, int n, int* out);
/* image_operations.rs:47-78 */
void orc_ft_build_pyramid(const float* img, int w, int h, int nlevels, double ratio, int blur, float sigma,
                          float* out);
/* image_operations.rs:140-229: returns 0 when out of bounds; out3 = {value, d/dx, d/dy} */
int orc_ft_bicubic(const float* img, int w, int h, float x, float y, float* out3);
/* feature_tracking.rs:195-219, twist {theta, vx, vy} -> {cos, sin, tx, ty} */
void orc_ft_exp_se2(const float* twist, float* out4);
/* feature_tracking.rs:221-244, {cos, sin, tx, ty} -> {theta, vx, vy} */
void orc_ft_log_se2(const float* iso4, float* out3);
/* patch.rs:240-255: data[52], jac[52*3] row-major, hinv[9]; returns try_inverse's success */
int orc_ft_patch_new(const float* img, int w, int h, float cx, float cy, float lambda, int cost, float* data,
                     float* jac, float* hinv);
/* feature_tracking.rs:16-61 per feature: iso_out n x 4 (forward transform), valid n */
void orc_ft_track_points(const float* pyr0, const float* pyr1, int w, int h, int nlevels, double ratio,
                         const float* xy, int n, int max_iter, float lambda, int cost, float* iso_out,
                         uint8_t* valid);
/* feature_detection.rs:82-164 */
void orc_ft_shi_tomasi_score(const float* img, int w, int h, float blur, float* score);
/* feature_detection.rs:171-253; returns the full count (writes <= cap) */
int orc_ft_suppress_non_maximum(const float* score, int w, int h, int radius, float threshold, uint32_t* out_xy,
                                float* out_score, int cap);
/* feature_detection.rs:47-80; returns the full count of new corners (writes <= cap) */
int orc_ft_add_points(const float* fine, int w, int h, const float* tracked_xy, int n_tracked, float threshold,
                      int min_dist, float blur, uint32_t* out_xy, int cap);

typedef struct orc_ft orc_ft;
orc_ft* orc_ft_create(const orc_ft_config* cfg, int w, int h);
void orc_ft_destroy(orc_ft* t);
/* feature_tracker.rs:77-185: frame features = tracked (previous order) then new (ids ascending) */
int orc_ft_process_frame(orc_ft* t, const float* img, uint64_t* ids_out, float* xy_out, int cap, int* n_out);

/* ---------------- camera unprojection (src/estimator/frame.rs:107-134) ---------------- */

/* Same layout as rsvio_camera (include/rsvio_gpu.h): model 0 = OpenCVModel5
 * {fx,fy,cx,cy,k1,k2,p1,p2,k3}, 1 = EUCM {fx,fy,cx,cy,alpha,beta}; convention 0 = (x/z, y/z),
 * 1 = unit-ray components.  Parity unpinned (camera_oracle.cpp header). */
typedef struct {
    int32_t model;
    int32_t convention;
    int32_t max_iterations;
    int32_t reserved;
    double params[9];
} orc_camera;

/* px: n x 2 f32 pixels -> out_xy n x 2 f32 (NaN + valid 0 on failure); returns #valid */
int orc_unproject(const orc_camera* cam, const float* px, size_t n, float* out_xy, uint8_t* valid);
/* pts: n x 3 f64 camera-frame points -> out_uv n x 2 f64 pixels; returns #valid */
int orc_project(const orc_camera* cam, const double* pts, size_t n, double* out_uv, uint8_t* valid);

/* ---------------- bundle adjustment (src/optimization/factors.rs, sliding_window.rs) ---------------- */

typedef struct {
    int max_iterations;        /* sliding_window.rs:131 -> 20 */
    double cost_tolerance;     /* :132 -> 1e-6 */
    double parameter_tolerance;/* :133 -> 1e-9 */
    double huber_delta;        /* :295 -> 2.0 */
    double lambda_init;        /* build's own LM -> 1e-4 */
    int linear_solver;         /* 0 SparseSchurComplement, 1 SparseCholesky fallback (:334-341) */
} orc_lm_cfg;

typedef struct {
    int status;      /* RSVIO_LM_* codes, shared with include/rsvio_gpu.h */
    int iterations;
    double initial_cost;
    double final_cost;
} orc_ba_result;

/* factors.rs:350-447 -- one observation; J is 2x9 row-major [dp_W | dt | dw];
 * pose7 == NULL means "fixed pose" given by T_B_W_fixed (3x4 row-major). */
void orc_ba_factor_linearize(const double* p_W, const double* pose7, const double* T_B_W_fixed,
                             const double* T_C_B, const double* uv, double* r, double* J);

/* Reduced camera system at a given lambda for the current parameters.
 * S is n x n (n = 6 * free KFs, free KFs in ascending KF order), b is n. */
int orc_ba_build_system(int n_kf, const double* pose7, const uint8_t* kf_fixed,
                        int n_lm, const double* p_W,
                        int n_obs, const int32_t* obs_lm, const int32_t* obs_kf,
                        const uint8_t* obs_cam, const double* obs_uv, const double* T_C_B2,
                        double huber_delta, double lambda, double* S, double* b, double* cost);

/* Full LM solve (build's restatement of apex-solver LM with Schur elimination). */
/* threads of the BA restatement (1 = sequential reference order; T > 1: T contiguous landmark
 * ranges summed in range order -- the threaded-Schur CPU baseline leg) */
void orc_set_ba_threads(int threads);
int orc_ba_solve(int n_kf, double* pose7, const uint8_t* kf_fixed,
                 int n_lm, double* p_W,
                 int n_obs, const int32_t* obs_lm, const int32_t* obs_kf,
                 const uint8_t* obs_cam, const double* obs_uv, const double* T_C_B2,
                 const orc_lm_cfg* cfg, orc_ba_result* res);

/* SE3 right-plus used by the LM update: pose7 <- pose7 (+) delta ([rho; theta]) */
void orc_se3_plus(const double* pose7, const double* delta, double* out7);

/* SlidingWindow::track_motion (sliding_window.rs:490-587) + keyframe rule (estimator.rs:195-234):
 * PnP LM on one pose from the last keyframe, T_W_B = inv(SE3), keyframe iff ||t_rel|| > thr_t or
 * ||euler(R_rel)|| > thr_r; failure -> T_W_B = I, keyframe.  Map ids strictly ascending. */
typedef struct {
    int status, iterations, is_keyframe, n_observations;
    double initial_cost, final_cost, translation_norm, rotation_norm;
    double T_W_B[16];
    double pose7[7];
} orc_motion_result;
int orc_track_motion(const uint64_t* ids_l, const float* uv_l, int n_l, const uint64_t* ids_r,
                     const float* uv_r, int n_r, const uint64_t* map_ids, const float* map_pw, int n_map,
                     const double* T_W_B_last_kf, const double* T_C_B2, const orc_lm_cfg* cfg,
                     double thr_t, double thr_r, orc_motion_result* res);

/* nalgebra UnitQuaternion::from_matrix restatement (sliding_window.rs:221) */
void orc_quat_from_rotation(const double* R, double* qwxyz);
/* UnitQuaternion::from_matrix: nalgebra's iterative from_matrix_eps, then from_rotation_matrix */
void orc_quat_from_matrix(const double* R, double* qwxyz);

#ifdef __cplusplus
}
#endif
#endif
