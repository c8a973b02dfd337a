// estimator.cpp -- Estimator::process_frame (src/estimator/estimator.rs:101-262) as a compiled
// caller runs it: the host logic of rsvio.estimator.Estimator (pipelined, the tracker one frame
// ahead) over the library's C ABI, without an interpreter between the calls.
//
// The reference's estimator is Rust; cargo is absent here, so the parity-tested host mirror is
// Python (rs-vio_amd/rsvio/estimator.py + ba.SlidingWindow).  This file restates the same logic
// step for step in C++ -- the keyframe FIFO, map_points as ascending ids + f32 points, the problem
// build and result apply by the library's own host code (rsvio_window_problem / _apply), the
// SparseCholesky retry, PnP + keyframe rule, the pending solve finished before the window is next
// read -- so the config-4 row can be measured with host overhead of the reference's kind.  The
// device handles (tracker with cameras, PnP, BA, their streams) are created by the caller; the
// library's entry points come in as function pointers of the library the caller loaded.
// tests/test_estimator_gpu.py checks it frame by frame against the Python Estimator.
#include <chrono>
#include <cstdint>
#include <cstring>
#include <deque>
#include <vector>

#include "rsvio_gpu.h"

namespace {

struct Keyframe {
    double T_W_B[16];
    std::vector<uint64_t> ids[2];  // left, right (feature order)
    std::vector<float> uv[2];      // undistorted, 2 per feature
};

}  // namespace

extern "C" {

struct rsvio_est_api {
    decltype(&rsvio_tracker_submit_device) submit_device;
    decltype(&rsvio_tracker_collect) collect;
    decltype(&rsvio_tracker_undistorted) undistorted;
    decltype(&rsvio_pnp_set_map) set_map;
    decltype(&rsvio_track_motion_tracker) track_motion;
    decltype(&rsvio_window_problem) window_problem;
    decltype(&rsvio_window_apply) window_apply;
    decltype(&rsvio_ba_set_problem) set_problem;
    decltype(&rsvio_ba_run_async) run_async;
    decltype(&rsvio_ba_wait) wait;
    decltype(&rsvio_ba_run) run;
    decltype(&rsvio_ba_get_state) get_state;
};

struct rsvio_est_setup {
    const rsvio_est_api* api;
    rsvio_tracker* tracker;      // cameras attached (rsvio_tracker_set_cameras)
    rsvio_pnp* pnp;
    rsvio_ba* ba;
    int32_t window;              // sliding window size (config/euroc_vio.yaml: 10)
    int32_t max_features;        // the tracker's capacity per camera
    double T_B_Cl[16], T_B_Cr[16];
    double T_C_B2[32];           // T_Cl_B, T_Cr_B of the (fixed) rig, as the caller inverts them
    rsvio_lm_cfg ba_cfg;         // sliding_window.rs:126-135
    rsvio_lm_cfg ba_fallback;    // the SparseCholesky retry (:333-341)
    rsvio_lm_cfg pnp_cfg;        // :494-501
    rsvio_keyframe_rule rule;    // estimator.rs:201-225
};

struct rsvio_est_frame {         // rsvio.estimator.FrameResult; "none" fields are INT32_MIN
    int32_t frame_id, is_keyframe, n_left, n_right;
    int32_t pnp_status, pnp_iterations, ba_status, ba_iterations;
    double pnp_cost;
    double T_W_B[16];
};

struct rsvio_est_stats {         // host wall seconds per stage (the Python row's _StageTimer)
    double track, track_motion, ba, ba_wait, total;
    int32_t n_solves, ba_iterations, fallbacks, reserved;
};

// Runs Estimator.run over n frames (device-resident images, tightly packed): out[k] per frame.
// Returns 0 or a negative RSVIO_ERR_* of the first failing call.
int rsvio_est_run(const rsvio_est_setup* S, const uint8_t* const* d_left, const uint8_t* const* d_right,
                  int32_t n_frames, rsvio_est_frame* out, rsvio_est_stats* stats) {
    if (!S || !S->api || !S->tracker || !S->pnp || !S->ba || !out || !stats || S->window < 1 || n_frames < 0 ||
        S->max_features < 1)
        return RSVIO_ERR_INVALID_ARG;
    const rsvio_est_api& A = *S->api;
    constexpr int32_t kNone = INT32_MIN;
    using clk = std::chrono::steady_clock;
    auto secs = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
    *stats = rsvio_est_stats{};
    const auto t_start = clk::now();

    std::deque<Keyframe> kfs;
    std::vector<uint64_t> map_ids;     // map_points: ascending ids, [f32; 3] points
    std::vector<float> map_pw;
    long map_version = 0, map_key = -1;
    // the pending solve (optimize_async): its landmark ids and its frame's result slot
    bool pending = false;
    int32_t pending_out = -1;
    std::vector<uint64_t> lm_ids;
    // scratch
    const size_t cap = (size_t)S->max_features;
    std::vector<rsvio_feature> fl(cap), fr(cap);
    std::vector<double> pose7, p_init, obs_uv, pose_out, pw_out, T_all;
    std::vector<uint8_t> fixed, obs_cam;
    std::vector<int32_t> obs_lm, obs_kf, n_feat;
    std::vector<uint64_t> ids_all, lm_buf, new_map_ids;
    std::vector<float> uv_all, new_map_pw;
    int rc = 0;

    // SlidingWindow.finish + Estimator.flush: wait, the SparseCholesky retry, read back, apply
    auto flush = [&]() -> int {
        if (!pending) return 0;
        pending = false;
        const auto t0 = clk::now();
        rsvio_ba_result res{};
        int r = A.wait(S->ba, &res);
        if (r) return r;
        if (res.status == RSVIO_LM_LINEAR_SOLVE_FAILED) {
            ++stats->fallbacks;
            if ((r = A.run(S->ba, &S->ba_fallback, &res))) return r;
        }
        const int32_t n = (int32_t)kfs.size(), m = (int32_t)lm_ids.size();
        stats->n_solves += 1;
        stats->ba_iterations += res.iterations;
        if (res.status > 0) {
            pose_out.resize((size_t)7 * n);
            pw_out.resize((size_t)3 * (m ? m : 1));
            if ((r = A.get_state(S->ba, pose_out.data(), pw_out.data()))) return r;
            T_all.resize((size_t)16 * n);
            new_map_ids.resize(m ? m : 1);
            new_map_pw.resize((size_t)3 * (m ? m : 1));
            if ((r = A.window_apply(n, pose_out.data(), m, m ? lm_ids.data() : nullptr, m ? pw_out.data() : nullptr,
                                    T_all.data(), m ? new_map_ids.data() : nullptr, m ? new_map_pw.data() : nullptr)))
                return r;
            map_ids.assign(new_map_ids.begin(), new_map_ids.begin() + m);
            map_pw.assign(new_map_pw.begin(), new_map_pw.begin() + (size_t)3 * m);
            ++map_version;
            for (int32_t k = 0; k < n; ++k) std::memcpy(kfs[k].T_W_B, &T_all[(size_t)16 * k], sizeof(double) * 16);
        }
        rsvio_est_frame& o = out[pending_out];
        o.ba_status = res.status;
        o.ba_iterations = res.iterations;
        std::memcpy(o.T_W_B, kfs.back().T_W_B, sizeof o.T_W_B);  // the solve refined this keyframe too
        stats->ba_wait += secs(t0, clk::now());
        return 0;
    };

    if (n_frames == 0) return 0;
    auto t0 = clk::now();
    if ((rc = A.submit_device(S->tracker, d_left[0], d_right[0]))) return rc;
    stats->track += secs(t0, clk::now());
    for (int32_t k = 0; k < n_frames; ++k) {
        // collect frame k, submit frame k + 1 (the tracker one frame ahead)
        t0 = clk::now();
        size_t nl = 0, nr = 0;
        if ((rc = A.collect(S->tracker, fl.data(), cap, &nl, fr.data(), cap, &nr))) return rc;
        Keyframe f;
        for (int c = 0; c < 2; ++c) {
            const size_t nc = c ? nr : nl;
            const rsvio_feature* src = c ? fr.data() : fl.data();
            f.ids[c].resize(nc);
            for (size_t i = 0; i < nc; ++i) f.ids[c][i] = src[i].id;
            f.uv[c].resize(2 * (nc ? nc : 1));
        }
        if ((rc = A.undistorted(S->tracker, f.uv[0].data(), nl, f.uv[1].data(), nr))) return rc;
        if (k + 1 < n_frames && (rc = A.submit_device(S->tracker, d_left[k + 1], d_right[k + 1]))) return rc;
        stats->track += secs(t0, clk::now());

        // _process_tracked (estimator.rs:195-248)
        rsvio_est_frame& o = out[k];
        o.frame_id = k + 1;
        o.n_left = (int32_t)nl;
        o.n_right = (int32_t)nr;
        o.pnp_status = o.pnp_iterations = o.ba_status = o.ba_iterations = kNone;
        o.pnp_cost = 0.0;
        for (int i = 0; i < 16; ++i) f.T_W_B[i] = (i % 5 == 0) ? 1.0 : 0.0;
        bool is_kf = true;
        if ((rc = flush())) return rc;
        if ((int32_t)kfs.size() >= S->window) {
            t0 = clk::now();
            if (map_version != map_key) {  // map_points changes only in optimize
                if ((rc = A.set_map(S->pnp, map_ids.empty() ? nullptr : map_ids.data(),
                                    map_pw.empty() ? nullptr : map_pw.data(), (int32_t)map_ids.size())))
                    return rc;
                map_key = map_version;
            }
            rsvio_motion_result mr{};
            if ((rc = A.track_motion(S->pnp, S->tracker, kfs.back().T_W_B, S->T_C_B2, &S->pnp_cfg, &S->rule, &mr)))
                return rc;
            o.pnp_status = mr.status;
            o.pnp_iterations = mr.iterations;
            o.pnp_cost = mr.final_cost;
            if (mr.status > 0) {
                std::memcpy(f.T_W_B, mr.T_W_B, sizeof f.T_W_B);
                is_kf = mr.is_keyframe != 0;
            }
            stats->track_motion += secs(t0, clk::now());
        }
        o.is_keyframe = is_kf ? 1 : 0;
        std::memcpy(o.T_W_B, f.T_W_B, sizeof o.T_W_B);
        if (is_kf) {
            // SlidingWindow.add_frame, then optimize_async once full (sliding_window.rs:137-381)
            if ((int32_t)kfs.size() >= S->window) kfs.pop_front();
            kfs.push_back(std::move(f));
            if ((int32_t)kfs.size() >= S->window) {
                t0 = clk::now();
                const int32_t n = (int32_t)kfs.size();
                size_t tot = 0;
                for (const Keyframe& q : kfs) tot += q.ids[0].size() + q.ids[1].size();
                ids_all.resize(tot ? tot : 1);
                uv_all.resize(2 * (tot ? tot : 1));
                n_feat.resize((size_t)2 * n);
                T_all.resize((size_t)16 * n);
                size_t at = 0;
                for (int32_t i = 0; i < n; ++i) {
                    std::memcpy(&T_all[(size_t)16 * i], kfs[i].T_W_B, sizeof(double) * 16);
                    for (int c = 0; c < 2; ++c) {
                        const size_t nc = kfs[i].ids[c].size();
                        if (nc) {
                            std::memcpy(&ids_all[at], kfs[i].ids[c].data(), sizeof(uint64_t) * nc);
                            std::memcpy(&uv_all[2 * at], kfs[i].uv[c].data(), sizeof(float) * 2 * nc);
                        }
                        n_feat[(size_t)2 * i + c] = (int32_t)nc;
                        at += nc;
                    }
                }
                double T_B_C2[32];
                std::memcpy(T_B_C2, S->T_B_Cl, sizeof(double) * 16);
                std::memcpy(T_B_C2 + 16, S->T_B_Cr, sizeof(double) * 16);
                const size_t c1 = tot ? tot : 1;
                pose7.resize((size_t)7 * n);
                fixed.resize(n);
                lm_buf.resize(c1);
                p_init.resize(3 * c1);
                obs_lm.resize(c1);
                obs_kf.resize(c1);
                obs_cam.resize(c1);
                obs_uv.resize(2 * c1);
                double tcb[32];
                int32_t n_lm = 0, n_obs = 0;
                if ((rc = A.window_problem(n, T_all.data(), T_B_C2, tot ? ids_all.data() : nullptr,
                                           tot ? uv_all.data() : nullptr, n_feat.data(),
                                           map_ids.empty() ? nullptr : map_ids.data(),
                                           map_pw.empty() ? nullptr : map_pw.data(), (int32_t)map_ids.size(),
                                           pose7.data(), fixed.data(), tcb, (int32_t)c1, lm_buf.data(), p_init.data(),
                                           &n_lm, (int32_t)c1, obs_lm.data(), obs_kf.data(), obs_cam.data(),
                                           obs_uv.data(), &n_obs)))
                    return rc;
                const int32_t num_vars = n + n_lm;  // KF_0 is in initial_values too (:217-226)
                if (n_obs < 6 || n_obs < num_vars) {
                    o.ba_status = kNone;  // the guards of :303-319: last_result None, no solve
                } else {
                    if ((rc = A.set_problem(S->ba, n, pose7.data(), fixed.data(), n_lm, p_init.data(), n_obs,
                                            obs_lm.data(), obs_kf.data(), obs_cam.data(), obs_uv.data(), tcb)))
                        return rc;
                    if ((rc = A.run_async(S->ba, &S->ba_cfg))) return rc;
                    lm_ids.assign(lm_buf.begin(), lm_buf.begin() + n_lm);
                    pending = true;
                    pending_out = k;
                }
                stats->ba += secs(t0, clk::now());
            }
        }
    }
    if ((rc = flush())) return rc;
    stats->total = secs(t_start, clk::now());
    return 0;
}

// Layout check for the caller's ctypes mirror (sizes, then the last fields' offsets)
int rsvio_est_layout(int64_t* o, int32_t n) {
    const int64_t v[] = {(int64_t)sizeof(rsvio_est_api), (int64_t)sizeof(rsvio_est_setup),
                         (int64_t)sizeof(rsvio_est_frame), (int64_t)sizeof(rsvio_est_stats),
                         (int64_t)offsetof(rsvio_est_setup, rule), (int64_t)offsetof(rsvio_est_setup, pnp_cfg),
                         (int64_t)offsetof(rsvio_est_frame, T_W_B), (int64_t)offsetof(rsvio_est_stats, n_solves)};
    const int32_t m = (int32_t)(sizeof v / sizeof v[0]);
    for (int32_t i = 0; i < n && i < m; ++i) o[i] = v[i];
    return m;
}

}  // extern "C"
