// pnp.hip -- B8: SlidingWindow::track_motion + the estimator's keyframe rule on gfx950 (f64).
//
// Replaces, per frame once the window is full (src/estimator/estimator.rs:195-234):
//   * the initial pose from the last keyframe, T_B_W = inv(T_W_B), q = from_matrix(R_B_W)
//     (src/estimator/sliding_window.rs:506-517);
//   * the factor list: every left then right feature whose id is in map_points gives one
//     PnPFactor (:519-547; src/optimization/factors.rs:455-583 -- no cheirality guard, 2x6
//     Jacobian [dt | dw]) with Huber(2.0);
//   * apex LM, SparseCholesky, 10 iterations, tolerances 1e-6 / 1e-9 (:494-501) -- the
//     build's LM restatement, here on a dense 6x6 system;
//   * success test (:384-395), T_W_B = inv(SE3(F)) (:566-569);
//   * the keyframe rule: T_rel = T_W_B inv(T_W_B_last_kf), ||t_rel|| > thr_t or
//     ||euler(from_matrix(R_rel))|| > thr_r (estimator.rs:201-225); on failure the frame keeps
//     is_keyframe = true and T_W_B = I (estimator.rs:228-234, frame.rs:95, state.rs:26).
//
// One workgroup of 512 lanes runs the whole sequence in one launch (no host round trip, no
// grid-wide synchronisation): the map ids are staged in LDS for the join (binary search), the
// matched observations (<= 4096 features per frame) stay in LDS, and every pass linearises all
// of them at one pose and reduces H (21), g (6) and the cost in a fixed order (DPP wave sums, then
// waves in order).  Lane 0 runs the LM control (6x6 Cholesky, SE3 (+), gain ratio) between
// passes with its state in LDS.  Each pass after the first is at a trial pose: if the step is
// accepted its H and g are the next system, so an accepted iteration costs one pass.
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "common.hpp"
#include "rotation.hpp"
#include "se3.hpp"

namespace rsvio {
namespace {

RSVIO_DBG_DECL

constexpr int kPnpThreads = 512;
constexpr int kPnpWaves = kPnpThreads / 64;
constexpr int kPnpMaxFeatures = 4096; // features per frame (both cameras), observations in LDS
constexpr int kPnpMapLds = 4096;      // map ids staged in LDS (32 KB) up to this size
constexpr int kRed = 28;          // H upper (21), g (6), cost

enum { LM_COST_TOL = 1, LM_PARAM_TOL = 2, LM_MAX_ITERS = 3, LM_TRUST_REGION = 4, LM_NUMFAIL = -1, LM_SKIPPED = -2,
       LM_LINSOLVE = -3 };

struct PnpArgs {
    const uint8_t* ids[2];   // u64 feature ids, `id_stride` bytes apart
    int id_stride;
    const float2* uv[2];     // undistorted coordinates (frame.rs:118-119,131-132)
    const int* dcount;       // device (n_l, n_r), or null: n[] below
    int n[2];
    const uint64_t* map_ids; // strictly ascending
    const float* map_pw;     // [f32; 3] per map point (sliding_window.rs:466-475)
    int n_map;
    double T_last[16];
    double q0[4];            // from_matrix(R_B_W) of the last keyframe (host, rotation.hpp)
    double TCB[2][16];
    int max_iter;
    double cost_tol, param_tol, huber_delta, lambda0, thr_t, thr_r;
    rsvio_motion_result* out;  // pinned host memory
    double wclk_khz;           // device wall clock rate (kernel_ms)
};

struct Ctl {
    double x[7], xt[7], H[21], g[6];
    double R[9], Rt[9];       // R_BW of x and of xt (pose_from7), cached for SE3 (+) and the pass
    double cost, lambda, nu, initial_cost, pred;
    int it, status, phase, run, n_obs;
};

__device__ __forceinline__ int utri6(int a, int c) { return a * 6 - (a * (a - 1)) / 2 + (c - a); }

// 64-bit cross-lane moves built from 32-bit lane ops
__device__ __forceinline__ void swap32_f64(double& x, double& y) {  // v_permlane32_swap
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double(hi[0], lo[0]);
    y = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ void swap16_f64(double& x, double& y) {  // v_permlane16_swap
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double(hi[0], lo[0]);
    y = __hiloint2double(hi[1], lo[1]);
}

// Deterministic reduce-scatter of 32 per-lane values over the wave: afterwards lanes 2p and
// 2p+1 hold the wave total of value p.  Pairings (fixed, so results are run-to-run
// identical): lanes l / l+32 (permlane32 swap), rows 0/1 and 2/3 (permlane16 swap), then
// inside each row l / l^8 (row_ror 8), the half-row mirror, quad xor 2, quad xor 1.  About
// 125 instructions instead of 32 separate wave sums (~700).
__device__ __forceinline__ double wave_reduce_scatter32(double (&v)[32], int lane) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        swap32_f64(v[i], v[16 + i]);
        v[i] = v[i] + v[16 + i];   // lanes 0-31: value i, lanes 32-63: value 16+i
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        swap16_f64(v[i], v[8 + i]);
        v[i] = v[i] + v[8 + i];    // row r: value 8r' + i (r' = row parity within the half)
    }
    const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double keep = b3 ? v[4 + i] : v[i], send = b3 ? v[i] : v[4 + i];
        v[i] = keep + dpp64<0x128>(send);    // row_ror:8 -> lane l^8
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const double keep = b2 ? v[2 + i] : v[i], send = b2 ? v[i] : v[2 + i];
        v[i] = keep + dpp64<0x141>(send);    // row_half_mirror: l <-> 7-l in each half-row
    }
    {
        const double keep = b1 ? v[1] : v[0], send = b1 ? v[0] : v[1];
        v[0] = keep + dpp64<0x4E>(send);     // quad_perm [2,3,0,1]
    }
    return v[0] + dpp64<0xB1>(v[0]);         // quad_perm [1,0,3,2]
}

// PnPFactor::linearize restated in T_C_W = T_C_B T_B_W (computed once per pass): p_C = R p_W + t,
// r = (x/z, y/z) - obs, dr/dt = jac_proj R_CW, dr/dw = jac_proj R_CB (-R_BW [p_W]x) = -(dr/dt) [p_W]x,
// i.e. row i of dr/dw is -(row i of dr/dt) x p_W.  Same values as factors.rs:545-571 up to
// rounding (~60 flops instead of ~180; tolerance parity with the oracle's reference order).
__device__ __forceinline__ void pnp_linearize_cw(const double pW[3], const double uv[2], const double* T,
                                                 double r[2], double J[2][6]) {
    const double pC0 = ((T[0] * pW[0] + T[1] * pW[1]) + T[2] * pW[2]) + T[9];
    const double pC1 = ((T[3] * pW[0] + T[4] * pW[1]) + T[5] * pW[2]) + T[10];
    const double pC2 = ((T[6] * pW[0] + T[7] * pW[1]) + T[8] * pW[2]) + T[11];
    const double iz = 1.0 / pC2;
    const double x = pC0 * iz, y = pC1 * iz;
    r[0] = x - uv[0];
    r[1] = y - uv[1];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        J[0][j] = iz * (T[j] - x * T[6 + j]);
        J[1][j] = iz * (T[3 + j] - y * T[6 + j]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        J[i][3] = J[i][2] * pW[1] - J[i][1] * pW[2];
        J[i][4] = J[i][0] * pW[2] - J[i][2] * pW[0];
        J[i][5] = J[i][1] * pW[0] - J[i][0] * pW[1];
    }
}

// (H + lambda I) dx = -g by LDL^T with hardware-reciprocal pivots (no square root, no IEEE
// division on the serial chain).  Positive definiteness is tested on the pivots exactly like
// the oracle's Cholesky (chol_solve) tests d > 0; the solution agrees to rounding (tolerance
// parity).
__device__ bool ldl6(const double* __restrict__ Hp, double lambda, const double* __restrict__ g, double* dx) {
    double A[6][6];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = a; c < 6; ++c) A[c][a] = Hp[utri6(a, c)];  // lower triangle
#pragma unroll
    for (int a = 0; a < 6; ++a) A[a][a] += lambda;
    double L[6][6], U[6][6], inv[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= L[j][k] * U[j][k];
        if (!(d > 0.0) || !isfinite(d)) return false;
        inv[j] = rcp_f64(d);
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double u = A[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) u -= L[i][k] * U[j][k];
            U[i][j] = u;
            L[i][j] = u * inv[j];
        }
    }
    double z[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double s = -g[i];
#pragma unroll
        for (int k = 0; k < i; ++k) s -= L[i][k] * z[k];
        z[i] = s;
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double s = z[i] * inv[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) s -= L[k][i] * dx[k];
        dx[i] = s;
    }
    return true;
}

// The pass pose: R_BW (9) and t_BW (3) into LDS; threads 0..23 expand it to T_C_W per camera
__device__ __forceinline__ void write_pose(double* s_pose, const double* R, const double* x7) {
#pragma unroll
    for (int k = 0; k < 9; ++k) s_pose[k] = R[k];
    s_pose[9] = x7[0];
    s_pose[10] = x7[1];
    s_pose[11] = x7[2];
}

__device__ __forceinline__ void rot_from_unit_quat(const double* q, double* R) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double ww = w * w, xx = x * x, yy = y * y, zz = z * z;
    const double xy = x * y * 2.0, wz = w * z * 2.0, wy = w * y * 2.0;
    const double xz = x * z * 2.0, yz = y * z * 2.0, wx = w * x * 2.0;
    R[0] = ww + xx - yy - zz; R[1] = xy - wz;           R[2] = wy + xz;
    R[3] = wz + xy;           R[4] = ww - xx + yy - zz; R[5] = yz - wx;
    R[6] = xz - wy;           R[7] = wx + yz;           R[8] = ww - xx - yy + zz;
}

// se3_plus with the rotation of x7 given (cached) and the rotation of the result returned
// (from its normalised quaternion): same operations as se3.hpp se3_plus otherwise.
__device__ __forceinline__ void se3_plus_r(const double* p7, const double* R, const double* d, double* out,
                                           double* Rout) {
    const double* rho = d;
    const double* om = d + 3;
    const double th2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
    const double th = sqrt(th2);
    double qd[4], Ac, Bc;
    if (th < 1e-8) {
        qd[0] = 1.0; qd[1] = 0.5 * om[0]; qd[2] = 0.5 * om[1]; qd[3] = 0.5 * om[2];
        Ac = 0.5 - th2 / 24.0;
        Bc = 1.0 / 6.0 - th2 / 120.0;
    } else {
        double sh, ch;
        sincos(0.5 * th, &sh, &ch);
        const double ith = rcp_f64(th);
        const double sth = sh * ith;
        qd[0] = ch; qd[1] = sth * om[0]; qd[2] = sth * om[1]; qd[3] = sth * om[2];
        const double ith2 = ith * ith;
        Ac = 2.0 * sh * sh * ith2;
        Bc = (th - 2.0 * sh * ch) * ith2 * ith;
    }
    const double wx[3] = {om[1] * rho[2] - om[2] * rho[1], om[2] * rho[0] - om[0] * rho[2],
                          om[0] * rho[1] - om[1] * rho[0]};
    const double wwx[3] = {om[1] * wx[2] - om[2] * wx[1], om[2] * wx[0] - om[0] * wx[2],
                           om[0] * wx[1] - om[1] * wx[0]};
    double td[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) td[i] = rho[i] + Ac * wx[i] + Bc * wwx[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) out[i] = p7[i] + ((R[3 * i] * td[0] + R[3 * i + 1] * td[1]) + R[3 * i + 2] * td[2]);
    const double w0 = p7[3], x0 = p7[4], y0 = p7[5], z0 = p7[6];
    double qn[4] = {w0 * qd[0] - x0 * qd[1] - y0 * qd[2] - z0 * qd[3], w0 * qd[1] + x0 * qd[0] + y0 * qd[3] - z0 * qd[2],
                    w0 * qd[2] - x0 * qd[3] + y0 * qd[0] + z0 * qd[1], w0 * qd[3] + x0 * qd[2] - y0 * qd[1] + z0 * qd[0]};
    const double inn = rsqrt_f64(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[3 + i] = qn[i] * inn;
    rot_from_unit_quat(out + 3, Rout);
}

// Lane 0 between passes: consume the pass in s_sum, then either set up the next pass (run = 1)
// or finish (run = 0).  Mirrors oracle orc_track_motion's loop step for step.
__device__ void pnp_control(const PnpArgs& A, Ctl* __restrict__ C, const double* __restrict__ s_sum,
                            double* __restrict__ s_pose) {
    bool done = false;
    if (C->phase == 0) {
#pragma unroll
        for (int k = 0; k < 21; ++k) C->H[k] = s_sum[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) C->g[k] = s_sum[21 + k];
        C->cost = s_sum[27];
        C->initial_cost = C->cost;
        C->phase = 1;
    } else {
        const double new_cost = s_sum[27];
        const double dcost = C->cost - new_cost;
        const double rho = dcost / C->pred;
        if (isfinite(new_cost) && fabs(dcost) <= A.cost_tol * C->cost) {
            // converged: the change is within the tolerance whatever its sign, the candidate not
            // applied (the BA's lm_update takes the same decision).  This
            // build's rule, a deliberate departure: apex-solver's is absent offline (unpinned)
            C->status = LM_COST_TOL;
            done = true;
        } else if (isfinite(new_cost) && rho > 0.0) {
#pragma unroll
            for (int k = 0; k < 7; ++k) C->x[k] = C->xt[k];
#pragma unroll
            for (int k = 0; k < 9; ++k) C->R[k] = C->Rt[k];
#pragma unroll
            for (int k = 0; k < 21; ++k) C->H[k] = s_sum[k];
#pragma unroll
            for (int k = 0; k < 6; ++k) C->g[k] = s_sum[21 + k];
            const double f = 2.0 * rho - 1.0;
            C->lambda *= fmax(1.0 / 3.0, 1.0 - f * f * f);
            C->nu = 2.0;
            C->cost = new_cost;
        } else {
            C->lambda *= C->nu;
            C->nu *= 2.0;
            if (C->lambda > 1e32) {
                C->status = LM_TRUST_REGION;
                done = true;
            }
        }
    }
    while (!done) {
        if (C->it >= A.max_iter) {
            C->status = LM_MAX_ITERS;
            break;
        }
        C->it += 1;
        if (!isfinite(C->cost)) {
            C->status = LM_NUMFAIL;
            break;
        }
        double dx[6];
        const bool solved = ldl6(C->H, C->lambda, C->g, dx);
        STAMP(30);
        if (!solved) {  // Err(LinearSolveFailed) -> track_motion returns Ok(None) (:554-560)
            C->status = LM_LINSOLVE;
            break;
        }
        double dx2 = 0.0, gdx = 0.0, x2 = 0.0;
        for (int k = 0; k < 6; ++k) {
            dx2 += dx[k] * dx[k];
            gdx += C->g[k] * dx[k];
        }
        for (int k = 0; k < 7; ++k) x2 += C->x[k] * C->x[k];
        if (sqrt(dx2) <= A.param_tol * (sqrt(x2) + A.param_tol)) {
            C->status = LM_PARAM_TOL;
            break;
        }
        se3_plus_r(C->x, C->R, dx, C->xt, C->Rt);
        STAMP(31);
        C->pred = 0.5 * (C->lambda * dx2 - gdx);
        write_pose(s_pose, C->Rt, C->xt);
        C->run = 1;
        return;
    }
    C->run = 0;
}

__device__ void pnp_finish(const PnpArgs& A, const Ctl& C, unsigned long long t_entry) {
    rsvio_motion_result r;
    r.status = C.status;
    r.iterations = C.it;
    r.n_observations = C.n_obs;
    r.initial_cost = C.initial_cost;
    r.final_cost = C.cost;
    r.translation_norm = 0.0;
    r.rotation_norm = 0.0;
    const bool ok = C.status > 0;
    if (ok) {
        // T_W_B = inv(SE3(F).matrix()) (sliding_window.rs:566-569)
        const Pose P = pose_from7(C.x);
        double TBW[16];
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) TBW[4 * i + j] = P.R[i][j];
            TBW[4 * i + 3] = P.t[i];
        }
        TBW[12] = 0.0; TBW[13] = 0.0; TBW[14] = 0.0; TBW[15] = 1.0;
        rigid_inverse(TBW, r.T_W_B);
        // the keyframe rule (estimator.rs:204-225) runs on the host after the kernel
        // (keyframe_rule(): nalgebra's iterative from_matrix is a long serial loop)
        r.is_keyframe = 0;
    } else {
        for (int k = 0; k < 16; ++k) r.T_W_B[k] = (k % 5 == 0) ? 1.0 : 0.0;
        r.is_keyframe = 1;
    }
    r.kernel_ms = (double)(wall_clock64() - t_entry) / A.wclk_khz;
    *A.out = r;
}

__global__ __launch_bounds__(kPnpThreads) void pnp_track_motion_kernel(PnpArgs A) {
    __shared__ uint64_t s_ids[kPnpMapLds];       // map ids (small maps)
    __shared__ float s_mpw[3][kPnpMapLds];       // small maps: map p_W by map index; large: by feature
    __shared__ float s_uv[2][kPnpMaxFeatures];   // undistorted coordinates per feature
    __shared__ int16_t s_idx[kPnpMaxFeatures];   // feature -> s_mpw column
    __shared__ int8_t s_cam[kPnpMaxFeatures];    // feature -> camera, -1: no map point
    __shared__ double s_red[kPnpWaves][kRed];
    __shared__ double s_sum[kRed];
    __shared__ double s_pose[12];                // R_BW, t_BW of the pass pose
    __shared__ double s_tcb[2][16];
    __shared__ double s_tcw[2][12];              // T_C_W = T_C_B T_B_W per camera at the pass pose
    __shared__ Ctl C;
    __shared__ int s_nobs;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    STAMP(0);
    const unsigned long long t_entry = wall_clock64();  // (kept by thread 0 for kernel_ms)
    const int n0 = A.dcount ? A.dcount[0] : A.n[0];
    const int n1 = A.dcount ? A.dcount[1] : A.n[1];
    const int nf = n0 + n1;
    const bool lds_map = A.n_map <= kPnpMapLds;
    // this lane's first two features: their loads are issued before the map staging so the two
    // memory latencies overlap
    auto feat = [&](int j, int& c, int& i, uint64_t& id, float2& q) {
        c = j < n0 ? 0 : 1;
        i = c == 0 ? j : j - n0;
        id = *reinterpret_cast<const uint64_t*>(A.ids[c] + (size_t)i * A.id_stride);
        q = A.uv[c][i];
    };
    const bool fits = nf <= kPnpMaxFeatures;
    int pc0 = 0, pi0 = 0, pc1 = 0, pi1 = 0;
    uint64_t pid0 = 0, pid1 = 0;
    float2 pq0 = make_float2(0.0f, 0.0f), pq1 = pq0;
    if (fits && tid < nf) feat(tid, pc0, pi0, pid0, pq0);
    if (fits && tid + kPnpThreads < nf) feat(tid + kPnpThreads, pc1, pi1, pid1, pq1);
    if (tid < 32) s_tcb[tid >> 4][tid & 15] = A.TCB[tid >> 4][tid & 15];
    if (lds_map)
        for (int i = tid; i < A.n_map; i += kPnpThreads) {
            s_ids[i] = A.map_ids[i];
            s_mpw[0][i] = A.map_pw[3 * i];
            s_mpw[1][i] = A.map_pw[3 * i + 1];
            s_mpw[2][i] = A.map_pw[3 * i + 2];
        }
    if (tid == 0) {
        s_nobs = 0;
        C.it = 0;
        C.status = LM_MAX_ITERS;
        C.phase = 0;
        C.lambda = A.lambda0;
        C.nu = 2.0;
        C.cost = 0.0;
        C.initial_cost = 0.0;
        // sliding_window.rs:506-517: F = (t_B_W, from_matrix(R_B_W)) of the last keyframe
        double TBW[16];
        rigid_inverse(A.T_last, TBW);
        C.x[0] = TBW[3];
        C.x[1] = TBW[7];
        C.x[2] = TBW[11];
#pragma unroll
        for (int k = 0; k < 4; ++k) C.x[3 + k] = A.q0[k];  // UnitQuaternion::from_matrix(R_B_W) (host)
        const Pose P0 = pose_from7(C.x);  // SE3::from (apex) of the initial 7-vector
#pragma unroll
        for (int k = 0; k < 9; ++k) C.R[k] = P0.R[k / 3][k % 3];
        write_pose(s_pose, C.R, C.x);
    }
    __syncthreads();
    STAMP(1);

    // the factor list: features with a map point, left then right (sliding_window.rs:519-547);
    // feature j's observation goes to LDS entry j (cam -1: no map point)
    // two features per lane per round: ids and uv loads issued together, then both
    // branchless lower_bound searches (fixed trip count) interleaved, then the p_W loads
    int mine = 0;
    const int nm = A.n_map;
    auto map_at = [&](int k) -> uint64_t { return lds_map ? s_ids[k] : A.map_ids[k]; };
    for (int j0 = tid; j0 < nf && fits; j0 += 2 * kPnpThreads) {
        const int j1 = j0 + kPnpThreads;
        const bool v1 = j1 < nf;
        int c0 = pc0, i0 = pi0, c1 = pc1, i1 = pi1;
        uint64_t id0 = pid0, id1 = pid1;
        float2 q0 = pq0, q1 = pq1;
        if (j0 != tid) {  // rounds after the first (more than 1024 features)
            feat(j0, c0, i0, id0, q0);
            if (v1) feat(j1, c1, i1, id1, q1);
        }
        int b0 = 0, b1 = 0;
        for (int len = nm; len > 1;) {
            const int half = len >> 1;
            const uint64_t m0 = map_at(b0 + half), m1 = map_at(b1 + half);
            b0 = m0 < id0 ? b0 + half : b0;
            b1 = m1 < id1 ? b1 + half : b1;
            len -= half;
        }
        bool hit0 = false, hit1 = false;
        if (nm > 0) {
            const uint64_t m0 = map_at(b0), m1 = map_at(b1);
            b0 += m0 < id0 ? 1 : 0;
            b1 += m1 < id1 ? 1 : 0;
            hit0 = b0 < nm && map_at(b0) == id0;
            hit1 = v1 && b1 < nm && map_at(b1) == id1;
        }
        s_cam[j0] = hit0 ? (int8_t)c0 : (int8_t)-1;
        if (v1) s_cam[j1] = hit1 ? (int8_t)c1 : (int8_t)-1;
        if (hit0) {
            s_uv[0][j0] = q0.x;
            s_uv[1][j0] = q0.y;
            s_idx[j0] = (int16_t)(lds_map ? b0 : j0);
            if (!lds_map) {
                s_mpw[0][j0] = A.map_pw[3 * b0];
                s_mpw[1][j0] = A.map_pw[3 * b0 + 1];
                s_mpw[2][j0] = A.map_pw[3 * b0 + 2];
            }
            ++mine;
        }
        if (hit1) {
            s_uv[0][j1] = q1.x;
            s_uv[1][j1] = q1.y;
            s_idx[j1] = (int16_t)(lds_map ? b1 : j1);
            if (!lds_map) {
                s_mpw[0][j1] = A.map_pw[3 * b1];
                s_mpw[1][j1] = A.map_pw[3 * b1 + 1];
                s_mpw[2][j1] = A.map_pw[3 * b1 + 2];
            }
            ++mine;
        }
    }
    // per-wave total (one LDS atomic per wave instead of one per lane)
    for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off);
    if (lane == 0 && mine) atomicAdd(&s_nobs, mine);
    __syncthreads();
    STAMP(2);
    int pass = 0;
    if (tid == 0) {
        C.n_obs = s_nobs;
        C.run = 1;
        if (nf > kPnpMaxFeatures) {
            C.n_obs = -1;
            C.status = LM_SKIPPED;
            C.run = 0;
        } else if (s_nobs == 0) {
            C.status = LM_SKIPPED;  // no factor: treated as a failed optimisation
            C.run = 0;
        }
    }

    while (true) {
        __syncthreads();
        if (!C.run) break;
        if (pass < 12) STAMP(3 + 2 * pass);
        if (tid < 24) {  // T_C_W = T_C_B T_B_W, one entry per thread
            const int c = tid / 12, e = tid % 12;
            const double* T = s_tcb[c];
            if (e < 9) {
                const int i = e / 3, j = e % 3;
                s_tcw[c][e] = (T[4 * i] * s_pose[j] + T[4 * i + 1] * s_pose[3 + j]) + T[4 * i + 2] * s_pose[6 + j];
            } else {
                const int i = e - 9;
                s_tcw[c][e] = ((T[4 * i] * s_pose[9] + T[4 * i + 1] * s_pose[10]) + T[4 * i + 2] * s_pose[11]) +
                              T[4 * i + 3];
            }
        }
        __syncthreads();
        // one pass at the pose in s_tcw: H, g, cost over this lane's observations (j order)
        double acc[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) acc[k] = 0.0;
#pragma unroll 1
        for (int j = tid; j < nf; j += kPnpThreads) {
            const int cam = s_cam[j];
            if (cam < 0) continue;
            const int m = s_idx[j];
            const double pW[3] = {(double)s_mpw[0][m], (double)s_mpw[1][m], (double)s_mpw[2][m]};
            const double uv[2] = {(double)s_uv[0][j], (double)s_uv[1][j]};
            double r[2], J[2][6];
            pnp_linearize_cw(pW, uv, s_tcw[cam], r, J);
            const double s2 = r[0] * r[0] + r[1] * r[1];
            double rho, w;
            huber(s2, A.huber_delta, &rho, &w);
            acc[27] += 0.5 * rho;
            const double wr0 = w * r[0], wr1 = w * r[1];
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double w0 = w * J[0][a], w1 = w * J[1][a];
#pragma unroll
                for (int c = a; c < 6; ++c) acc[utri6(a, c)] += w0 * J[0][c] + w1 * J[1][c];
                acc[21 + a] += J[0][a] * wr0 + J[1][a] * wr1;
            }
        }
        {
            const double v = wave_reduce_scatter32(acc, lane);
            if ((lane & 1) == 0 && (lane >> 1) < kRed) s_red[wv][lane >> 1] = v;
        }
        __syncthreads();
        if (tid < kRed) {
            double v = s_red[0][tid];
            for (int w = 1; w < kPnpWaves; ++w) v += s_red[w][tid];
            s_sum[tid] = v;
        }
        __syncthreads();
        if (pass < 12) STAMP(4 + 2 * pass);
        ++pass;
        if (tid == 0) pnp_control(A, &C, s_sum, s_pose);
    }
    STAMP(28);
    if (tid == 0) pnp_finish(A, C, t_entry);
    STAMP(29);
}

}  // namespace

RSVIO_DBG_READER(rsvio_dbg_pnp_stamps)

struct Pnp {
    int device = 0;
    hipStream_t stream = nullptr;      // the handle's own
    hipStream_t user = nullptr;        // rsvio_pnp_set_stream
    hipStream_t active() const { return user ? user : stream; }
    DevBuf<uint64_t> map_ids;
    DevBuf<float> map_pw;
    int n_map = 0;
    DevBuf<uint8_t> feat;            // [ids_l | ids_r | uv_l | uv_r]
    HostBuf<uint8_t> hfeat;
    HostBuf<rsvio_motion_result> hres;
    double wclk_khz = 1.0e5;
    double q0_key[16] = {};              // T_W_B_last_kf of the cached initial quaternion
    double q0[4] = {1.0, 0.0, 0.0, 0.0};

    void init(int dev) {
        device = dev;
        RSVIO_HIP(hipSetDevice(dev));
        RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        hres.alloc(1);
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
            wclk_khz = khz;
        (void)hipGetLastError();
    }
    ~Pnp() {
        if (stream) (void)hipStreamDestroy(stream);
    }
};

PnpArgs make_args(Pnp& p, const double* T_last, const double* TCB2, const rsvio_lm_cfg* cfg,
                  const rsvio_keyframe_rule* rule) {
    PnpArgs A{};
    A.map_ids = p.map_ids.p;
    A.map_pw = p.map_pw.p;
    A.n_map = p.n_map;
    std::memcpy(A.T_last, T_last, sizeof(A.T_last));
    std::memcpy(A.TCB, TCB2, sizeof(A.TCB));
    A.max_iter = cfg->max_iterations;
    A.cost_tol = cfg->cost_tolerance;
    A.param_tol = cfg->parameter_tolerance;
    A.huber_delta = cfg->huber_delta;
    A.lambda0 = cfg->lambda_init;
    A.thr_t = rule->translation_threshold;
    A.thr_r = rule->rotation_threshold;
    A.out = p.hres.p;
    A.wclk_khz = p.wclk_khz;
    // sliding_window.rs:506-517: F starts from the last keyframe's T_B_W = inv(T_W_B) with
    // q = UnitQuaternion::from_matrix(R_B_W); cached per keyframe pose
    if (std::memcmp(p.q0_key, T_last, sizeof p.q0_key) != 0) {
        double TBW[16];
        rigid_inverse(T_last, TBW);
        const double R[9] = {TBW[0], TBW[1], TBW[2], TBW[4], TBW[5], TBW[6], TBW[8], TBW[9], TBW[10]};
        rot::quat_from_matrix(R, p.q0);
        std::memcpy(p.q0_key, T_last, sizeof p.q0_key);
    }
    std::memcpy(A.q0, p.q0, sizeof A.q0);
    return A;
}

// The keyframe rule (estimator.rs:204-225) on the PnP result: T_rel = T_W_B inv(T_W_B_last_kf),
// keyframe iff |t_rel| > thr_t or |euler(from_matrix(R_rel))| > thr_r.  A failed PnP keeps
// is_keyframe = 1 and T_W_B = I (written by the kernel, estimator.rs:228-234).
void keyframe_rule(const PnpArgs& A, rsvio_motion_result* r) {
    if (r->status <= 0) return;
    double Tl_inv[16], Tr[16];
    rigid_inverse(A.T_last, Tl_inv);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += r->T_W_B[4 * i + k] * Tl_inv[4 * k + j];
            Tr[4 * i + j] = s;
        }
    r->translation_norm = std::sqrt((Tr[3] * Tr[3] + Tr[7] * Tr[7]) + Tr[11] * Tr[11]);
    const double Rr[9] = {Tr[0], Tr[1], Tr[2], Tr[4], Tr[5], Tr[6], Tr[8], Tr[9], Tr[10]};
    double q[4], Q[9];
    rot::quat_from_matrix(Rr, q);
    rot::rotation_of_quat(q, Q);
    r->rotation_norm = rot::euler_norm(Q);
    r->is_keyframe = (r->translation_norm > A.thr_t || r->rotation_norm > A.thr_r) ? 1 : 0;
}

int run_pnp(Pnp& p, const PnpArgs& A, hipStream_t stream, rsvio_motion_result* res) {
    hipLaunchKernelGGL(pnp_track_motion_kernel, dim3(1), dim3(kPnpThreads), 0, stream, A);
    RSVIO_HIP(hipGetLastError());
    RSVIO_HIP(hipStreamSynchronize(stream));
    *res = *p.hres.p;
    keyframe_rule(A, res);
    if (res->n_observations < 0) {
        set_last_error("track_motion: more than 4096 features in one frame");
        return RSVIO_ERR_CAPACITY;
    }
    return RSVIO_OK;
}

}  // namespace rsvio

struct rsvio_pnp {
    rsvio::Pnp p;
};

using rsvio::guarded;

extern "C" {

int rsvio_quat_from_matrix(const double* R, size_t n, double* q) {
    if (n && (!R || !q)) return RSVIO_ERR_INVALID_ARG;
    for (size_t i = 0; i < n; ++i) rsvio::rot::quat_from_matrix(R + 9 * i, q + 4 * i);
    return RSVIO_OK;
}

int rsvio_pnp_create(int32_t device, rsvio_pnp** out) {
    if (!out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto* h = new rsvio_pnp();
        try {
            h->p.init(device);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
        return (int)RSVIO_OK;
    });
}

void rsvio_pnp_destroy(rsvio_pnp* p) { delete p; }

int rsvio_pnp_set_stream(rsvio_pnp* h, void* stream) {
    if (!h) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        RSVIO_HIP(hipStreamSynchronize(h->p.active()));
        h->p.user = static_cast<hipStream_t>(stream);
        return (int)RSVIO_OK;
    });
}

int rsvio_pnp_set_map(rsvio_pnp* h, const uint64_t* ids, const float* p_W, int32_t n) {
    if (!h || n < 0 || (n && (!ids || !p_W))) return RSVIO_ERR_INVALID_ARG;
    for (int32_t i = 1; i < n; ++i)
        if (!(ids[i - 1] < ids[i])) {
            rsvio::set_last_error("rsvio_pnp_set_map: ids must be strictly ascending");
            return RSVIO_ERR_INVALID_ARG;
        }
    return guarded([&] {
        auto& P = h->p;
        RSVIO_HIP(hipSetDevice(P.device));
        if (P.map_ids.n < (size_t)n) {
            P.map_ids.alloc((size_t)n);
            P.map_pw.alloc((size_t)3 * n);
        }
        if (n) {
            RSVIO_HIP(hipMemcpyAsync(P.map_ids.p, ids, sizeof(uint64_t) * n, hipMemcpyHostToDevice, P.active()));
            RSVIO_HIP(hipMemcpyAsync(P.map_pw.p, p_W, sizeof(float) * 3 * n, hipMemcpyHostToDevice, P.active()));
        }
        RSVIO_HIP(hipStreamSynchronize(P.active()));
        P.n_map = n;
        return (int)RSVIO_OK;
    });
}

int rsvio_track_motion(rsvio_pnp* h, const uint64_t* ids_l, const float* uv_l, size_t n_l, const uint64_t* ids_r,
                       const float* uv_r, size_t n_r, const double* T_W_B_last_kf, const double* T_C_B2,
                       const rsvio_lm_cfg* cfg, const rsvio_keyframe_rule* rule, rsvio_motion_result* res) {
    if (!h || !T_W_B_last_kf || !T_C_B2 || !cfg || !rule || !res || (n_l && (!ids_l || !uv_l)) ||
        (n_r && (!ids_r || !uv_r)))
        return RSVIO_ERR_INVALID_ARG;
    if (n_l + n_r > (size_t)rsvio::kPnpMaxFeatures) {
        rsvio::set_last_error("track_motion: more than 4096 features in one frame");
        return RSVIO_ERR_CAPACITY;
    }
    return guarded([&] {
        auto& P = h->p;
        RSVIO_HIP(hipSetDevice(P.device));
        const size_t n = n_l + n_r, bytes = n * 16;
        if (P.feat.n < bytes || !P.feat.p) {
            const size_t cap = (size_t)rsvio::kPnpMaxFeatures * 16;
            P.feat.alloc(cap);
            P.hfeat.alloc(cap);
        }
        uint8_t* hb = P.hfeat.p;
        if (n_l) std::memcpy(hb, ids_l, 8 * n_l);
        if (n_r) std::memcpy(hb + 8 * n_l, ids_r, 8 * n_r);
        if (n_l) std::memcpy(hb + 8 * n, uv_l, 8 * n_l);
        if (n_r) std::memcpy(hb + 8 * n + 8 * n_l, uv_r, 8 * n_r);
        if (n) RSVIO_HIP(hipMemcpyAsync(P.feat.p, hb, bytes, hipMemcpyHostToDevice, P.active()));
        rsvio::PnpArgs A = rsvio::make_args(P, T_W_B_last_kf, T_C_B2, cfg, rule);
        A.ids[0] = P.feat.p;
        A.ids[1] = P.feat.p + 8 * n_l;
        A.id_stride = 8;
        A.uv[0] = reinterpret_cast<const float2*>(P.feat.p + 8 * n);
        A.uv[1] = reinterpret_cast<const float2*>(P.feat.p + 8 * n + 8 * n_l);
        A.dcount = nullptr;
        A.n[0] = (int)n_l;
        A.n[1] = (int)n_r;
        return rsvio::run_pnp(P, A, P.active(), res);
    });
}

int rsvio_track_motion_tracker(rsvio_pnp* h, rsvio_tracker* t, const double* T_W_B_last_kf, const double* T_C_B2,
                               const rsvio_lm_cfg* cfg, const rsvio_keyframe_rule* rule, rsvio_motion_result* res) {
    if (!h || !t || !T_W_B_last_kf || !T_C_B2 || !cfg || !rule || !res) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& P = h->p;
        const rsvio::TrackerView v = rsvio::tracker_view(t);
        if (!v.undist[0]) {
            rsvio::set_last_error("rsvio_track_motion_tracker: attach cameras to the tracker first");
            return (int)RSVIO_ERR_INVALID_ARG;
        }
        if (v.device != P.device) {
            rsvio::set_last_error("rsvio_track_motion_tracker: tracker and pnp handle on different devices");
            return (int)RSVIO_ERR_INVALID_ARG;
        }
        RSVIO_HIP(hipSetDevice(P.device));
        if (v.n[0] + v.n[1] > rsvio::kPnpMaxFeatures) {
            rsvio::set_last_error("track_motion: more than 4096 features in one frame");
            return (int)RSVIO_ERR_CAPACITY;
        }
        // the map upload (set_map) is ordered before this launch: it synchronised its stream.  The
        // view is the last collected frame's output slot, complete on the device (its collect
        // waited for it), so the launch goes on the handle's own stream: it runs beside a next
        // frame already submitted to the tracker's stream, which writes the other slot
        rsvio::PnpArgs A = rsvio::make_args(P, T_W_B_last_kf, T_C_B2, cfg, rule);
        A.ids[0] = reinterpret_cast<const uint8_t*>(v.out[0]);
        A.ids[1] = reinterpret_cast<const uint8_t*>(v.out[1]);
        A.id_stride = (int)sizeof(rsvio_feature);
        A.uv[0] = v.undist[0];
        A.uv[1] = v.undist[1];
        A.dcount = nullptr;
        A.n[0] = v.n[0];
        A.n[1] = v.n[1];
        return rsvio::run_pnp(P, A, P.active(), res);
    });
}

}  // extern "C"
