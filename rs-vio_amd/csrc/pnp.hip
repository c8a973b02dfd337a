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
#include "se3.hpp"

namespace rsvio {
namespace {

constexpr int kPnpThreads = 512;
constexpr int kPnpWaves = kPnpThreads / 64;
constexpr int kPnpMaxFeatures = 4096; // features per frame (both cameras), observations in LDS
constexpr int kPnpMapLds = 4096;      // map ids staged in LDS (32 KB) up to this size
constexpr int kRed = 28;          // H upper (21), g (6), cost

enum { LM_COST_TOL = 1, LM_PARAM_TOL = 2, LM_MAX_ITERS = 3, LM_TRUST_REGION = 4, LM_NUMFAIL = -1, LM_SKIPPED = -2 };

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
    double TCB[2][16];
    int max_iter;
    double cost_tol, param_tol, huber_delta, lambda0, thr_t, thr_r;
    rsvio_motion_result* out;  // pinned host memory
};

struct Ctl {
    double x[7], xt[7], H[21], g[6];
    double cost, lambda, nu, initial_cost, pred;
    int it, status, phase, run, n_obs;
};

__device__ __forceinline__ int utri6(int a, int c) { return a * 6 - (a * (a - 1)) / 2 + (c - a); }

// PnPFactor::linearize (factors.rs:527-578): p_C = R_CB (R_BW p_W + t_BW) + t_CB, r = p_C/z - obs,
// J = [jac_proj R_CB R_BW | jac_proj R_CB (-R_BW [p_W]x)]
__device__ __forceinline__ void pnp_linearize(const double pW[3], const double uv[2], const double* TCB,
                                              const Pose& P, double r[2], double J[2][6]) {
    double RCB[3][3] = {{TCB[0], TCB[1], TCB[2]}, {TCB[4], TCB[5], TCB[6]}, {TCB[8], TCB[9], TCB[10]}};
    double pB[3], pC[3], tmp[3];
    mat3vec(P.R, pW, tmp);
#pragma unroll
    for (int i = 0; i < 3; ++i) pB[i] = tmp[i] + P.t[i];
    mat3vec(RCB, pB, tmp);
    pC[0] = tmp[0] + TCB[3];
    pC[1] = tmp[1] + TCB[7];
    pC[2] = tmp[2] + TCB[11];
    r[0] = pC[0] / pC[2] - uv[0];
    r[1] = pC[1] / pC[2] - uv[1];
    const double iz = 1.0 / pC[2];
    const double iz2 = iz * iz;
    const double Jp[2][3] = {{iz, 0.0, -pC[0] * iz2}, {0.0, iz, -pC[1] * iz2}};
    double A[2][3], M[3][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A[i][j] = (Jp[i][0] * RCB[0][j] + Jp[i][1] * RCB[1][j]) + Jp[i][2] * RCB[2][j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) J[i][j] = (A[i][0] * P.R[0][j] + A[i][1] * P.R[1][j]) + A[i][2] * P.R[2][j];
    const double S[3][3] = {{0.0, -pW[2], pW[1]}, {pW[2], 0.0, -pW[0]}, {-pW[1], pW[0], 0.0}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            M[i][j] = ((-P.R[i][0]) * S[0][j] + (-P.R[i][1]) * S[1][j]) + (-P.R[i][2]) * S[2][j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) J[i][3 + j] = (A[i][0] * M[0][j] + A[i][1] * M[1][j]) + A[i][2] * M[2][j];
}

// (H + lambda I) dx = -g by Cholesky, same loop order as oracle chol_solve
__device__ bool chol6(const double* Hp, double lambda, const double* g, double* dx) {
    double A[6][6];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = a; c < 6; ++c) {
            const double v = Hp[utri6(a, c)];
            A[a][c] = v;
            A[c][a] = v;
        }
#pragma unroll
    for (int a = 0; a < 6; ++a) A[a][a] += lambda;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= A[j][k] * A[j][k];
        if (!(d > 0.0) || !isfinite(d)) return false;
        const double ljj = sqrt(d);
        A[j][j] = ljj;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double s = A[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) s -= A[i][k] * A[j][k];
            A[i][j] = s / ljj;
        }
    }
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double s = -g[i];
#pragma unroll
        for (int k = 0; k < i; ++k) s -= A[i][k] * x[k];
        x[i] = s / A[i][i];
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double s = x[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) s -= A[k][i] * x[k];
        x[i] = s / A[i][i];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) dx[i] = x[i];
    return true;
}

__device__ __forceinline__ void write_pose(double* s_pose, const double* x7) {
    const Pose P = pose_from7(x7);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) s_pose[3 * i + j] = P.R[i][j];
        s_pose[9 + i] = P.t[i];
    }
}

// Lane 0 between passes: consume the pass in s_sum, then either set up the next pass (run = 1)
// or finish (run = 0).  Mirrors oracle orc_track_motion's loop step for step.
__device__ void pnp_control(const PnpArgs& A, Ctl& C, const double* s_sum, double* s_pose) {
    bool done = false;
    if (C.phase == 0) {
#pragma unroll
        for (int k = 0; k < 21; ++k) C.H[k] = s_sum[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) C.g[k] = s_sum[21 + k];
        C.cost = s_sum[27];
        C.initial_cost = C.cost;
        C.phase = 1;
    } else {
        const double new_cost = s_sum[27];
        const double rho = (C.cost - new_cost) / C.pred;
        if (isfinite(new_cost) && rho > 0.0) {
            const double dcost = C.cost - new_cost;
#pragma unroll
            for (int k = 0; k < 7; ++k) C.x[k] = C.xt[k];
#pragma unroll
            for (int k = 0; k < 21; ++k) C.H[k] = s_sum[k];
#pragma unroll
            for (int k = 0; k < 6; ++k) C.g[k] = s_sum[21 + k];
            const double f = 2.0 * rho - 1.0;
            C.lambda *= fmax(1.0 / 3.0, 1.0 - f * f * f);
            C.nu = 2.0;
            C.cost = new_cost;
            if (dcost <= A.cost_tol * (C.cost + dcost)) {
                C.status = LM_COST_TOL;
                done = true;
            }
        } else {
            C.lambda *= C.nu;
            C.nu *= 2.0;
            if (C.lambda > 1e32) {
                C.status = LM_TRUST_REGION;
                done = true;
            }
        }
    }
    while (!done) {
        if (C.it >= A.max_iter) {
            C.status = LM_MAX_ITERS;
            break;
        }
        C.it += 1;
        if (!isfinite(C.cost)) {
            C.status = LM_NUMFAIL;
            break;
        }
        double dx[6];
        if (!chol6(C.H, C.lambda, C.g, dx)) {
            C.lambda *= C.nu;
            C.nu *= 2.0;
            if (C.lambda > 1e32) {
                C.status = LM_TRUST_REGION;
                break;
            }
            continue;
        }
        double dx2 = 0.0, gdx = 0.0, x2 = 0.0;
        for (int k = 0; k < 6; ++k) {
            dx2 += dx[k] * dx[k];
            gdx += C.g[k] * dx[k];
        }
        for (int k = 0; k < 7; ++k) x2 += C.x[k] * C.x[k];
        if (sqrt(dx2) <= A.param_tol * (sqrt(x2) + A.param_tol)) {
            C.status = LM_PARAM_TOL;
            break;
        }
        se3_plus(C.x, dx, C.xt);
        C.pred = 0.5 * (C.lambda * dx2 - gdx);
        write_pose(s_pose, C.xt);
        C.run = 1;
        return;
    }
    C.run = 0;
}

// nalgebra Rotation3::euler_angles (roll, pitch, yaw) of a rotation matrix (estimator.rs:207-212)
__device__ __forceinline__ double euler_norm(const double R[3][3]) {
    double roll, pitch, yaw;
    if (fabs(R[2][0]) < 1.0) {
        pitch = -asin(R[2][0]);
        const double c = cos(pitch);
        roll = atan2(R[2][1] / c, R[2][2] / c);
        yaw = atan2(R[1][0] / c, R[0][0] / c);
    } else if (R[2][0] <= -1.0) {
        roll = atan2(R[0][1], R[0][2]);
        pitch = M_PI_2;
        yaw = 0.0;
    } else {
        roll = -atan2(-R[0][1], -R[0][2]);
        pitch = -M_PI_2;
        yaw = 0.0;
    }
    return sqrt((roll * roll + pitch * pitch) + yaw * yaw);
}

__device__ void pnp_finish(const PnpArgs& A, const Ctl& C) {
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
        double TBW[16], Tl_inv[16];
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) TBW[4 * i + j] = P.R[i][j];
            TBW[4 * i + 3] = P.t[i];
        }
        TBW[12] = 0.0; TBW[13] = 0.0; TBW[14] = 0.0; TBW[15] = 1.0;
        rigid_inverse(TBW, r.T_W_B);
        rigid_inverse(A.T_last, Tl_inv);
        // T_rel = T_W_B * inv(T_W_B_last_kf) (estimator.rs:205)
        double Tr[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double s = 0.0;
                for (int k = 0; k < 4; ++k) s += r.T_W_B[4 * i + k] * Tl_inv[4 * k + j];
                Tr[4 * i + j] = s;
            }
        r.translation_norm = sqrt((Tr[3] * Tr[3] + Tr[7] * Tr[7]) + Tr[11] * Tr[11]);
        const double Rr[9] = {Tr[0], Tr[1], Tr[2], Tr[4], Tr[5], Tr[6], Tr[8], Tr[9], Tr[10]};
        double q7[7] = {0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0};
        quat_from_rot(Rr, q7 + 3);
        const Pose Q = pose_from7(q7);  // UnitQuaternion -> rotation matrix
        r.rotation_norm = euler_norm(Q.R);
        r.is_keyframe = (r.translation_norm > A.thr_t || r.rotation_norm > A.thr_r) ? 1 : 0;
    } else {
        for (int k = 0; k < 16; ++k) r.T_W_B[k] = (k % 5 == 0) ? 1.0 : 0.0;
        r.is_keyframe = 1;
    }
    *A.out = r;
}

__global__ __launch_bounds__(kPnpThreads) void pnp_track_motion_kernel(PnpArgs A) {
    __shared__ uint64_t s_ids[kPnpMapLds];
    __shared__ float s_obs[5][kPnpMaxFeatures];  // p_W (3), undistorted uv (2) per feature
    __shared__ int8_t s_cam[kPnpMaxFeatures];
    __shared__ double s_red[kPnpWaves][kRed];
    __shared__ double s_sum[kRed];
    __shared__ double s_pose[12];
    __shared__ double s_tcb[2][16];
    __shared__ Ctl C;
    __shared__ int s_nobs;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n0 = A.dcount ? A.dcount[0] : A.n[0];
    const int n1 = A.dcount ? A.dcount[1] : A.n[1];
    const int nf = n0 + n1;
    const bool lds_map = A.n_map <= kPnpMapLds;
    if (lds_map)
        for (int i = tid; i < A.n_map; i += kPnpThreads) s_ids[i] = A.map_ids[i];
    if (tid < 32) s_tcb[tid >> 4][tid & 15] = A.TCB[tid >> 4][tid & 15];
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
        const double R[9] = {TBW[0], TBW[1], TBW[2], TBW[4], TBW[5], TBW[6], TBW[8], TBW[9], TBW[10]};
        C.x[0] = TBW[3];
        C.x[1] = TBW[7];
        C.x[2] = TBW[11];
        quat_from_rot(R, C.x + 3);
        write_pose(s_pose, C.x);
    }
    __syncthreads();

    // the factor list: features with a map point, left then right (sliding_window.rs:519-547);
    // feature j's observation goes to LDS entry j (cam -1: no map point)
    int mine = 0;
    for (int j = tid; j < nf && nf <= kPnpMaxFeatures; j += kPnpThreads) {
        const int c = j < n0 ? 0 : 1;
        const int i = c == 0 ? j : j - n0;
        const uint64_t id = *reinterpret_cast<const uint64_t*>(A.ids[c] + (size_t)i * A.id_stride);
        int lo = 0, hi = A.n_map;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const uint64_t v = lds_map ? s_ids[mid] : A.map_ids[mid];
            if (v < id) lo = mid + 1; else hi = mid;
        }
        const bool hit = lo < A.n_map && (lds_map ? s_ids[lo] : A.map_ids[lo]) == id;
        s_cam[j] = hit ? (int8_t)c : (int8_t)-1;
        if (hit) {
            s_obs[0][j] = A.map_pw[3 * lo];
            s_obs[1][j] = A.map_pw[3 * lo + 1];
            s_obs[2][j] = A.map_pw[3 * lo + 2];
            const float2 q = A.uv[c][i];
            s_obs[3][j] = q.x;
            s_obs[4][j] = q.y;
            ++mine;
        }
    }
    if (mine) atomicAdd(&s_nobs, mine);
    __syncthreads();
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
        // one pass at s_pose: H, g, cost over this lane's observations (slot order)
        Pose P;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) P.R[i][j] = s_pose[3 * i + j];
            P.t[i] = s_pose[9 + i];
        }
        double acc[kRed];
#pragma unroll
        for (int k = 0; k < kRed; ++k) acc[k] = 0.0;
#pragma unroll 1
        for (int j = tid; j < nf; j += kPnpThreads) {
            const int cam = s_cam[j];
            if (cam < 0) continue;
            const double pW[3] = {(double)s_obs[0][j], (double)s_obs[1][j], (double)s_obs[2][j]};
            const double uv[2] = {(double)s_obs[3][j], (double)s_obs[4][j]};
            double r[2], J[2][6];
            pnp_linearize(pW, uv, s_tcb[cam], P, r, J);
            const double s2 = r[0] * r[0] + r[1] * r[1];
            double rho, w;
            huber(s2, A.huber_delta, &rho, &w);
            acc[27] += 0.5 * rho;
            const double wr0 = w * r[0], wr1 = w * r[1];
#pragma unroll
            for (int a = 0; a < 6; ++a) {
#pragma unroll
                for (int c = a; c < 6; ++c) acc[utri6(a, c)] += w * (J[0][a] * J[0][c] + J[1][a] * J[1][c]);
                acc[21 + a] += J[0][a] * wr0 + J[1][a] * wr1;
            }
        }
#pragma unroll
        for (int k = 0; k < kRed; ++k) {
            const double v = wave_sum_det(acc[k]);
            if (lane == 0) s_red[wv][k] = v;
        }
        __syncthreads();
        if (tid < kRed) {
            double v = s_red[0][tid];
            for (int w = 1; w < kPnpWaves; ++w) v += s_red[w][tid];
            s_sum[tid] = v;
        }
        __syncthreads();
        if (tid == 0) pnp_control(A, C, s_sum, s_pose);
    }
    if (tid == 0) pnp_finish(A, C);
}

}  // namespace

struct Pnp {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf<uint64_t> map_ids;
    DevBuf<float> map_pw;
    int n_map = 0;
    DevBuf<uint8_t> feat;            // [ids_l | ids_r | uv_l | uv_r]
    HostBuf<uint8_t> hfeat;
    HostBuf<rsvio_motion_result> hres;

    void init(int dev) {
        device = dev;
        RSVIO_HIP(hipSetDevice(dev));
        RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        hres.alloc(1);
    }
    ~Pnp() {
        if (stream) (void)hipStreamDestroy(stream);
    }
};

PnpArgs make_args(const Pnp& p, const double* T_last, const double* TCB2, const rsvio_lm_cfg* cfg,
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
    return A;
}

int run_pnp(Pnp& p, const PnpArgs& A, hipStream_t stream, rsvio_motion_result* res) {
    hipLaunchKernelGGL(pnp_track_motion_kernel, dim3(1), dim3(kPnpThreads), 0, stream, A);
    RSVIO_HIP(hipGetLastError());
    RSVIO_HIP(hipStreamSynchronize(stream));
    *res = *p.hres.p;
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
            RSVIO_HIP(hipMemcpyAsync(P.map_ids.p, ids, sizeof(uint64_t) * n, hipMemcpyHostToDevice, P.stream));
            RSVIO_HIP(hipMemcpyAsync(P.map_pw.p, p_W, sizeof(float) * 3 * n, hipMemcpyHostToDevice, P.stream));
        }
        RSVIO_HIP(hipStreamSynchronize(P.stream));
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
        if (n) RSVIO_HIP(hipMemcpyAsync(P.feat.p, hb, bytes, hipMemcpyHostToDevice, P.stream));
        rsvio::PnpArgs A = rsvio::make_args(P, T_W_B_last_kf, T_C_B2, cfg, rule);
        A.ids[0] = P.feat.p;
        A.ids[1] = P.feat.p + 8 * n_l;
        A.id_stride = 8;
        A.uv[0] = reinterpret_cast<const float2*>(P.feat.p + 8 * n);
        A.uv[1] = reinterpret_cast<const float2*>(P.feat.p + 8 * n + 8 * n_l);
        A.dcount = nullptr;
        A.n[0] = (int)n_l;
        A.n[1] = (int)n_r;
        return rsvio::run_pnp(P, A, P.stream, res);
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
        // the map upload (set_map) is ordered before this launch: it synchronised P.stream
        rsvio::PnpArgs A = rsvio::make_args(P, T_W_B_last_kf, T_C_B2, cfg, rule);
        A.ids[0] = reinterpret_cast<const uint8_t*>(v.out[0]);
        A.ids[1] = reinterpret_cast<const uint8_t*>(v.out[1]);
        A.id_stride = (int)sizeof(rsvio_feature);
        A.uv[0] = v.undist[0];
        A.uv[1] = v.undist[1];
        A.dcount = v.counts;
        return rsvio::run_pnp(P, A, v.stream, res);
    });
}

}  // extern "C"
