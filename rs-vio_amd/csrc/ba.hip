// ba.hip -- HP-B: sliding-window bundle adjustment on gfx950 (f64), landmark-sharded over ranks.
//
// Replaces SlidingWindow::optimize's solver call (src/estimator/sliding_window.rs:159-381):
// BundleAdjustmentFactor::linearize (src/optimization/factors.rs:350-447) for every observation,
// Huber(2.0) (sliding_window.rs:295-296), and apex-solver's LevenbergMarquardt with
// SparseSchurComplement (sliding_window.rs:126-135,325) -- restated as DESIGN.md "BA LM".
//
// Layout (landmark-major, built once per problem on the host, CSR):
//   obs   sorted by (landmark, keyframe, camera)
//   slot  = (landmark, keyframe) group of 1-2 observations; slots sorted like obs
//   pairs = for every upper-triangular camera block (fa <= fb), the (slot_a, slot_b) pairs of
//           landmarks that both keyframes observe (ascending landmark)
// Per LM iteration (all on one HIP stream, one status read-back):
//   K4a ba_slot_linearize   thread / slot     residual, Jacobian, Huber; V, g_p, W, U, g_c slot sums
//   K4b ba_landmark_eliminate thread / landmark (V + lambda I)^-1, Y = W V^-1, Y g_p
//   K4c ba_schur_blocks     workgroup / 6x6 camera block: S = U + lambda I - sum Y W^T, b, cost
//   [RCCL all-reduce of S, b, g_c, cost when sharded]
//   K5  ba_dense_solve      1 workgroup: Cholesky of the 6(W-1) camera system in LDS, SE3 (+) trial poses
//   K6a ba_backsub_cost     thread / landmark: dp = V^-1 (-g_p - W^T dc), trial point, trial cost
//   K6b ba_reduce_trial     1 workgroup: fixed-order tree sums of the per-landmark partials
//   [RCCL all-reduce of the 5 trial scalars when sharded]
//   K7  ba_lm_decide        1 workgroup: gain ratio, accept/reject, lambda update, termination
// Every reduction has a fixed order (no floating-point atomics): results are run-to-run identical.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "common.hpp"

namespace rsvio {

namespace {

constexpr int kMaxFree = 20;           // 6 * 20 = 120-dim camera system in LDS
constexpr int kSlotFields = 55;        // V6 gp3 W18 U21 gc6 cost1
enum { F_V = 0, F_GP = 6, F_W = 9, F_U = 27, F_GC = 48, F_COST = 54 };

struct Mat4 {
    double m[16];
};

struct Pose {
    double R[3][3];
    double t[3];
};

// nalgebra UnitQuaternion::to_rotation_matrix after normalisation (apex SE3::from)
__device__ __forceinline__ Pose pose_from7(const double* p7) {
    double w = p7[3], x = p7[4], y = p7[5], z = p7[6];
    double n = sqrt(w * w + x * x + y * y + z * z);
    w /= n; x /= n; y /= n; z /= n;
    double ww = w * w, xx = x * x, yy = y * y, zz = z * z;
    double xy = x * y * 2.0, wz = w * z * 2.0, wy = w * y * 2.0;
    double xz = x * z * 2.0, yz = y * z * 2.0, wx = w * x * 2.0;
    Pose P;
    P.R[0][0] = ww + xx - yy - zz; P.R[0][1] = xy - wz;           P.R[0][2] = wy + xz;
    P.R[1][0] = wz + xy;           P.R[1][1] = ww - xx + yy - zz; P.R[1][2] = yz - wx;
    P.R[2][0] = xz - wy;           P.R[2][1] = wx + yz;           P.R[2][2] = ww - xx - yy + zz;
    P.t[0] = p7[0]; P.t[1] = p7[1]; P.t[2] = p7[2];
    return P;
}

__device__ __forceinline__ void mat3vec(const double R[3][3], const double* v, double* out) {
#pragma unroll
    for (int i = 0; i < 3; ++i) out[i] = (R[i][0] * v[0] + R[i][1] * v[1]) + R[i][2] * v[2];
}

// factors.rs:350-447 -- residual and the 2x9 Jacobian [dp_W | dt | dw]; false on cheirality failure
__device__ __forceinline__ bool linearize(const double* pW, const Pose& P, const double* TCB, const double* uv,
                                          double r[2], double J[2][9], bool want_j) {
    double RCB[3][3] = {{TCB[0], TCB[1], TCB[2]}, {TCB[4], TCB[5], TCB[6]}, {TCB[8], TCB[9], TCB[10]}};
    double pB[3], pC[3], tmp[3];
    mat3vec(P.R, pW, tmp);
#pragma unroll
    for (int i = 0; i < 3; ++i) pB[i] = tmp[i] + P.t[i];
    mat3vec(RCB, pB, tmp);
    pC[0] = tmp[0] + TCB[3];
    pC[1] = tmp[1] + TCB[7];
    pC[2] = tmp[2] + TCB[11];
    if (pC[2] <= 0.0) {
        r[0] = 1e6;
        r[1] = 1e6;
        if (want_j)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 9; ++b) J[a][b] = 0.0;
        return false;
    }
    r[0] = pC[0] / pC[2] - uv[0];
    r[1] = pC[1] / pC[2] - uv[1];
    if (!want_j) return true;
    double iz = 1.0 / pC[2];
    double iz2 = iz * iz;
    double Jp[2][3] = {{iz, 0.0, -pC[0] * iz2}, {0.0, iz, -pC[1] * iz2}};
    double A[2][3], M[3][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A[i][j] = (Jp[i][0] * RCB[0][j] + Jp[i][1] * RCB[1][j]) + Jp[i][2] * RCB[2][j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double v = (A[i][0] * P.R[0][j] + A[i][1] * P.R[1][j]) + A[i][2] * P.R[2][j];
            J[i][j] = v;
            J[i][3 + j] = v;
        }
    double S[3][3] = {{0.0, -pW[2], pW[1]}, {pW[2], 0.0, -pW[0]}, {-pW[1], pW[0], 0.0}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            M[i][j] = ((-P.R[i][0]) * S[0][j] + (-P.R[i][1]) * S[1][j]) + (-P.R[i][2]) * S[2][j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) J[i][6 + j] = (A[i][0] * M[0][j] + A[i][1] * M[1][j]) + A[i][2] * M[2][j];
    return true;
}

__device__ __forceinline__ void huber(double s, double d, double* rho, double* w) {
    double d2 = d * d;
    if (s <= d2) {
        *rho = s;
        *w = 1.0;
    } else {
        double rs = sqrt(s);
        *rho = 2.0 * d * rs - d2;
        *w = d / rs;
    }
}

__device__ __forceinline__ bool inv3(const double A[3][3], double X[3][3]) {
    double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
    double c01 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
    double c02 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
    double det = A[0][0] * c00 + A[0][1] * c01 + A[0][2] * c02;
    if (!(det > 0.0) || !isfinite(det)) return false;
    double id = 1.0 / det;
    X[0][0] = c00 * id;
    X[1][0] = c01 * id;
    X[2][0] = c02 * id;
    X[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) * id;
    X[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) * id;
    X[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) * id;
    X[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) * id;
    X[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) * id;
    X[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) * id;
    return true;
}

// T (+) delta = T * Exp([rho; theta]) (same formula as oracle orc_se3_plus)
__device__ void se3_plus(const double* p7, const double* d, double* out) {
    const double* rho = d;
    const double* om = d + 3;
    double th2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
    double th = sqrt(th2);
    double qd[4], A, Bc;
    if (th < 1e-8) {
        qd[0] = 1.0; qd[1] = 0.5 * om[0]; qd[2] = 0.5 * om[1]; qd[3] = 0.5 * om[2];
        A = 0.5 - th2 / 24.0;
        Bc = 1.0 / 6.0 - th2 / 120.0;
    } else {
        double s = sin(0.5 * th) / th;
        qd[0] = cos(0.5 * th); qd[1] = s * om[0]; qd[2] = s * om[1]; qd[3] = s * om[2];
        A = (1.0 - cos(th)) / th2;
        Bc = (th - sin(th)) / (th2 * th);
    }
    double wx[3] = {om[1] * rho[2] - om[2] * rho[1], om[2] * rho[0] - om[0] * rho[2], om[0] * rho[1] - om[1] * rho[0]};
    double wwx[3] = {om[1] * wx[2] - om[2] * wx[1], om[2] * wx[0] - om[0] * wx[2], om[0] * wx[1] - om[1] * wx[0]};
    double td[3];
    for (int i = 0; i < 3; ++i) td[i] = rho[i] + A * wx[i] + Bc * wwx[i];
    Pose P = pose_from7(p7);
    double Rt[3];
    mat3vec(P.R, td, Rt);
    out[0] = p7[0] + Rt[0];
    out[1] = p7[1] + Rt[1];
    out[2] = p7[2] + Rt[2];
    double w0 = p7[3], x0 = p7[4], y0 = p7[5], z0 = p7[6];
    double qn[4] = {w0 * qd[0] - x0 * qd[1] - y0 * qd[2] - z0 * qd[3], w0 * qd[1] + x0 * qd[0] + y0 * qd[3] - z0 * qd[2],
                    w0 * qd[2] - x0 * qd[3] + y0 * qd[0] + z0 * qd[1], w0 * qd[3] + x0 * qd[2] - y0 * qd[1] + z0 * qd[0]};
    double nn = sqrt(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int i = 0; i < 4; ++i) out[3 + i] = qn[i] / nn;
}

// LM bookkeeping that lives on the device (read back once per iteration)
struct LmState {
    double lambda, nu, cost, initial_cost;
    double dc2, gcdc;                    // from K5
    double new_cost, dp2, gpdp, x2p;     // from K6b (after the all-reduce)
    int iter, status, done, solve_ok;
    int accepted;
};

struct Geometry {
    int n_kf, n_free, n_lm, n_obs, n_slot, n_pb;
    Mat4 TCB[2];
    double huber_delta;
};

// --------------------------------------------------------------------------------------
// K4a: per slot (landmark, keyframe): linearise its observations
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ba_slot_linearize(Geometry G, const double* __restrict__ pose7,
                                                         const double* __restrict__ pW, const int* __restrict__ slot_lm,
                                                         const int* __restrict__ slot_kf, const int* __restrict__ slot_obs,
                                                         const uint8_t* __restrict__ obs_cam,
                                                         const double* __restrict__ obs_uv, const int* __restrict__ free_idx,
                                                         double* __restrict__ sf, const LmState* __restrict__ st) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= G.n_slot || st->done) return;
    const int l = slot_lm[s], kf = slot_kf[s];
    const bool fr = free_idx[kf] >= 0;
    const Pose P = pose_from7(pose7 + 7 * kf);
    double p[3] = {pW[3 * l], pW[3 * l + 1], pW[3 * l + 2]};
    double V[6] = {0, 0, 0, 0, 0, 0}, gp[3] = {0, 0, 0}, W[18], U[21], gc[6], cost = 0.0;
#pragma unroll
    for (int i = 0; i < 18; ++i) W[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 21; ++i) U[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) gc[i] = 0.0;
    for (int o = slot_obs[s]; o < slot_obs[s + 1]; ++o) {
        double r[2], J[2][9];
        linearize(p, P, G.TCB[obs_cam[o]].m, obs_uv + 2 * o, r, J, true);
        double sq = r[0] * r[0] + r[1] * r[1], rho, w;
        huber(sq, G.huber_delta, &rho, &w);
        cost += 0.5 * rho;
        const double wr0 = w * r[0], wr1 = w * r[1];
        int k = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
#pragma unroll
            for (int c = a; c < 3; ++c) V[k++] += w * (J[0][a] * J[0][c] + J[1][a] * J[1][c]);
            gp[a] += J[0][a] * wr0 + J[1][a] * wr1;
        }
        if (fr) {
            int u = 0;
#pragma unroll
            for (int a = 0; a < 6; ++a) {
#pragma unroll
                for (int c = 0; c < 3; ++c) W[a * 3 + c] += w * (J[0][3 + a] * J[0][c] + J[1][3 + a] * J[1][c]);
#pragma unroll
                for (int c = a; c < 6; ++c) U[u++] += w * (J[0][3 + a] * J[0][3 + c] + J[1][3 + a] * J[1][3 + c]);
                gc[a] += J[0][3 + a] * wr0 + J[1][3 + a] * wr1;
            }
        }
    }
    const int n = G.n_slot;
#pragma unroll
    for (int i = 0; i < 6; ++i) sf[(F_V + i) * n + s] = V[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) sf[(F_GP + i) * n + s] = gp[i];
#pragma unroll
    for (int i = 0; i < 18; ++i) sf[(F_W + i) * n + s] = W[i];
#pragma unroll
    for (int i = 0; i < 21; ++i) sf[(F_U + i) * n + s] = U[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) sf[(F_GC + i) * n + s] = gc[i];
    sf[F_COST * n + s] = cost;
}

// --------------------------------------------------------------------------------------
// K4b: per landmark: V* = V + lambda I, V*^-1, Y_s = W_s V*^-1, Y_s g_p
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ba_landmark_eliminate(Geometry G, const int* __restrict__ lm_slot,
                                                             const int* __restrict__ slot_kf, const int* __restrict__ free_idx,
                                                             const double* __restrict__ sf, double* __restrict__ Y,
                                                             double* __restrict__ yg, double* __restrict__ lmd,
                                                             LmState* __restrict__ st) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= G.n_lm || st->done) return;
    const int n = G.n_slot;
    const double lambda = st->lambda;
    double V[6] = {0, 0, 0, 0, 0, 0}, gp[3] = {0, 0, 0}, cost = 0.0;
    const int s0 = lm_slot[l], s1 = lm_slot[l + 1];
    for (int s = s0; s < s1; ++s) {
#pragma unroll
        for (int i = 0; i < 6; ++i) V[i] += sf[(F_V + i) * n + s];
#pragma unroll
        for (int i = 0; i < 3; ++i) gp[i] += sf[(F_GP + i) * n + s];
        cost += sf[F_COST * n + s];
    }
    double A[3][3] = {{V[0] + lambda, V[1], V[2]}, {V[1], V[3] + lambda, V[4]}, {V[2], V[4], V[5] + lambda}};
    double Vi[3][3];
    bool ok = inv3(A, Vi);
    if (!ok)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c) Vi[a][c] = 0.0;
    for (int s = s0; s < s1; ++s) {
        if (free_idx[slot_kf[s]] < 0) continue;
        double Ys[18];
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                Ys[a * 3 + c] = (sf[(F_W + a * 3) * n + s] * Vi[0][c] + sf[(F_W + a * 3 + 1) * n + s] * Vi[1][c]) +
                                sf[(F_W + a * 3 + 2) * n + s] * Vi[2][c];
#pragma unroll
        for (int i = 0; i < 18; ++i) Y[i * n + s] = Ys[i];
#pragma unroll
        for (int a = 0; a < 6; ++a)
            yg[a * n + s] = (Ys[a * 3] * gp[0] + Ys[a * 3 + 1] * gp[1]) + Ys[a * 3 + 2] * gp[2];
    }
    const int m = G.n_lm;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c) lmd[(a * 3 + c) * m + l] = Vi[a][c];
#pragma unroll
    for (int a = 0; a < 3; ++a) lmd[(9 + a) * m + l] = gp[a];
    lmd[12 * m + l] = cost;
    lmd[13 * m + l] = ok ? 0.0 : 1.0;
}

// fixed-order tree reduction of `nv` doubles held by every thread of a 256-thread block
template <int NV>
__device__ __forceinline__ void block_reduce(double (&v)[NV], double* sh) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) sh[i * 256 + tid] = v[i];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off)
#pragma unroll
            for (int i = 0; i < NV; ++i) sh[i * 256 + tid] += sh[i * 256 + tid + off];
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = sh[i * 256];
    __syncthreads();
}

// --------------------------------------------------------------------------------------
// K4c: one workgroup per upper-triangular 6x6 camera block (fa <= fb)
//   S_ab = [a == b] (sum U_s + lambda I) - sum_pairs Y_sa W_sb^T
//   diagonal blocks also produce g_c (sum of slot g_c) and b = -g_c + sum Y g_p;
//   block 0 also sums the per-landmark costs.
// out: [n_pb * 36 S blocks][n_free * 6 b][n_free * 6 g_c][cost]
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ba_schur_blocks(Geometry G, const int* __restrict__ pb_fa,
                                                       const int* __restrict__ pb_fb, const int* __restrict__ pair_ptr,
                                                       const int* __restrict__ pair_a, const int* __restrict__ pair_b,
                                                       const double* __restrict__ sf, const double* __restrict__ Y,
                                                       const double* __restrict__ yg, const double* __restrict__ lmd,
                                                       double* __restrict__ out, const LmState* __restrict__ st,
                                                       int lambda_owner) {
    __shared__ double sh[12 * 256];
    if (st->done) return;
    const int pb = blockIdx.x;
    const int n = G.n_slot;
    const int tid = threadIdx.x;
    if (pb == G.n_pb) {  // cost block (+ count of landmarks whose V + lambda I is not invertible)
        double c[2] = {0.0, 0.0};
        for (int l = tid; l < G.n_lm; l += 256) {
            c[0] += lmd[12 * G.n_lm + l];
            c[1] += lmd[13 * G.n_lm + l];
        }
        block_reduce<2>(c, sh);
        if (tid == 0) {
            out[G.n_pb * 36 + 12 * G.n_free] = c[0];
            out[G.n_pb * 36 + 12 * G.n_free + 1] = c[1];
        }
        return;
    }
    const int fa = pb_fa[pb], fb = pb_fb[pb];
    const bool diag = fa == fb;
    double acc[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) acc[i] = 0.0;
    for (int p = pair_ptr[pb] + tid; p < pair_ptr[pb + 1]; p += 256) {
        const int sa = pair_a[p], sb = pair_b[p];
        double Ya[18], Wb[18];
#pragma unroll
        for (int i = 0; i < 18; ++i) {
            Ya[i] = Y[i * n + sa];
            Wb[i] = sf[(F_W + i) * n + sb];
        }
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int c = 0; c < 6; ++c)
                acc[a * 6 + c] -= (Ya[a * 3] * Wb[c * 3] + Ya[a * 3 + 1] * Wb[c * 3 + 1]) + Ya[a * 3 + 2] * Wb[c * 3 + 2];
        if (diag) {
            int u = 0;
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int c = a; c < 6; ++c) {
                    double v = sf[(F_U + u) * n + sa];
                    acc[a * 6 + c] += v;
                    if (c != a) acc[c * 6 + a] += v;
                    ++u;
                }
        }
    }
    // fixed-order reduction of 36 values in three chunks of 12 (LDS = 12 * 256 doubles per pass)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        double v[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) v[i] = acc[ch * 12 + i];
        block_reduce<12>(v, sh);
#pragma unroll
        for (int i = 0; i < 12; ++i) acc[ch * 12 + i] = v[i];
    }
    // lambda I on the camera diagonal is added by one rank only (the blocks are summed over ranks)
    if (tid < 36) out[pb * 36 + tid] = acc[tid] + ((diag && lambda_owner && (tid / 6 == tid % 6)) ? st->lambda : 0.0);
    if (diag) {
        double g[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) g[i] = 0.0;
        for (int p = pair_ptr[pb] + tid; p < pair_ptr[pb + 1]; p += 256) {
            const int s = pair_a[p];
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                g[a] += sf[(F_GC + a) * n + s];
                g[6 + a] += yg[a * n + s];
            }
        }
        block_reduce<12>(g, sh);
        if (tid < 6) {
            out[G.n_pb * 36 + 6 * fa + tid] = -g[tid] + g[6 + tid];           // b
            out[G.n_pb * 36 + 6 * G.n_free + 6 * fa + tid] = g[tid];          // g_c
        }
    }
}

// --------------------------------------------------------------------------------------
// K5: dense camera solve (one workgroup), trial poses
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ba_dense_solve(Geometry G, const int* __restrict__ pb_fa,
                                                      const int* __restrict__ pb_fb, const double* __restrict__ sys,
                                                      const double* __restrict__ pose7, const int* __restrict__ free_idx,
                                                      double* __restrict__ pose7_trial, double* __restrict__ dc_out,
                                                      LmState* __restrict__ st) {
    __shared__ double A[6 * kMaxFree * 6 * kMaxFree];
    __shared__ double x[6 * kMaxFree];
    __shared__ int fail;
    __shared__ double red[2 * 256];
    if (st->done) return;
    const int n = 6 * G.n_free;
    const int tid = threadIdx.x;
    if (tid == 0) fail = 0;
    for (int pb = 0; pb < G.n_pb; ++pb) {
        const int fa = pb_fa[pb], fb = pb_fb[pb];
        for (int e = tid; e < 36; e += 256) {
            const int a = e / 6, c = e % 6;
            const double v = sys[pb * 36 + e];
            A[(6 * fa + a) * n + 6 * fb + c] = v;
            A[(6 * fb + c) * n + 6 * fa + a] = v;
        }
    }
    for (int i = tid; i < n; i += 256) x[i] = sys[G.n_pb * 36 + i];
    if (tid == 0 && sys[G.n_pb * 36 + 12 * G.n_free + 1] != 0.0) fail = 1;  // a landmark block was singular
    __syncthreads();
    // right-looking Cholesky, lower triangle in A
    for (int j = 0; j < n; ++j) {
        if (tid == 0) {
            const double d = A[j * n + j];
            if (!(d > 0.0) || !isfinite(d)) fail = 1;
            A[j * n + j] = sqrt(d);
        }
        __syncthreads();
        if (fail) break;
        const double ljj = A[j * n + j];
        for (int i = j + 1 + tid; i < n; i += 256) A[i * n + j] /= ljj;
        __syncthreads();
        const int m = n - j - 1;
        for (int e = tid; e < m * m; e += 256) {
            const int i = j + 1 + e / m, k = j + 1 + e % m;
            if (k <= i) A[i * n + k] -= A[i * n + j] * A[k * n + j];
        }
        __syncthreads();
    }
    if (fail) {
        if (tid == 0) {
            st->solve_ok = 0;
            st->dc2 = 0.0;
            st->gcdc = 0.0;
        }
        return;
    }
    // forward L y = b (column oriented), then backward L^T x = y
    for (int j = 0; j < n; ++j) {
        if (tid == 0) x[j] /= A[j * n + j];
        __syncthreads();
        for (int i = j + 1 + tid; i < n; i += 256) x[i] -= A[i * n + j] * x[j];
        __syncthreads();
    }
    for (int j = n - 1; j >= 0; --j) {
        if (tid == 0) x[j] /= A[j * n + j];
        __syncthreads();
        for (int i = tid; i < j; i += 256) x[i] -= A[j * n + i] * x[j];
        __syncthreads();
    }
    for (int i = tid; i < n; i += 256) dc_out[i] = x[i];
    // dc^2 and g_c . dc
    double v0 = 0.0, v1 = 0.0;
    const double* gc = sys + G.n_pb * 36 + n;
    for (int i = tid; i < n; i += 256) {
        v0 += x[i] * x[i];
        v1 += gc[i] * x[i];
    }
    red[tid] = v0;
    red[256 + tid] = v1;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off) {
            red[tid] += red[tid + off];
            red[256 + tid] += red[256 + tid + off];
        }
        __syncthreads();
    }
    for (int k = tid; k < G.n_kf; k += 256) {
        const int f = free_idx[k];
        if (f < 0)
            for (int i = 0; i < 7; ++i) pose7_trial[7 * k + i] = pose7[7 * k + i];
        else
            se3_plus(pose7 + 7 * k, x + 6 * f, pose7_trial + 7 * k);
    }
    if (tid == 0) {
        st->solve_ok = 1;
        st->dc2 = red[0];
        st->gcdc = red[256];
    }
}

// --------------------------------------------------------------------------------------
// K6a: per landmark: back-substitution, trial point and trial cost
// partials (SoA, n_lm each): new_cost, dp^2, g_p . dp, |p|^2
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ba_backsub_cost(Geometry G, const int* __restrict__ lm_slot,
                                                       const int* __restrict__ slot_kf, const int* __restrict__ slot_obs,
                                                       const uint8_t* __restrict__ obs_cam,
                                                       const double* __restrict__ obs_uv, const int* __restrict__ free_idx,
                                                       const double* __restrict__ sf, const double* __restrict__ lmd,
                                                       const double* __restrict__ dc, const double* __restrict__ pose7_trial,
                                                       const double* __restrict__ pW, double* __restrict__ pW_trial,
                                                       double* __restrict__ part, const LmState* __restrict__ st) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= G.n_lm || st->done || !st->solve_ok) return;
    const int n = G.n_slot, m = G.n_lm;
    double rhs[3] = {-lmd[9 * m + l], -lmd[10 * m + l], -lmd[11 * m + l]};
    const int s0 = lm_slot[l], s1 = lm_slot[l + 1];
    for (int s = s0; s < s1; ++s) {
        const int f = free_idx[slot_kf[s]];
        if (f < 0) continue;
        const double* d6 = dc + 6 * f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double acc = 0.0;
#pragma unroll
            for (int a = 0; a < 6; ++a) acc += sf[(F_W + a * 3 + c) * n + s] * d6[a];
            rhs[c] -= acc;
        }
    }
    double dp[3], p[3], pt[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
        dp[c] = (lmd[(c * 3) * m + l] * rhs[0] + lmd[(c * 3 + 1) * m + l] * rhs[1]) + lmd[(c * 3 + 2) * m + l] * rhs[2];
    double dp2 = 0.0, gpdp = 0.0, p2 = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        p[c] = pW[3 * l + c];
        pt[c] = p[c] + dp[c];
        pW_trial[3 * l + c] = pt[c];
        dp2 += dp[c] * dp[c];
        gpdp += lmd[(9 + c) * m + l] * dp[c];
        p2 += p[c] * p[c];
    }
    double cost = 0.0;
    for (int s = s0; s < s1; ++s) {
        const Pose P = pose_from7(pose7_trial + 7 * slot_kf[s]);
        for (int o = slot_obs[s]; o < slot_obs[s + 1]; ++o) {
            double r[2], J[2][9];
            linearize(pt, P, G.TCB[obs_cam[o]].m, obs_uv + 2 * o, r, J, false);
            double rho, w;
            huber(r[0] * r[0] + r[1] * r[1], G.huber_delta, &rho, &w);
            cost += 0.5 * rho;
        }
    }
    part[l] = cost;
    part[m + l] = dp2;
    part[2 * m + l] = gpdp;
    part[3 * m + l] = p2;
}

// K6b: fixed-order sums of the per-landmark partials (+ free pose |x|^2 on rank 0's view)
__global__ __launch_bounds__(256) void ba_reduce_trial(Geometry G, const double* __restrict__ part,
                                                       const double* __restrict__ pose7, const int* __restrict__ free_idx,
                                                       double* __restrict__ out4, const LmState* __restrict__ st,
                                                       int include_poses) {
    __shared__ double sh[4 * 256];
    if (st->done) return;
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    if (st->solve_ok) {
        for (int l = threadIdx.x; l < G.n_lm; l += 256)
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += part[i * G.n_lm + l];
    }
    block_reduce<4>(v, sh);
    if (threadIdx.x == 0) {
        double x2 = v[3];
        if (include_poses)
            for (int k = 0; k < G.n_kf; ++k)
                if (free_idx[k] >= 0)
                    for (int i = 0; i < 7; ++i) x2 += pose7[7 * k + i] * pose7[7 * k + i];
        out4[0] = v[0];
        out4[1] = v[1];
        out4[2] = v[2];
        out4[3] = x2;
    }
}

// K7: LM decision (single thread); accepted -> copy trial state into the current state
__global__ __launch_bounds__(256) void ba_lm_decide(Geometry G, LmState* __restrict__ st, const double* __restrict__ sys,
                                                    const double* __restrict__ trial4, double* __restrict__ pose7,
                                                    const double* __restrict__ pose7_trial, double* __restrict__ pW,
                                                    const double* __restrict__ pW_trial, int max_iter, double cost_tol,
                                                    double param_tol) {
    __shared__ int accept;
    if (st->done) return;
    if (threadIdx.x == 0) {
        LmState s = *st;
        const double cost = sys[G.n_pb * 36 + 12 * G.n_free];  // cost at the current state
        if (s.iter == 0) s.initial_cost = cost;
        s.cost = cost;
        s.iter += 1;
        accept = 0;
        if (!isfinite(cost)) {
            s.status = RSVIO_LM_NUMERICAL_FAILURE;
            s.done = 1;
        } else if (!s.solve_ok) {
            s.lambda *= s.nu;
            s.nu *= 2.0;
            if (s.lambda > 1e32) {
                s.status = RSVIO_LM_TRUST_REGION;
                s.done = 1;
            }
        } else {
            s.new_cost = trial4[0];
            s.dp2 = trial4[1];
            s.gpdp = trial4[2];
            s.x2p = trial4[3];
            const double dx2 = s.dc2 + s.dp2;
            const double dxn = sqrt(dx2), xn = sqrt(s.x2p);
            if (dxn <= param_tol * (xn + param_tol)) {
                s.status = RSVIO_LM_PARAMETER_TOLERANCE;
                s.done = 1;
            } else {
                const double pred = 0.5 * (s.lambda * dx2 - (s.gcdc + s.gpdp));
                const double rho = (cost - s.new_cost) / pred;
                if (isfinite(s.new_cost) && rho > 0.0) {
                    const double dcost = cost - s.new_cost;
                    accept = 1;
                    const double f = 2.0 * rho - 1.0;
                    s.lambda *= fmax(1.0 / 3.0, 1.0 - f * f * f);
                    s.nu = 2.0;
                    s.cost = s.new_cost;
                    if (dcost <= cost_tol * (s.cost + dcost)) {
                        s.status = RSVIO_LM_COST_TOLERANCE;
                        s.done = 1;
                    }
                } else {
                    s.lambda *= s.nu;
                    s.nu *= 2.0;
                    if (s.lambda > 1e32) {
                        s.status = RSVIO_LM_TRUST_REGION;
                        s.done = 1;
                    }
                }
            }
        }
        s.accepted = accept;
        if (!s.done && s.iter >= max_iter) {
            s.status = RSVIO_LM_MAX_ITERATIONS;
            s.done = 1;
        }
        *st = s;
    }
    __syncthreads();
    if (accept) {
        for (int i = threadIdx.x; i < 7 * G.n_kf; i += blockDim.x) pose7[i] = pose7_trial[i];
        for (int i = threadIdx.x; i < 3 * G.n_lm; i += blockDim.x) pW[i] = pW_trial[i];
    }
}

}  // namespace

// ======================================================================================
struct BundleAdjuster {
    rsvio_ba_params P{};
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    Geometry G{};
    bool has_problem = false;
    // device
    DevBuf<double> d_pose, d_pose_init, d_pose_trial, d_pw, d_pw_init, d_pw_trial, d_uv;
    DevBuf<uint8_t> d_cam;
    DevBuf<int> d_free, d_slot_lm, d_slot_kf, d_slot_obs, d_lm_slot, d_pb_fa, d_pb_fb, d_pair_ptr, d_pair_a, d_pair_b;
    DevBuf<double> d_sf, d_Y, d_yg, d_lmd, d_sys, d_dc, d_part, d_trial4;
    DevBuf<LmState> d_state;
    HostBuf<LmState> h_state;
    // multi-rank
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;

    void init(const rsvio_ba_params& p) {
        P = p;
        if (P.max_keyframes < 2 || P.max_keyframes > kMaxFree + 1 || P.max_landmarks < 1 || P.max_observations < 1)
            throw std::invalid_argument("invalid BA capacities (max_keyframes in [2, 21])");
        RSVIO_HIP(hipSetDevice(P.device));
        RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        RSVIO_HIP(hipEventCreate(&ev0));
        RSVIO_HIP(hipEventCreate(&ev1));
        h_state.alloc(1);
    }
    ~BundleAdjuster() {
        if (comm) ncclCommDestroy(comm);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (stream) (void)hipStreamDestroy(stream);
    }

    template <class T>
    static void grow(DevBuf<T>& b, size_t n) {
        if (b.n < n) b.alloc(std::max<size_t>(n, 1));
    }
    template <class T>
    void up(DevBuf<T>& b, const T* src, size_t n) {
        grow(b, n);
        if (n) RSVIO_HIP(hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, stream));
    }

    void set_problem(int n_kf, const double* pose7, const uint8_t* kf_fixed, int n_lm, const double* pW, int n_obs,
                     const int32_t* obs_lm, const int32_t* obs_kf, const uint8_t* obs_cam, const double* obs_uv,
                     const double* TCB2) {
        if (n_kf < 1 || n_kf > P.max_keyframes || n_lm < 0 || n_lm > P.max_landmarks || n_obs < 0 ||
            n_obs > P.max_observations)
            throw std::invalid_argument("problem exceeds the handle's capacities");
        std::vector<int> free_idx(n_kf, -1);
        int n_free = 0;
        for (int k = 0; k < n_kf; ++k)
            if (!kf_fixed[k]) free_idx[k] = n_free++;
        if (n_free > kMaxFree) throw std::invalid_argument("too many free keyframes");
        for (int i = 0; i < n_obs; ++i)
            if (obs_lm[i] < 0 || obs_lm[i] >= n_lm || obs_kf[i] < 0 || obs_kf[i] >= n_kf || obs_cam[i] > 1)
                throw std::invalid_argument("observation index out of range");
        // landmark-major CSR of observations sorted by (landmark, keyframe, camera)
        std::vector<int> order(n_obs);
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
            if (obs_lm[a] != obs_lm[b]) return obs_lm[a] < obs_lm[b];
            if (obs_kf[a] != obs_kf[b]) return obs_kf[a] < obs_kf[b];
            return obs_cam[a] < obs_cam[b];
        });
        std::vector<double> uv(2 * (size_t)n_obs);
        std::vector<uint8_t> cam(n_obs);
        std::vector<int> slot_lm, slot_kf, slot_obs, lm_slot(n_lm + 1, 0);
        for (int q = 0; q < n_obs; ++q) {
            const int o = order[q];
            uv[2 * q] = obs_uv[2 * o];
            uv[2 * q + 1] = obs_uv[2 * o + 1];
            cam[q] = obs_cam[o];
            if (q == 0 || obs_lm[o] != obs_lm[order[q - 1]] || obs_kf[o] != obs_kf[order[q - 1]]) {
                slot_lm.push_back(obs_lm[o]);
                slot_kf.push_back(obs_kf[o]);
                slot_obs.push_back(q);
                lm_slot[obs_lm[o] + 1] += 1;
            }
        }
        const int n_slot = (int)slot_lm.size();
        slot_obs.push_back(n_obs);
        for (int l = 0; l < n_lm; ++l) lm_slot[l + 1] += lm_slot[l];
        // camera blocks (fa <= fb), row-major upper triangle, and their slot pairs
        std::vector<int> pb_fa, pb_fb, pb_of((size_t)n_free * n_free, -1);
        for (int a = 0; a < n_free; ++a)
            for (int b = a; b < n_free; ++b) {
                pb_of[a * n_free + b] = (int)pb_fa.size();
                pb_fa.push_back(a);
                pb_fb.push_back(b);
            }
        const int n_pb = (int)pb_fa.size();
        std::vector<std::vector<std::pair<int, int>>> pairs(n_pb);
        for (int l = 0; l < n_lm; ++l)
            for (int sa = lm_slot[l]; sa < lm_slot[l + 1]; ++sa) {
                const int fa = free_idx[slot_kf[sa]];
                if (fa < 0) continue;
                for (int sb = sa; sb < lm_slot[l + 1]; ++sb) {
                    const int fb = free_idx[slot_kf[sb]];
                    if (fb < 0) continue;
                    pairs[pb_of[fa * n_free + fb]].push_back({sa, sb});
                }
            }
        std::vector<int> pair_ptr(n_pb + 1, 0), pa, pbv;
        for (int b = 0; b < n_pb; ++b) {
            pair_ptr[b + 1] = pair_ptr[b] + (int)pairs[b].size();
            for (auto& pr : pairs[b]) {
                pa.push_back(pr.first);
                pbv.push_back(pr.second);
            }
        }
        G.n_kf = n_kf;
        G.n_free = n_free;
        G.n_lm = n_lm;
        G.n_obs = n_obs;
        G.n_slot = n_slot;
        G.n_pb = n_pb;
        for (int c = 0; c < 2; ++c)
            for (int i = 0; i < 16; ++i) G.TCB[c].m[i] = TCB2[16 * c + i];
        up(d_pose_init, pose7, 7 * (size_t)n_kf);
        up(d_pw_init, pW, 3 * (size_t)n_lm);
        grow(d_pose, 7 * (size_t)n_kf);
        grow(d_pose_trial, 7 * (size_t)n_kf);
        grow(d_pw, 3 * (size_t)n_lm);
        grow(d_pw_trial, 3 * (size_t)n_lm);
        up(d_uv, uv.data(), uv.size());
        up(d_cam, cam.data(), cam.size());
        up(d_free, free_idx.data(), free_idx.size());
        up(d_slot_lm, slot_lm.data(), slot_lm.size());
        up(d_slot_kf, slot_kf.data(), slot_kf.size());
        up(d_slot_obs, slot_obs.data(), slot_obs.size());
        up(d_lm_slot, lm_slot.data(), lm_slot.size());
        up(d_pb_fa, pb_fa.data(), pb_fa.size());
        up(d_pb_fb, pb_fb.data(), pb_fb.size());
        up(d_pair_ptr, pair_ptr.data(), pair_ptr.size());
        up(d_pair_a, pa.data(), pa.size());
        up(d_pair_b, pbv.data(), pbv.size());
        grow(d_sf, (size_t)kSlotFields * n_slot);
        grow(d_Y, (size_t)18 * n_slot);
        grow(d_yg, (size_t)6 * n_slot);
        grow(d_lmd, (size_t)14 * n_lm);
        grow(d_sys, (size_t)36 * n_pb + 12 * n_free + 2);
        grow(d_dc, (size_t)6 * n_free);
        grow(d_part, (size_t)4 * n_lm);
        grow(d_trial4, 4);
        grow(d_state, 1);
        RSVIO_HIP(hipStreamSynchronize(stream));
        has_problem = true;
    }

    void reset_state(double lambda0) {
        RSVIO_HIP(hipMemcpyAsync(d_pose.p, d_pose_init.p, sizeof(double) * 7 * G.n_kf, hipMemcpyDeviceToDevice, stream));
        if (G.n_lm)
            RSVIO_HIP(hipMemcpyAsync(d_pw.p, d_pw_init.p, sizeof(double) * 3 * G.n_lm, hipMemcpyDeviceToDevice, stream));
        LmState s{};
        s.lambda = lambda0;
        s.nu = 2.0;
        *h_state.p = s;
        RSVIO_HIP(hipMemcpyAsync(d_state.p, h_state.p, sizeof(LmState), hipMemcpyHostToDevice, stream));
    }

    void allreduce(double* buf, size_t n) {
        if (!comm || n == 0) return;
        if (ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm, stream) != ncclSuccess)
            throw std::runtime_error("RCCL all-reduce failed");
    }

    void enqueue_linear_system() {
        const int B = 256;
        if (G.n_slot)
            hipLaunchKernelGGL(ba_slot_linearize, dim3((G.n_slot + B - 1) / B), dim3(B), 0, stream, G, d_pose.p, d_pw.p,
                               d_slot_lm.p, d_slot_kf.p, d_slot_obs.p, d_cam.p, d_uv.p, d_free.p, d_sf.p, d_state.p);
        if (G.n_lm)
            hipLaunchKernelGGL(ba_landmark_eliminate, dim3((G.n_lm + B - 1) / B), dim3(B), 0, stream, G, d_lm_slot.p,
                               d_slot_kf.p, d_free.p, d_sf.p, d_Y.p, d_yg.p, d_lmd.p, d_state.p);
        hipLaunchKernelGGL(ba_schur_blocks, dim3(G.n_pb + 1), dim3(256), 0, stream, G, d_pb_fa.p, d_pb_fb.p,
                           d_pair_ptr.p, d_pair_a.p, d_pair_b.p, d_sf.p, d_Y.p, d_yg.p, d_lmd.p, d_sys.p, d_state.p,
                           rank == 0 ? 1 : 0);
        RSVIO_HIP(hipGetLastError());
        // S, b, g_c and the cost are sums over landmarks: sum the per-rank partials
        allreduce(d_sys.p, (size_t)36 * G.n_pb + 12 * G.n_free + 2);
    }

    void enqueue_iteration(const rsvio_lm_cfg& cfg) {
        const int B = 256;
        enqueue_linear_system();
        hipLaunchKernelGGL(ba_dense_solve, dim3(1), dim3(256), 0, stream, G, d_pb_fa.p, d_pb_fb.p, d_sys.p, d_pose.p,
                           d_free.p, d_pose_trial.p, d_dc.p, d_state.p);
        if (G.n_lm)
            hipLaunchKernelGGL(ba_backsub_cost, dim3((G.n_lm + B - 1) / B), dim3(B), 0, stream, G, d_lm_slot.p,
                               d_slot_kf.p, d_slot_obs.p, d_cam.p, d_uv.p, d_free.p, d_sf.p, d_lmd.p, d_dc.p,
                               d_pose_trial.p, d_pw.p, d_pw_trial.p, d_part.p, d_state.p);
        hipLaunchKernelGGL(ba_reduce_trial, dim3(1), dim3(256), 0, stream, G, d_part.p, d_pose.p, d_free.p, d_trial4.p,
                           d_state.p, rank == 0 ? 1 : 0);
        RSVIO_HIP(hipGetLastError());
        allreduce(d_trial4.p, 4);
        hipLaunchKernelGGL(ba_lm_decide, dim3(1), dim3(256), 0, stream, G, d_state.p, d_sys.p, d_trial4.p, d_pose.p,
                           d_pose_trial.p, d_pw.p, d_pw_trial.p, cfg.max_iterations, cfg.cost_tolerance,
                           cfg.parameter_tolerance);
        RSVIO_HIP(hipGetLastError());
    }

    void run(const rsvio_lm_cfg& cfg, rsvio_ba_result* res) {
        if (!has_problem) throw std::invalid_argument("no problem uploaded");
        G.huber_delta = cfg.huber_delta;
        res->iterations = 0;
        // sliding_window.rs:303-319: too few residuals / underconstrained -> skip (Ok(false))
        if (G.n_obs < 6 || G.n_obs < G.n_free + G.n_lm) {
            if (!comm) {
                res->status = RSVIO_LM_SKIPPED;
                res->initial_cost = res->final_cost = 0.0;
                res->solve_ms = 0.0;
                return;
            }
        }
        // with sharding every rank adds lambda/nranks to its diagonal so the sum carries lambda once
        reset_state(cfg.lambda_init);
        RSVIO_HIP(hipEventRecord(ev0, stream));
        const int max_it = std::max(cfg.max_iterations, 1);
        for (int it = 0; it < max_it; ++it) {
            enqueue_iteration(cfg);
            RSVIO_HIP(hipMemcpyAsync(h_state.p, d_state.p, sizeof(LmState), hipMemcpyDeviceToHost, stream));
            RSVIO_HIP(hipStreamSynchronize(stream));
            if (h_state.p->done) break;
        }
        RSVIO_HIP(hipEventRecord(ev1, stream));
        RSVIO_HIP(hipEventSynchronize(ev1));
        float ms = 0.0f;
        RSVIO_HIP(hipEventElapsedTime(&ms, ev0, ev1));
        const LmState& s = *h_state.p;
        res->status = s.status;
        res->iterations = s.iter;
        res->initial_cost = s.initial_cost;
        res->final_cost = s.cost;
        res->solve_ms = ms;
    }

    void build_system(double lambda, double huber_delta, double* S, double* b, double* cost) {
        if (!has_problem) throw std::invalid_argument("no problem uploaded");
        G.huber_delta = huber_delta;
        reset_state(lambda);
        enqueue_linear_system();
        std::vector<double> sys((size_t)36 * G.n_pb + 12 * G.n_free + 2);
        RSVIO_HIP(hipMemcpyAsync(sys.data(), d_sys.p, sizeof(double) * sys.size(), hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
        const int n = 6 * G.n_free;
        std::vector<int> fa, fb;
        for (int a = 0; a < G.n_free; ++a)
            for (int c = a; c < G.n_free; ++c) {
                fa.push_back(a);
                fb.push_back(c);
            }
        for (int pb = 0; pb < G.n_pb; ++pb)
            for (int e = 0; e < 36; ++e) {
                const int a = e / 6, c = e % 6;
                S[(size_t)(6 * fa[pb] + a) * n + 6 * fb[pb] + c] = sys[pb * 36 + e];
                S[(size_t)(6 * fb[pb] + c) * n + 6 * fa[pb] + a] = sys[pb * 36 + e];
            }
        for (int i = 0; i < n; ++i) b[i] = sys[36 * G.n_pb + i];
        *cost = sys[36 * G.n_pb + 12 * G.n_free];
    }
};

}  // namespace rsvio

struct rsvio_ba {
    rsvio::BundleAdjuster b;
};

using rsvio::guarded;

extern "C" {

int rsvio_ba_create(const rsvio_ba_params* params, rsvio_ba** out) {
    if (!params || !out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto* h = new rsvio_ba();
        try {
            h->b.init(*params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
        return (int)RSVIO_OK;
    });
}

void rsvio_ba_destroy(rsvio_ba* ba) { delete ba; }

static bool problem_args_ok(int32_t n_kf, const double* pose7, const uint8_t* kf_fixed, int32_t n_lm, const double* p_W,
                            int32_t n_obs, const int32_t* obs_lm, const int32_t* obs_kf, const uint8_t* obs_cam,
                            const double* obs_uv, const double* T_C_B2) {
    if (n_kf < 1 || n_lm < 0 || n_obs < 0 || !pose7 || !kf_fixed || !T_C_B2) return false;
    if (n_lm > 0 && !p_W) return false;
    if (n_obs > 0 && (!obs_lm || !obs_kf || !obs_cam || !obs_uv)) return false;
    return true;
}

int rsvio_ba_set_problem(rsvio_ba* ba, int32_t n_kf, const double* pose7, const uint8_t* kf_fixed, int32_t n_lm,
                         const double* p_W, int32_t n_obs, const int32_t* obs_lm, const int32_t* obs_kf,
                         const uint8_t* obs_cam, const double* obs_uv, const double* T_C_B2) {
    if (!ba || !problem_args_ok(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2))
        return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.set_problem(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_run(rsvio_ba* ba, const rsvio_lm_cfg* cfg, rsvio_ba_result* res) {
    if (!ba || !cfg || !res) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.run(*cfg, res);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_get_state(rsvio_ba* ba, double* pose7, double* p_W) {
    if (!ba || !pose7 || (!p_W && ba->b.G.n_lm)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& B = ba->b;
        RSVIO_HIP(hipMemcpyAsync(pose7, B.d_pose.p, sizeof(double) * 7 * B.G.n_kf, hipMemcpyDeviceToHost, B.stream));
        if (B.G.n_lm)
            RSVIO_HIP(hipMemcpyAsync(p_W, B.d_pw.p, sizeof(double) * 3 * B.G.n_lm, hipMemcpyDeviceToHost, B.stream));
        RSVIO_HIP(hipStreamSynchronize(B.stream));
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_solve(rsvio_ba* ba, int32_t n_kf, double* pose7, const uint8_t* kf_fixed, int32_t n_lm, double* p_W,
                   int32_t n_obs, const int32_t* obs_lm, const int32_t* obs_kf, const uint8_t* obs_cam,
                   const double* obs_uv, const double* T_C_B2, const rsvio_lm_cfg* cfg, rsvio_ba_result* res) {
    if (!ba || !cfg || !res ||
        !problem_args_ok(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2))
        return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& B = ba->b;
        B.set_problem(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2);
        B.run(*cfg, res);
        if (res->status > 0) {  // success: hand back the optimised state (sliding_window.rs:364-374)
            RSVIO_HIP(hipMemcpyAsync(pose7, B.d_pose.p, sizeof(double) * 7 * n_kf, hipMemcpyDeviceToHost, B.stream));
            if (n_lm)
                RSVIO_HIP(hipMemcpyAsync(p_W, B.d_pw.p, sizeof(double) * 3 * n_lm, hipMemcpyDeviceToHost, B.stream));
            RSVIO_HIP(hipStreamSynchronize(B.stream));
        }
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_build_system(rsvio_ba* ba, double lambda, double huber_delta, double* S, double* b, double* cost) {
    if (!ba || !S || !b || !cost) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.build_system(lambda, huber_delta, S, b, cost);
        return (int)RSVIO_OK;
    });
}

int rsvio_rccl_unique_id(uint8_t* out, size_t cap) {
    if (!out || cap < sizeof(ncclUniqueId)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ncclUniqueId id;
        if (ncclGetUniqueId(&id) != ncclSuccess) {
            rsvio::set_last_error("ncclGetUniqueId failed");
            return (int)RSVIO_ERR_RCCL;
        }
        __builtin_memcpy(out, &id, sizeof(id));
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_attach_comm(rsvio_ba* ba, int32_t nranks, int32_t rank, const uint8_t* unique_id) {
    if (!ba || !unique_id || nranks < 1 || rank < 0 || rank >= nranks) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& B = ba->b;
        if (nranks == 1) return (int)RSVIO_OK;
        ncclUniqueId id;
        __builtin_memcpy(&id, unique_id, sizeof(id));
        RSVIO_HIP(hipSetDevice(B.P.device));
        if (ncclCommInitRank(&B.comm, nranks, id, rank) != ncclSuccess) {
            rsvio::set_last_error("ncclCommInitRank failed");
            return (int)RSVIO_ERR_RCCL;
        }
        B.nranks = nranks;
        B.rank = rank;
        return (int)RSVIO_OK;
    });
}

}  // extern "C"
