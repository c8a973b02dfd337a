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
// grid-wide synchronisation).  Round 6 layout:
//   * the join: rsvio_pnp_set_map builds a bucketed hash table of the map on the host (4 entries of
//     {id, p_W} per 128-B bucket, load <= 1/4) and uploads it once per map; a feature's id is looked
//     up with ONE bucket load (its map point inside the entry), so a frame pays two dependent round
//     trips (feature, bucket) instead of staging the map in LDS and an 11-step binary search
//     (10.1k of the kernel's 53.8k cycles, profiles/r05pnp_stamps.txt);
//   * the LM control runs on all of wave 0 at once, its state in registers (every lane the same
//     values) instead of lane 0 against an LDS struct; T_C_W of the next pass is written by the
//     same wave, so a pass costs two workgroup barriers instead of four.
// Every pass linearises all matched observations at one pose and reduces H (21), g (6) and the
// cost in a fixed order (DPP reduce-scatter per wave, then the waves in order).  Each pass after
// the first is at a trial pose: if the step is accepted its H and g are the next system, so an
// accepted iteration costs one pass.
#include <cmath>
#include <cstring>
#include <algorithm>
#include <stdexcept>
#include <vector>

#include "common.hpp"
#include "rotation.hpp"
#include "se3.hpp"

namespace rsvio {
namespace {

RSVIO_DBG_DECL

constexpr int kPnpThreads = 512;
constexpr int kPnpWaves = kPnpThreads / 64;
constexpr int kPnpMaxFeatures = 4096; // features per frame (both cameras), observations in LDS
constexpr int kRed = 28;          // H upper (21), g (6), cost
constexpr uint64_t kEmptyId = ~0ull;  // a free hash-table entry
constexpr int kBucket = 4;            // entries per 128-B bucket

// One hash-table entry: the map id and its point (sliding_window.rs:466-475 keeps map_points as
// [f32; 3]); 32 B, 4 per 128-B line
struct alignas(32) PnpEntry {
    uint64_t id;
    float pw[3];
    uint32_t pad;
};
static_assert(sizeof(PnpEntry) == 32, "4 entries per 128-B bucket");

__host__ __device__ __forceinline__ uint32_t map_bucket(uint64_t id, int mask) {
    return (uint32_t)((id * 0x9E3779B97F4A7C15ull) >> 40) & (uint32_t)mask;  // Fibonacci hashing
}

enum { LM_COST_TOL = 1, LM_PARAM_TOL = 2, LM_MAX_ITERS = 3, LM_TRUST_REGION = 4, LM_NUMFAIL = -1, LM_SKIPPED = -2,
       LM_LINSOLVE = -3 };

struct PnpArgs {
    const uint8_t* ids[2];   // u64 feature ids, `id_stride` bytes apart
    int id_stride;
    const float2* uv[2];     // undistorted coordinates (frame.rs:118-119,131-132)
    const int* dcount;       // device (n_l, n_r), or null: n[] below
    int n[2];
    const PnpEntry* table;   // the map as a bucketed hash table (MapTable)
    int bucket_mask;         // buckets - 1 (a power of two)
    int max_probe;           // the longest bucket run an insertion took (lookups stop there)
    int has_top;             // a map point has the id kEmptyId (not representable in the table)
    float top_pw[3];         // ... its p_W
    int n_map;
    double T_last[16];
    double q0[4];            // from_matrix(R_B_W) of the last keyframe (host, rotation.hpp)
    double TCB[2][16];
    int max_iter;
    double cost_tol, param_tol, huber_delta, lambda0, thr_t, thr_r;
    rsvio_motion_result* out;  // pinned host memory
    double wclk_khz;           // device wall clock rate (kernel_ms)
};

// LM control state: wave 0's registers, every lane holding the same values
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
// rounding (~60 flops instead of ~180; 1/z by the refined hardware reciprocal; tolerance parity
// with the oracle's reference order).
__device__ __forceinline__ void pnp_linearize_cw(const double pW[3], const double uv[2], const double* T,
                                                 double r[2], double J[2][6]) {
    const double pC0 = ((T[0] * pW[0] + T[1] * pW[1]) + T[2] * pW[2]) + T[9];
    const double pC1 = ((T[3] * pW[0] + T[4] * pW[1]) + T[5] * pW[2]) + T[10];
    const double pC2 = ((T[6] * pW[0] + T[7] * pW[1]) + T[8] * pW[2]) + T[11];
    const double iz = rcp_f64(pC2);
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

// Huber(delta) (factors.rs, the Ceres-style rho and IRLS weight as se3.hpp's huber) with one
// refined reciprocal square root instead of sqrt + a division: rho = 2 d s / sqrt(s) - d^2,
// w = d / sqrt(s) (tolerance parity)
__device__ __forceinline__ void pnp_huber(double s, double d, double* rho, double* w) {
    const double d2 = d * d;
    if (s <= d2) {
        *rho = s;
        *w = 1.0;
    } else {
        const double is = rsqrt_f64(s);
        *rho = 2.0 * d * (s * is) - d2;
        *w = d * is;
    }
}

// (H + lambda I) dx = -g by LDL^T with hardware-reciprocal pivots (no square root, no IEEE
// division on the serial chain).  Positive definiteness is tested on the pivots exactly like
// the oracle's Cholesky (chol_solve) tests d > 0; the solution agrees to rounding (tolerance
// parity).  All operands in registers (wave 0, every lane the same values).
__device__ __forceinline__ bool ldl6(const double (&Hp)[21], double lambda, const double (&g)[6], double (&dx)[6]) {
    double A[6][6];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = a; c < 6; ++c) A[c][a] = Hp[utri6(a, c)];  // lower triangle
#pragma unroll
    for (int a = 0; a < 6; ++a) A[a][a] += lambda;
    double L[6][6], U[6][6], inv[6];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= L[j][k] * U[j][k];
        ok &= (d > 0.0) && isfinite(d);
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
    return ok;
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
// (from its normalised quaternion).  The four functions of theta by se3.hpp's power series in
// theta^2 for |theta| < 1/4 (an LM step's rotation: no square root, sincos or division on the
// chain), one sincos of theta / 2 otherwise -- the BA's se3_plus; tolerance parity.
__device__ __forceinline__ void se3_plus_r(const double (&p7)[7], const double (&R)[9], const double (&d)[6],
                                           double (&out)[7], double (&Rout)[9]) {
    const double* rho = d;
    const double* om = d + 3;
    const double th2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
    double qd[4], Ac, Bc;
    if (th2 < 0.0625) {
        const double s = se3_series<1>(th2);  // sin(theta/2) / theta
        qd[0] = se3_series<0>(th2);           // cos(theta/2)
        qd[1] = s * om[0]; qd[2] = s * om[1]; qd[3] = s * om[2];
        Ac = se3_series<2>(th2);
        Bc = se3_series<3>(th2);
    } else {
        const double th = sqrt(th2);
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

// Lane 0 of wave 0 between passes (the state in LDS: its registers are the pass's): consume the
// pass sums, then either set up the next pass at a trial pose (C.run = 1, its R_BW and t_BW in
// pose[12]) or finish (run = 0).  Mirrors oracle orc_track_motion's loop step for step.
__device__ __forceinline__ void pnp_control(const PnpArgs& A, Ctl& C, const double* __restrict__ sum,
                                         double* __restrict__ pose) {
    bool done = false;
    if (C.phase == 0) {
#pragma unroll
        for (int k = 0; k < 21; ++k) C.H[k] = sum[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) C.g[k] = sum[21 + k];
        C.cost = sum[27];
        C.initial_cost = C.cost;
        C.phase = 1;
    } else {
        const double new_cost = sum[27];
        const double dcost = C.cost - new_cost;
        const double rho = dcost / C.pred;
        if (isfinite(new_cost) && fabs(dcost) <= A.cost_tol * C.cost) {
            // converged: the change is within the tolerance whatever its sign, the candidate not
            // applied (the BA's lm_update takes the same decision).  This
            // build's rule, a deliberate departure: apex-solver's is absent offline (unpinned)
            C.status = LM_COST_TOL;
            done = true;
        } else if (isfinite(new_cost) && rho > 0.0) {
#pragma unroll
            for (int k = 0; k < 7; ++k) C.x[k] = C.xt[k];
#pragma unroll
            for (int k = 0; k < 9; ++k) C.R[k] = C.Rt[k];
#pragma unroll
            for (int k = 0; k < 21; ++k) C.H[k] = sum[k];
#pragma unroll
            for (int k = 0; k < 6; ++k) C.g[k] = sum[21 + k];
            const double f = 2.0 * rho - 1.0;
            C.lambda *= fmax(1.0 / 3.0, 1.0 - f * f * f);
            C.nu = 2.0;
            C.cost = new_cost;
        } else {
            C.lambda *= C.nu;
            C.nu *= 2.0;
            if (C.lambda > 1e32) {
                C.status = LM_TRUST_REGION;
                done = true;
            }
        }
    }
    C.run = 0;
    if (done) return;
    if (C.it >= A.max_iter) {
        C.status = LM_MAX_ITERS;
        return;
    }
    C.it += 1;
    if (!isfinite(C.cost)) {
        C.status = LM_NUMFAIL;
        return;
    }
    double dx[6], H[21], g[6];
#pragma unroll
    for (int k = 0; k < 21; ++k) H[k] = C.H[k];
#pragma unroll
    for (int k = 0; k < 6; ++k) g[k] = C.g[k];
    const bool solved = ldl6(H, C.lambda, g, dx);
    STAMP(30);
    if (!solved) {  // Err(LinearSolveFailed) -> track_motion returns Ok(None) (:554-560)
        C.status = LM_LINSOLVE;
        return;
    }
    double dx2 = 0.0, gdx = 0.0, x2 = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        dx2 += dx[k] * dx[k];
        gdx += g[k] * dx[k];
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) x2 += C.x[k] * C.x[k];
    if (sqrt(dx2) <= A.param_tol * (sqrt(x2) + A.param_tol)) {
        C.status = LM_PARAM_TOL;
        return;
    }
    double x[7], R[9], xt[7], Rt[9];
#pragma unroll
    for (int k = 0; k < 7; ++k) x[k] = C.x[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = C.R[k];
    se3_plus_r(x, R, dx, xt, Rt);
#pragma unroll
    for (int k = 0; k < 7; ++k) C.xt[k] = xt[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) C.Rt[k] = Rt[k];
    STAMP(31);
    C.pred = 0.5 * (C.lambda * dx2 - gdx);
#pragma unroll
    for (int k = 0; k < 9; ++k) pose[k] = Rt[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) pose[9 + k] = xt[k];
    C.run = 1;
}

// lane 0 of wave 0
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

// The map point of `id` (map_points.get, sliding_window.rs:526-545): the bucket of its hash, then
// the following ones up to the longest run an insertion took; a bucket with a free entry ends a
// miss.  One 128-B load per bucket visited (almost always one).
__device__ __forceinline__ bool map_lookup(const PnpArgs& A, uint64_t id, float (&pw)[3]) {
    if (id == kEmptyId) {
        pw[0] = A.top_pw[0]; pw[1] = A.top_pw[1]; pw[2] = A.top_pw[2];
        return A.has_top != 0;
    }
    uint32_t b = map_bucket(id, A.bucket_mask);
    for (int p = 0; p <= A.max_probe; ++p) {
        // the bucket's 4 entries as 8 16-B loads, all in flight; the match picked by selects (no
        // runtime-indexed local array: that would go through scratch)
        const uint4* e = reinterpret_cast<const uint4*>(A.table + (size_t)b * kBucket);
        uint4 v[2 * kBucket];
#pragma unroll
        for (int k = 0; k < 2 * kBucket; ++k) v[k] = e[k];
        bool hit = false, free_slot = false;
        uint32_t x = 0, y = 0, z = 0;
#pragma unroll
        for (int k = 0; k < kBucket; ++k) {
            const uint64_t key = (uint64_t)v[2 * k].x | ((uint64_t)v[2 * k].y << 32);
            const bool m = key == id;
            x = m ? v[2 * k].z : x;
            y = m ? v[2 * k].w : y;
            z = m ? v[2 * k + 1].x : z;
            hit |= m;
            free_slot |= key == kEmptyId;
        }
        if (hit) {
            pw[0] = __uint_as_float(x); pw[1] = __uint_as_float(y); pw[2] = __uint_as_float(z);
            return true;
        }
        if (free_slot) return false;
        b = (b + 1) & (uint32_t)A.bucket_mask;
    }
    return false;
}

__global__ __launch_bounds__(kPnpThreads) void pnp_track_motion_kernel(PnpArgs A) {
    __shared__ float s_mpw[3][kPnpMaxFeatures];  // the matched map point per feature
    __shared__ float s_uv[2][kPnpMaxFeatures];   // undistorted coordinates per feature
    __shared__ int8_t s_cam[kPnpMaxFeatures];    // feature -> camera, -1: no map point
    __shared__ double s_red[kPnpWaves][kRed];
    __shared__ double s_sum[kRed];
    __shared__ double s_pose[12];                // R_BW, t_BW of the pass pose (wave 0's)
    __shared__ double s_tcb[2][16];
    __shared__ double s_tcw[2][12];              // T_C_W = T_C_B T_B_W per camera at the pass pose
    __shared__ int s_nobs;
    __shared__ int s_run;
    __shared__ Ctl s_ctl;                        // the LM state between controls (wave 0's)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    STAMP(0);
    const unsigned long long t_entry = wall_clock64();  // (kept by thread 0 for kernel_ms)
    const int n0 = A.dcount ? A.dcount[0] : A.n[0];
    const int n1 = A.dcount ? A.dcount[1] : A.n[1];
    const int nf = n0 + n1;
    const bool fits = nf <= kPnpMaxFeatures;
    // the factor list: features with a map point, left then right (sliding_window.rs:519-547);
    // feature j's observation goes to LDS entry j (cam -1: no map point).  Two features per lane
    // per round: both id / uv loads, then both bucket loads in flight together.
    int mine = 0;
    if (tid == 0) s_nobs = 0;
    if (tid < 32) s_tcb[tid >> 4][tid & 15] = A.TCB[tid >> 4][tid & 15];
    for (int j0 = tid; j0 < nf && fits; j0 += 2 * kPnpThreads) {
        uint64_t id[2];
        float2 q[2];
        int cam[2];
        bool v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = j0 + h * kPnpThreads;
            v[h] = j < nf;
            const int jj = v[h] ? j : j0;
            cam[h] = jj < n0 ? 0 : 1;
            const int i = cam[h] == 0 ? jj : jj - n0;
            id[h] = *reinterpret_cast<const uint64_t*>(A.ids[cam[h]] + (size_t)i * A.id_stride);
            q[h] = A.uv[cam[h]][i];
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (!v[h]) continue;
            const int j = j0 + h * kPnpThreads;
            float pw[3];
            const bool hit = A.n_map > 0 && map_lookup(A, id[h], pw);
            s_cam[j] = hit ? (int8_t)cam[h] : (int8_t)-1;
            if (hit) {
                s_uv[0][j] = q[h].x;
                s_uv[1][j] = q[h].y;
                s_mpw[0][j] = pw[0];
                s_mpw[1][j] = pw[1];
                s_mpw[2][j] = pw[2];
                ++mine;
            }
        }
    }
    // wave 0: the LM state (LDS between controls, registers during one); F starts from the last
    // keyframe (sliding_window.rs:506-517)
    if (wv == 0) {
        Ctl C;
        C.it = 0;
        C.status = LM_MAX_ITERS;
        C.phase = 0;
        C.lambda = A.lambda0;
        C.nu = 2.0;
        C.cost = 0.0;
        C.initial_cost = 0.0;
        C.pred = 0.0;
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
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 9; ++k) s_pose[k] = C.R[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) s_pose[9 + k] = C.x[k];
            s_ctl = C;
        }
    }
    // per-wave total (one LDS atomic per wave instead of one per lane)
    for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off);
    __syncthreads();  // s_nobs = 0, s_tcb and s_pose (wave 0) before their uses
    if (lane == 0 && mine) atomicAdd(&s_nobs, mine);
    if (wv == 0) {
        if (lane < 24) {  // T_C_W = T_C_B T_B_W, one entry per lane
            const int c = lane / 12, e = lane % 12;
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
    }
    STAMP(1);
    __syncthreads();  // the factor list, s_nobs and the first T_C_W
    STAMP(2);
    const int nobs = s_nobs;
    int run = (fits && nobs > 0) ? 1 : 0;
    if (tid == 0) {
        s_ctl.n_obs = fits ? nobs : -1;
        if (!run) s_ctl.status = LM_SKIPPED;  // no factor: treated as a failed optimisation
    }
    int pass = 0;
    while (run) {
        if (pass < 12) STAMP(3 + 2 * pass);
        // one pass at the pose in s_tcw: H, g, cost over this lane's observations (j order)
        double acc[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) acc[k] = 0.0;
#pragma unroll 1
        for (int j = tid; j < nf; j += kPnpThreads) {
            const int cam = s_cam[j];
            if (cam < 0) continue;
            const double pW[3] = {(double)s_mpw[0][j], (double)s_mpw[1][j], (double)s_mpw[2][j]};
            const double uv[2] = {(double)s_uv[0][j], (double)s_uv[1][j]};
            double r[2], J[2][6];
            pnp_linearize_cw(pW, uv, s_tcw[cam], r, J);
            const double s2 = r[0] * r[0] + r[1] * r[1];
            double rho, w;
            pnp_huber(s2, A.huber_delta, &rho, &w);
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
        __syncthreads();  // every wave's partials
        if (pass < 12) STAMP(4 + 2 * pass);
        ++pass;
        if (wv == 0) {
            // the waves in order (lane k sums value k), then lane 0's control
            if (lane < kRed) {
                double v = s_red[0][lane];
#pragma unroll
                for (int w = 1; w < kPnpWaves; ++w) v += s_red[w][lane];
                s_sum[lane] = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                pnp_control(A, s_ctl, s_sum, s_pose);
                s_run = s_ctl.run;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (s_run && lane < 24) {
                const int c = lane / 12, e = lane % 12;
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
        }
        __syncthreads();  // s_run and the next pass's T_C_W
        run = s_run;
    }
    STAMP(28);
    if (tid == 0) pnp_finish(A, s_ctl, t_entry);
    STAMP(29);
}

}  // namespace

RSVIO_DBG_READER(rsvio_dbg_pnp_stamps)

struct Pnp {
    int device = 0;
    hipStream_t stream = nullptr;      // the handle's own
    hipStream_t user = nullptr;        // rsvio_pnp_set_stream
    hipStream_t active() const { return user ? user : stream; }
    // the map as a bucketed hash table (set_map): kBucket entries per bucket, a power of two of
    // buckets with at most one entry per kBucket slots used (load <= 1/4)
    DevBuf<PnpEntry> table;
    std::vector<PnpEntry> htable;
    int bucket_mask = 0, max_probe = 0, has_top = 0;
    float top_pw[3] = {0.f, 0.f, 0.f};
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
    A.table = p.table.p;
    A.bucket_mask = p.bucket_mask;
    A.max_probe = p.max_probe;
    A.has_top = p.has_top;
    for (int k = 0; k < 3; ++k) A.top_pw[k] = p.top_pw[k];
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
        // the hash table: >= 4 n entries (load <= 1/4: a bucket overflows into the next one for
        // well under 1 % of the ids), linear probing over buckets
        int nb = 16;
        while ((size_t)nb * rsvio::kBucket < (size_t)4 * n) nb *= 2;
        P.htable.assign((size_t)nb * rsvio::kBucket, rsvio::PnpEntry{rsvio::kEmptyId, {0.f, 0.f, 0.f}, 0u});
        P.bucket_mask = nb - 1;
        P.max_probe = 0;
        P.has_top = 0;
        for (int32_t i = 0; i < n; ++i) {
            if (ids[i] == rsvio::kEmptyId) {  // the one id the table cannot hold (the largest: last)
                P.has_top = 1;
                for (int k = 0; k < 3; ++k) P.top_pw[k] = p_W[3 * i + k];
                continue;
            }
            uint32_t b = rsvio::map_bucket(ids[i], P.bucket_mask);
            for (int probe = 0;; ++probe) {
                rsvio::PnpEntry* e = &P.htable[(size_t)b * rsvio::kBucket];
                int k = 0;
                while (k < rsvio::kBucket && e[k].id != rsvio::kEmptyId) ++k;
                if (k < rsvio::kBucket) {
                    e[k].id = ids[i];
                    for (int c = 0; c < 3; ++c) e[k].pw[c] = p_W[3 * i + c];
                    P.max_probe = std::max(P.max_probe, probe);
                    break;
                }
                b = (b + 1) & (uint32_t)P.bucket_mask;
            }
        }
        if (P.table.n < P.htable.size()) P.table.alloc(P.htable.size());
        RSVIO_HIP(hipMemcpyAsync(P.table.p, P.htable.data(), sizeof(rsvio::PnpEntry) * P.htable.size(),
                                 hipMemcpyHostToDevice, P.active()));
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
