// ba_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see rsvio_oracle.h).
//
// Scalar f64 restatement of the reference sliding-window bundle adjustment:
//   * the residual / analytic Jacobian of BundleAdjustmentFactor::linearize
//     (src/optimization/factors.rs:350-447),
//   * Huber(2.0) robustification (src/estimator/sliding_window.rs:295-296),
//   * the Schur-complement LM of apex-solver (LevenbergMarquardt + SparseSchurComplement,
//     sliding_window.rs:126-135,325).  apex-solver is an unpinned git dependency that is
//     not on disk; its LM is restated as documented in DESIGN.md ("BA LM definition").
// Accumulation order is sequential: landmarks ascending, observations of a landmark
// sorted by (kf, cam).
#include "pool.hpp"
#include "rsvio_oracle.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <limits>
#include <cstring>
#include <numeric>
#include <thread>
#include <vector>

namespace {

enum {
    LM_COST_TOL = 1,
    LM_PARAM_TOL = 2,
    LM_MAX_ITERS = 3,
    LM_TRUST_REGION = 4,
    LM_NUMERICAL_FAILURE = -1,
    LM_SKIPPED = -2,
    LM_LINEAR_SOLVE_FAILED = -3,
};

struct Pose {
    double R[3][3];
    double t[3];
};

// nalgebra UnitQuaternion::to_rotation_matrix after Quaternion normalisation (apex SE3::from)
Pose pose_from7(const double* p7) {
    double w = p7[3], x = p7[4], y = p7[5], z = p7[6];
    double n = std::sqrt(w * w + x * x + y * y + z * z);
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

inline void mat3vec(const double R[3][3], const double* v, double* out) {
    for (int i = 0; i < 3; ++i) out[i] = (R[i][0] * v[0] + R[i][1] * v[1]) + R[i][2] * v[2];
}

// factors.rs:350-447. J: 2x9 row-major [dp_W | dt | dw]; returns false on cheirality failure.
bool linearize(const double* pW, const Pose& P, const double* TCB, const double* uv, double r[2],
               double J[2][9]) {
    double RCB[3][3] = {{TCB[0], TCB[1], TCB[2]}, {TCB[4], TCB[5], TCB[6]}, {TCB[8], TCB[9], TCB[10]}};
    double tCB[3] = {TCB[3], TCB[7], TCB[11]};
    double pB[3], pC[3], tmp[3];
    mat3vec(P.R, pW, tmp);
    for (int i = 0; i < 3; ++i) pB[i] = tmp[i] + P.t[i];
    mat3vec(RCB, pB, tmp);
    for (int i = 0; i < 3; ++i) pC[i] = tmp[i] + tCB[i];
    if (pC[2] <= 0.0) {
        r[0] = 1e6;
        r[1] = 1e6;
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 9; ++b) J[a][b] = 0.0;
        return false;
    }
    r[0] = pC[0] / pC[2] - uv[0];
    r[1] = pC[1] / pC[2] - uv[1];
    double iz = 1.0 / pC[2];
    double iz2 = iz * iz;
    double Jp[2][3] = {{iz, 0.0, -pC[0] * iz2}, {0.0, iz, -pC[1] * iz2}};
    double A[2][3], JpW[2][3], M[3][3], Jw[2][3];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) A[i][j] = (Jp[i][0] * RCB[0][j] + Jp[i][1] * RCB[1][j]) + Jp[i][2] * RCB[2][j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) JpW[i][j] = (A[i][0] * P.R[0][j] + A[i][1] * P.R[1][j]) + A[i][2] * P.R[2][j];
    // M = (-R_B_W) * skew(p_W); skew = [[0,-z,y],[z,0,-x],[-y,x,0]] (factors.rs:136-139)
    double S[3][3] = {{0.0, -pW[2], pW[1]}, {pW[2], 0.0, -pW[0]}, {-pW[1], pW[0], 0.0}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            M[i][j] = ((-P.R[i][0]) * S[0][j] + (-P.R[i][1]) * S[1][j]) + (-P.R[i][2]) * S[2][j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) Jw[i][j] = (A[i][0] * M[0][j] + A[i][1] * M[1][j]) + A[i][2] * M[2][j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) {
            J[i][j] = JpW[i][j];
            J[i][3 + j] = JpW[i][j];
            J[i][6 + j] = Jw[i][j];
        }
    return true;
}

// Huber (Ceres convention): rho(s) = s (s <= d^2), 2 d sqrt(s) - d^2 otherwise; weight = rho'(s)
inline void huber(double s, double d, double* rho, double* w) {
    double d2 = d * d;
    if (s <= d2) {
        *rho = s;
        *w = 1.0;
    } else {
        double rs = std::sqrt(s);
        *rho = 2.0 * d * rs - d2;
        *w = d / rs;
    }
}

// 3x3 symmetric inverse by the adjugate (shared formula with the GPU kernel)
bool inv3(const double A[3][3], double X[3][3]) {
    double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
    double c01 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
    double c02 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
    double det = A[0][0] * c00 + A[0][1] * c01 + A[0][2] * c02;
    if (!(det > 0.0) || !std::isfinite(det)) return false;
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

struct Problem {
    int n_kf, n_lm, n_obs;
    const uint8_t* kf_fixed;
    const double* TCB2;
    double delta;
    std::vector<int> free_idx;     // kf -> free block index or -1
    int n_free;
    std::vector<int> lm_ptr;       // CSR over sorted obs
    std::vector<int> order;        // sorted obs index
    const int32_t* obs_kf;
    const uint8_t* obs_cam;
    const double* obs_uv;
};

Problem make_problem(int n_kf, const uint8_t* kf_fixed, int n_lm, int n_obs, const int32_t* obs_lm,
                     const int32_t* obs_kf, const uint8_t* obs_cam, const double* obs_uv,
                     const double* TCB2, double delta) {
    Problem pr;
    pr.n_kf = n_kf; pr.n_lm = n_lm; pr.n_obs = n_obs;
    pr.kf_fixed = kf_fixed; pr.TCB2 = TCB2; pr.delta = delta;
    pr.obs_kf = obs_kf; pr.obs_cam = obs_cam; pr.obs_uv = obs_uv;
    pr.free_idx.assign(n_kf, -1);
    pr.n_free = 0;
    for (int k = 0; k < n_kf; ++k)
        if (!kf_fixed[k]) pr.free_idx[k] = pr.n_free++;
    pr.order.resize(n_obs);
    std::iota(pr.order.begin(), pr.order.end(), 0);
    std::stable_sort(pr.order.begin(), pr.order.end(), [&](int a, int b) {
        if (obs_lm[a] != obs_lm[b]) return obs_lm[a] < obs_lm[b];
        if (obs_kf[a] != obs_kf[b]) return obs_kf[a] < obs_kf[b];
        return obs_cam[a] < obs_cam[b];
    });
    pr.lm_ptr.assign(n_lm + 1, 0);
    for (int i = 0; i < n_obs; ++i) pr.lm_ptr[obs_lm[i] + 1] += 1;
    for (int l = 0; l < n_lm; ++l) pr.lm_ptr[l + 1] += pr.lm_ptr[l];
    return pr;
}

// Linearisation of the whole problem at (poses, points) and the Schur-reduced system.
struct LmBlock {
    double Vi[3][3];   // (V + lambda I)^-1
    double gp[3];
    std::vector<std::pair<int, std::array<double, 18>>> W;  // (free kf block, W 6x3 row-major)
};

struct System {
    int n;
    std::vector<double> S, b;  // n x n, n
    std::vector<double> gc;    // camera gradient (for the predicted decrease)
    std::vector<LmBlock> lms;
    double cost;
    bool ok;
};

// Threads of the BA restatement (orc_set_ba_threads; 1 = the sequential reference order).  With
// T > 1 the landmarks are split into R <= T contiguous ranges (at least kMinRange landmarks each)
// whose sums (S, b, g_c, U, cost, the step norms) are combined in range order -- the "threaded
// Schur variant" CPU leg of BASELINE.md; deterministic for a given (T, n), tolerance-equal to
// T = 1.  The ranges run as tasks of the persistent pool (pool.hpp): an LM iteration's several
// parallel passes pay no thread start.
int g_ba_threads = 1;
constexpr int kMinRange = 48;

template <class F>
void for_ranges(int n, int T, F&& f) {  // f(range index, begin, end) over R <= T contiguous ranges
    const int R = std::min(T, n / kMinRange);
    if (R <= 1) {
        f(0, 0, n);
        return;
    }
    orc::Pool::get().run(R, R, [&](int t) { f(t, (int)((long long)n * t / R), (int)((long long)n * (t + 1) / R)); });
}

double eval_cost(const Problem& pr, const std::vector<Pose>& poses, const double* pW) {
    if (g_ba_threads > 1) {
        std::vector<double> part(g_ba_threads, 0.0);
        for_ranges(pr.n_lm, g_ba_threads, [&](int t, int l0, int l1) {
            double c = 0.0;
            for (int l = l0; l < l1; ++l)
                for (int q = pr.lm_ptr[l]; q < pr.lm_ptr[l + 1]; ++q) {
                    int o = pr.order[q];
                    double r[2], J[2][9];
                    linearize(pW + 3 * l, poses[pr.obs_kf[o]], pr.TCB2 + 16 * pr.obs_cam[o], pr.obs_uv + 2 * o, r, J);
                    double s = r[0] * r[0] + r[1] * r[1], rho, w;
                    huber(s, pr.delta, &rho, &w);
                    c += 0.5 * rho;
                }
            part[t] = c;
        });
        double cost = 0.0;
        for (double c : part) cost += c;
        return cost;
    }
    double cost = 0.0;
    for (int l = 0; l < pr.n_lm; ++l) {
        for (int q = pr.lm_ptr[l]; q < pr.lm_ptr[l + 1]; ++q) {
            int o = pr.order[q];
            double r[2], J[2][9];
            linearize(pW + 3 * l, poses[pr.obs_kf[o]], pr.TCB2 + 16 * pr.obs_cam[o], pr.obs_uv + 2 * o, r, J);
            double s = r[0] * r[0] + r[1] * r[1], rho, w;
            huber(s, pr.delta, &rho, &w);
            cost += 0.5 * rho;
        }
    }
    return cost;
}

// landmarks [l0, l1) into sy's S, b, g_c, cost and U (the per-landmark blocks into lms)
void build_range(const Problem& pr, const std::vector<Pose>& poses, const double* pW, double lambda, int l0, int l1,
                 System& sy, std::vector<double>& U, std::vector<LmBlock>& lms) {
    const int n = sy.n;
    for (int l = l0; l < l1; ++l) {
        double V[3][3] = {{0}}, gp[3] = {0, 0, 0};
        LmBlock& B = lms[l];
        B.W.clear();
        for (int q = pr.lm_ptr[l]; q < pr.lm_ptr[l + 1]; ++q) {
            int o = pr.order[q];
            int kf = pr.obs_kf[o];
            double r[2], J[2][9];
            linearize(pW + 3 * l, poses[kf], pr.TCB2 + 16 * pr.obs_cam[o], pr.obs_uv + 2 * o, r, J);
            double s = r[0] * r[0] + r[1] * r[1], rho, w;
            huber(s, pr.delta, &rho, &w);
            sy.cost += 0.5 * rho;
            double wr[2] = {w * r[0], w * r[1]};
            for (int a = 0; a < 3; ++a) {
                for (int c = 0; c < 3; ++c) V[a][c] += w * (J[0][a] * J[0][c] + J[1][a] * J[1][c]);
                gp[a] += J[0][a] * wr[0] + J[1][a] * wr[1];
            }
            int fb = pr.free_idx[kf];
            if (fb < 0) continue;
            if (B.W.empty() || B.W.back().first != fb) {
                std::array<double, 18> z{};
                B.W.push_back({fb, z});
            }
            auto& Wk = B.W.back().second;
            double* Uk = &U[(size_t)fb * 36];
            for (int a = 0; a < 6; ++a) {
                for (int c = 0; c < 3; ++c)
                    Wk[a * 3 + c] += w * (J[0][3 + a] * J[0][c] + J[1][3 + a] * J[1][c]);
                for (int c = 0; c < 6; ++c)
                    Uk[a * 6 + c] += w * (J[0][3 + a] * J[0][3 + c] + J[1][3 + a] * J[1][3 + c]);
                sy.gc[6 * fb + a] += J[0][3 + a] * wr[0] + J[1][3 + a] * wr[1];
            }
        }
        for (int a = 0; a < 3; ++a) V[a][a] += lambda;
        if (!inv3(V, B.Vi)) {
            sy.ok = false;
            for (int a = 0; a < 3; ++a)
                for (int c = 0; c < 3; ++c) B.Vi[a][c] = 0.0;
        }
        for (int a = 0; a < 3; ++a) B.gp[a] = gp[a];
        // Y_k = W_k Vi ; S_kk' -= Y_k W_k'^T ; b_k += Y_k gp
        std::array<double, 18> Y[64];  // <= 64 keyframes per landmark (the device's limit too)
        for (size_t i = 0; i < B.W.size(); ++i)
            for (int a = 0; a < 6; ++a)
                for (int c = 0; c < 3; ++c) {
                    const auto& Wk = B.W[i].second;
                    Y[i][a * 3 + c] = (Wk[a * 3 + 0] * B.Vi[0][c] + Wk[a * 3 + 1] * B.Vi[1][c]) + Wk[a * 3 + 2] * B.Vi[2][c];
                }
        for (size_t i = 0; i < B.W.size(); ++i) {
            int ki = B.W[i].first;
            for (size_t j = 0; j < B.W.size(); ++j) {
                int kj = B.W[j].first;
                const auto& Wj = B.W[j].second;
                for (int a = 0; a < 6; ++a)
                    for (int c = 0; c < 6; ++c) {
                        double v = (Y[i][a * 3 + 0] * Wj[c * 3 + 0] + Y[i][a * 3 + 1] * Wj[c * 3 + 1]) + Y[i][a * 3 + 2] * Wj[c * 3 + 2];
                        sy.S[(size_t)(6 * ki + a) * n + 6 * kj + c] -= v;
                    }
            }
            for (int a = 0; a < 6; ++a)
                sy.b[6 * ki + a] += (Y[i][a * 3 + 0] * gp[0] + Y[i][a * 3 + 1] * gp[1]) + Y[i][a * 3 + 2] * gp[2];
        }
    }
}

System build(const Problem& pr, const std::vector<Pose>& poses, const double* pW, double lambda) {
    System sy;
    int n = 6 * pr.n_free;
    sy.n = n;
    sy.S.assign((size_t)n * n, 0.0);
    sy.b.assign(n, 0.0);
    sy.gc.assign(n, 0.0);
    sy.lms.resize(pr.n_lm);
    sy.cost = 0.0;
    sy.ok = true;
    std::vector<double> U((size_t)pr.n_free * 36, 0.0);
    const int T = g_ba_threads;
    if (std::min(T, pr.n_lm / kMinRange) <= 1) {
        build_range(pr, poses, pW, lambda, 0, pr.n_lm, sy, U, sy.lms);
    } else {
        std::vector<System> part(T);
        std::vector<std::vector<double>> Up(T);
        for (int t = 0; t < T; ++t) {
            part[t].n = n;
            part[t].S.assign((size_t)n * n, 0.0);
            part[t].b.assign(n, 0.0);
            part[t].gc.assign(n, 0.0);
            part[t].cost = 0.0;
            part[t].ok = true;
            Up[t].assign((size_t)pr.n_free * 36, 0.0);
        }
        for_ranges(pr.n_lm, T, [&](int t, int l0, int l1) { build_range(pr, poses, pW, lambda, l0, l1, part[t], Up[t], sy.lms); });
        for (int t = 0; t < T; ++t) {  // range order
            for (size_t i = 0; i < sy.S.size(); ++i) sy.S[i] += part[t].S[i];
            for (int i = 0; i < n; ++i) {
                sy.b[i] += part[t].b[i];
                sy.gc[i] += part[t].gc[i];
            }
            for (size_t i = 0; i < U.size(); ++i) U[i] += Up[t][i];
            sy.cost += part[t].cost;
            sy.ok = sy.ok && part[t].ok;
        }
    }
    for (int f = 0; f < pr.n_free; ++f)
        for (int a = 0; a < 6; ++a) {
            for (int c = 0; c < 6; ++c) sy.S[(size_t)(6 * f + a) * n + 6 * f + c] += U[(size_t)f * 36 + a * 6 + c];
            sy.S[(size_t)(6 * f + a) * n + 6 * f + a] += lambda;
            sy.b[6 * f + a] -= sy.gc[6 * f + a];
        }
    return sy;
}

// The SparseCholesky fallback's system (sliding_window.rs:334-341): the FULL damped normal
// equations (H + lambda I) dx = -g, assembled densely and factored by a dense LL^T -- the
// oracle's independent restatement.  Unknowns are ordered [landmarks (3 each) | free poses (6
// each)]: the elimination order a fill-reducing sparse Cholesky gives the BA arrow matrix (the
// device eliminates the landmarks first with 3x3 LL^T blocks), so both fail on the same pivots.
// Returns the cost; H is N x N, g is N.
double build_full(const Problem& pr, const std::vector<Pose>& poses, const double* pW, double lambda,
                  std::vector<double>& H, std::vector<double>& g) {
    const int n = 6 * pr.n_free, m3 = 3 * pr.n_lm, N = n + m3;
    H.assign((size_t)N * N, 0.0);
    g.assign(N, 0.0);
    double cost = 0.0;
    for (int l = 0; l < pr.n_lm; ++l) {
        const int pl = 3 * l;
        for (int q = pr.lm_ptr[l]; q < pr.lm_ptr[l + 1]; ++q) {
            const int o = pr.order[q];
            const int kf = pr.obs_kf[o];
            double r[2], J[2][9];
            linearize(pW + 3 * l, poses[kf], pr.TCB2 + 16 * pr.obs_cam[o], pr.obs_uv + 2 * o, r, J);
            double s = r[0] * r[0] + r[1] * r[1], rho, w;
            huber(s, pr.delta, &rho, &w);
            cost += 0.5 * rho;
            const double wr[2] = {w * r[0], w * r[1]};
            // the observation's columns: point (3) then, for a free keyframe, the pose (6)
            int idx[9];
            int m = 3;
            for (int c = 0; c < 3; ++c) idx[c] = pl + c;
            const int fb = pr.free_idx[kf];
            if (fb >= 0) {
                for (int a = 0; a < 6; ++a) idx[3 + a] = m3 + 6 * fb + a;
                m = 9;
            }
            for (int a = 0; a < m; ++a) {
                for (int c = 0; c < m; ++c)
                    H[(size_t)idx[a] * N + idx[c]] += w * (J[0][a] * J[0][c] + J[1][a] * J[1][c]);
                g[idx[a]] += J[0][a] * wr[0] + J[1][a] * wr[1];
            }
        }
    }
    for (int i = 0; i < N; ++i) H[(size_t)i * N + i] += lambda;
    return cost;
}

// dense Cholesky solve (in place), returns false if not positive definite
bool chol_solve(std::vector<double> A, int n, const std::vector<double>& b, std::vector<double>& x) {
    for (int j = 0; j < n; ++j) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0) || !std::isfinite(d)) return false;
        double ljj = std::sqrt(d);
        A[(size_t)j * n + j] = ljj;
        for (int i = j + 1; i < n; ++i) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / ljj;
        }
    }
    x = b;
    for (int i = 0; i < n; ++i) {
        double s = x[i];
        for (int k = 0; k < i; ++k) s -= A[(size_t)i * n + k] * x[k];
        x[i] = s / A[(size_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = x[i];
        for (int k = i + 1; k < n; ++k) s -= A[(size_t)k * n + i] * x[k];
        x[i] = s / A[(size_t)i * n + i];
    }
    return true;
}

}  // namespace

extern "C" {

void orc_quat_from_rotation(const double* R, double* q) {
    auto m = [&](int i, int j) { return R[3 * i + j]; };
    double tr = m(0, 0) + m(1, 1) + m(2, 2);
    double w, x, y, z;
    if (tr > 0.0) {
        double d = std::sqrt(tr + 1.0) * 2.0;
        w = 0.25 * d; x = (m(2, 1) - m(1, 2)) / d; y = (m(0, 2) - m(2, 0)) / d; z = (m(1, 0) - m(0, 1)) / d;
    } else if (m(0, 0) > m(1, 1) && m(0, 0) > m(2, 2)) {
        double d = std::sqrt(1.0 + m(0, 0) - m(1, 1) - m(2, 2)) * 2.0;
        w = (m(2, 1) - m(1, 2)) / d; x = 0.25 * d; y = (m(0, 1) + m(1, 0)) / d; z = (m(0, 2) + m(2, 0)) / d;
    } else if (m(1, 1) > m(2, 2)) {
        double d = std::sqrt(1.0 + m(1, 1) - m(0, 0) - m(2, 2)) * 2.0;
        w = (m(0, 2) - m(2, 0)) / d; x = (m(0, 1) + m(1, 0)) / d; y = 0.25 * d; z = (m(1, 2) + m(2, 1)) / d;
    } else {
        double d = std::sqrt(1.0 + m(2, 2) - m(0, 0) - m(1, 1)) * 2.0;
        w = (m(1, 0) - m(0, 1)) / d; x = (m(0, 2) + m(2, 0)) / d; y = (m(1, 2) + m(2, 1)) / d; z = 0.25 * d;
    }
    q[0] = w; q[1] = x; q[2] = y; q[3] = z;
}

// nalgebra 0.33 UnitQuaternion::from_matrix(m) (sliding_window.rs:221,511; estimator.rs:209-211):
// Rotation3::from_matrix_eps(m, f64::EPSILON, 0, identity) -- Mueller et al.'s iteration
//   omega = sum_c r_c x m_c / (|sum_c r_c . m_c| + eps);  r <- AxisAngle(omega / |omega|, |omega|) r
// until |omega|^2 <= eps^2, then nalgebra's stationary-point check: perturb r by
// AxisAngle(axis, sqrt(eps)) (right product, repeated until ||m - r||_F^2 moves by > eps); a
// larger norm means a minimum (stop), else continue from the perturbed r with the axis
// swizzled .yzx() -- followed by UnitQuaternion::from_rotation_matrix.  Column-major matrices
// here (nalgebra's storage), so every sum runs in nalgebra's element order.
namespace {
struct M3 {
    double a[9];  // column-major: a[3 * c + r]
    double& operator()(int r, int c) { return a[3 * c + r]; }
    double operator()(int r, int c) const { return a[3 * c + r]; }
};
M3 m3_mul(const M3& A, const M3& B) {  // gemv per column: A[:,0] b0 + A[:,1] b1 + A[:,2] b2
    M3 C;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) C(r, c) = (A(r, 0) * B(0, c) + A(r, 1) * B(1, c)) + A(r, 2) * B(2, c);
    return C;
}
M3 m3_axis_angle(const double u[3], double ang) {  // Rotation3::from_axis_angle
    const double s = std::sin(ang), co = std::cos(ang), omc = 1.0 - co;
    M3 R;
    R(0, 0) = u[0] * u[0] + (1.0 - u[0] * u[0]) * co;
    R(0, 1) = u[0] * u[1] * omc - u[2] * s;
    R(0, 2) = u[0] * u[2] * omc + u[1] * s;
    R(1, 0) = u[0] * u[1] * omc + u[2] * s;
    R(1, 1) = u[1] * u[1] + (1.0 - u[1] * u[1]) * co;
    R(1, 2) = u[1] * u[2] * omc - u[0] * s;
    R(2, 0) = u[0] * u[2] * omc - u[1] * s;
    R(2, 1) = u[1] * u[2] * omc + u[0] * s;
    R(2, 2) = u[2] * u[2] + (1.0 - u[2] * u[2]) * co;
    return R;
}
double m3_dist2(const M3& A, const M3& B) {  // (A - B).norm_squared(), storage order
    double s = 0.0;
    for (int k = 0; k < 9; ++k) s += (A.a[k] - B.a[k]) * (A.a[k] - B.a[k]);
    return s;
}
}  // namespace

extern "C" void orc_quat_from_matrix(const double* Rrow, double* q) {
    const double eps = std::numeric_limits<double>::epsilon();
    const double dist = std::max(std::sqrt(eps), eps * eps);
    M3 m, r;
    for (int i = 0; i < 9; ++i) {
        m(i / 3, i % 3) = Rrow[i];
        r.a[i] = (i % 4 == 0) ? 1.0 : 0.0;
    }
    double pert[3] = {1.0, 0.0, 0.0};
    for (int guard = 0; guard < 100000; ++guard) {
        double w[3], den;
        {
            // sum over columns of cross(r_c, m_c) and dot(r_c, m_c), column order
            double cx[3][3], dt[3];
            for (int c = 0; c < 3; ++c) {
                cx[c][0] = r(1, c) * m(2, c) - r(2, c) * m(1, c);
                cx[c][1] = r(2, c) * m(0, c) - r(0, c) * m(2, c);
                cx[c][2] = r(0, c) * m(1, c) - r(1, c) * m(0, c);
                dt[c] = (r(0, c) * m(0, c) + r(1, c) * m(1, c)) + r(2, c) * m(2, c);
            }
            for (int k = 0; k < 3; ++k) w[k] = (cx[0][k] + cx[1][k]) + cx[2][k];
            den = (dt[0] + dt[1]) + dt[2];
        }
        const double scale = std::fabs(den) + eps;
        for (int k = 0; k < 3; ++k) w[k] = w[k] / scale;
        const double n2 = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
        if (n2 > eps * eps) {
            const double n = std::sqrt(n2);
            const double u[3] = {w[0] / n, w[1] / n, w[2] / n};
            r = m3_mul(m3_axis_angle(u, n), r);
            continue;
        }
        const double before = m3_dist2(m, r);
        M3 p = r;
        double after = before;
        do {
            p = m3_mul(p, m3_axis_angle(pert, dist));
            after = m3_dist2(m, p);
        } while (!(std::fabs(before - after) > eps));
        if (before < after) break;
        const double t = pert[0];
        pert[0] = pert[1];
        pert[1] = pert[2];
        pert[2] = t;
        r = p;
    }
    double R9[9];
    for (int i = 0; i < 9; ++i) R9[i] = r(i / 3, i % 3);
    orc_quat_from_rotation(R9, q);
}

// T (+) delta = T * Exp([rho; theta]) (right perturbation, translation-first tangent,
// matching the column order of factors.rs:437-441)
void orc_se3_plus(const double* p7, const double* d, double* out) {
    const double* rho = d;
    const double* om = d + 3;
    double th2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
    double th = std::sqrt(th2);
    double qd[4], A, Bc;  // V = I + A [w]x + Bc [w]x^2
    if (th < 1e-8) {
        qd[0] = 1.0; qd[1] = 0.5 * om[0]; qd[2] = 0.5 * om[1]; qd[3] = 0.5 * om[2];
        A = 0.5 - th2 / 24.0;
        Bc = 1.0 / 6.0 - th2 / 120.0;
    } else {
        double s = std::sin(0.5 * th) / th;
        qd[0] = std::cos(0.5 * th); qd[1] = s * om[0]; qd[2] = s * om[1]; qd[3] = s * om[2];
        A = (1.0 - std::cos(th)) / th2;
        Bc = (th - std::sin(th)) / (th2 * th);
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
    double qn[4] = {w0 * qd[0] - x0 * qd[1] - y0 * qd[2] - z0 * qd[3],
                    w0 * qd[1] + x0 * qd[0] + y0 * qd[3] - z0 * qd[2],
                    w0 * qd[2] - x0 * qd[3] + y0 * qd[0] + z0 * qd[1],
                    w0 * qd[3] + x0 * qd[2] - y0 * qd[1] + z0 * qd[0]};
    double nn = std::sqrt(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int i = 0; i < 4; ++i) out[3 + i] = qn[i] / nn;
}

void orc_ba_factor_linearize(const double* pW, const double* pose7, const double* TBW_fixed,
                             const double* TCB, const double* uv, double* r, double* J) {
    Pose P;
    if (pose7) {
        P = pose_from7(pose7);
    } else {
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) P.R[i][j] = TBW_fixed[4 * i + j];
            P.t[i] = TBW_fixed[4 * i + 3];
        }
    }
    double JJ[2][9];
    linearize(pW, P, TCB, uv, r, JJ);
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 9; ++b) J[a * 9 + b] = JJ[a][b];
}

int orc_ba_build_system(int n_kf, const double* pose7, const uint8_t* kf_fixed, int n_lm,
                        const double* p_W, int n_obs, const int32_t* obs_lm, const int32_t* obs_kf,
                        const uint8_t* obs_cam, const double* obs_uv, const double* TCB2,
                        double huber_delta, double lambda, double* S, double* b, double* cost) {
    Problem pr = make_problem(n_kf, kf_fixed, n_lm, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, TCB2, huber_delta);
    std::vector<Pose> poses(n_kf);
    for (int k = 0; k < n_kf; ++k) poses[k] = pose_from7(pose7 + 7 * k);
    System sy = build(pr, poses, p_W, lambda);
    memcpy(S, sy.S.data(), sizeof(double) * sy.S.size());
    memcpy(b, sy.b.data(), sizeof(double) * sy.b.size());
    *cost = sy.cost;
    return sy.ok ? 0 : -1;
}

void orc_set_ba_threads(int threads) { g_ba_threads = threads < 1 ? 1 : threads; }

int orc_ba_solve(int n_kf, double* pose7, const uint8_t* kf_fixed, int n_lm, double* p_W, int n_obs,
                 const int32_t* obs_lm, const int32_t* obs_kf, const uint8_t* obs_cam,
                 const double* obs_uv, const double* TCB2, const orc_lm_cfg* cfg, orc_ba_result* res) {
    Problem pr = make_problem(n_kf, kf_fixed, n_lm, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, TCB2, cfg->huber_delta);
    res->iterations = 0;
    // sliding_window.rs:303-319 guards
    int num_vars = n_kf + n_lm;  // every keyframe variable, KF_0 included (:217-226, :304)
    if (n_obs < 6 || n_obs < num_vars) {
        res->status = LM_SKIPPED;
        res->initial_cost = res->final_cost = 0.0;
        return 0;
    }
    std::vector<double> x7(pose7, pose7 + 7 * n_kf), pw(p_W, p_W + 3 * n_lm);
    std::vector<Pose> poses(n_kf);
    for (int k = 0; k < n_kf; ++k) poses[k] = pose_from7(&x7[7 * k]);
    double lambda = cfg->lambda_init, nu = 2.0;
    double cost = eval_cost(pr, poses, pw.data());
    res->initial_cost = cost;
    int status = LM_MAX_ITERS;
    int n = 6 * pr.n_free;
    std::vector<double> x7t(x7), pwt(pw), dc;
    for (int it = 0; it < cfg->max_iterations; ++it) {
        res->iterations = it + 1;
        System sy = build(pr, poses, pw.data(), lambda);
        if (!std::isfinite(sy.cost)) {
            status = LM_NUMERICAL_FAILURE;
            break;
        }
        double dx2 = 0.0, gdx = 0.0, x2 = 0.0;
        std::vector<double> dp(3 * (size_t)n_lm);
        if (cfg->linear_solver == 1) {
            // SparseCholesky fallback: the full damped system, solved densely
            std::vector<double> H, g, rhs, dx;
            build_full(pr, poses, pw.data(), lambda, H, g);
            const int N = n + 3 * n_lm;
            rhs.resize(N);
            for (int i = 0; i < N; ++i) rhs[i] = -g[i];
            if (!chol_solve(H, N, rhs, dx)) {  // Err(LinearSolveFailed): the caller reverts
                status = LM_LINEAR_SOLVE_FAILED;
                break;
            }
            const int m3 = 3 * n_lm;
            dc.assign(dx.begin() + m3, dx.end());
            for (int f = 0; f < n; ++f) {
                dx2 += dc[f] * dc[f];
                gdx += g[m3 + f] * dc[f];
            }
            for (int i = 0; i < m3; ++i) {
                dp[i] = dx[i];
                dx2 += dp[i] * dp[i];
                gdx += g[i] * dp[i];
            }
        } else {
        bool solved = sy.ok && chol_solve(sy.S, n, sy.b, dc);
        if (!solved) {  // Err(LinearSolveFailed / "Singular matrix"): sliding_window.rs:326-330 retries
            status = LM_LINEAR_SOLVE_FAILED;
            break;
        }
        // back substitution dp_l = Vi (-gp - sum_k W_k^T dc_k)
        for (int f = 0; f < n; ++f) {
            dx2 += dc[f] * dc[f];
            gdx += sy.gc[f] * dc[f];
        }
        {
            const int T = std::max(g_ba_threads, 1);
            std::vector<double> pdx(T, 0.0), pgd(T, 0.0);
            for_ranges(n_lm, T, [&](int t, int l0, int l1) {
                double d2 = 0.0, gd = 0.0;
                for (int l = l0; l < l1; ++l) {
                    const LmBlock& B = sy.lms[l];
                    double rhs[3] = {-B.gp[0], -B.gp[1], -B.gp[2]};
                    for (const auto& wk : B.W) {
                        const double* d6 = &dc[6 * wk.first];
                        for (int c = 0; c < 3; ++c) {
                            double s = 0.0;
                            for (int a = 0; a < 6; ++a) s += wk.second[a * 3 + c] * d6[a];
                            rhs[c] -= s;
                        }
                    }
                    for (int c = 0; c < 3; ++c) {
                        dp[3 * l + c] = (B.Vi[c][0] * rhs[0] + B.Vi[c][1] * rhs[1]) + B.Vi[c][2] * rhs[2];
                        if (T == 1) {  // the sequential reference order
                            dx2 += dp[3 * l + c] * dp[3 * l + c];
                            gdx += B.gp[c] * dp[3 * l + c];
                        } else {
                            d2 += dp[3 * l + c] * dp[3 * l + c];
                            gd += B.gp[c] * dp[3 * l + c];
                        }
                    }
                }
                pdx[t] = d2;
                pgd[t] = gd;
            });
            if (T > 1)
                for (int t = 0; t < T; ++t) {
                    dx2 += pdx[t];
                    gdx += pgd[t];
                }
        }
        }
        for (int k = 0; k < n_kf; ++k)
            if (!kf_fixed[k])
                for (int i = 0; i < 7; ++i) x2 += x7[7 * k + i] * x7[7 * k + i];
        for (double v : pw) x2 += v * v;
        double dxn = std::sqrt(dx2), xn = std::sqrt(x2);
        if (dxn <= cfg->parameter_tolerance * (xn + cfg->parameter_tolerance)) {
            status = LM_PARAM_TOL;
            break;
        }
        for (int k = 0; k < n_kf; ++k) {
            int f = pr.free_idx[k];
            if (f < 0) {
                for (int i = 0; i < 7; ++i) x7t[7 * k + i] = x7[7 * k + i];
            } else {
                orc_se3_plus(&x7[7 * k], &dc[6 * f], &x7t[7 * k]);
            }
        }
        for (size_t i = 0; i < pw.size(); ++i) pwt[i] = pw[i] + dp[i];
        std::vector<Pose> tposes(n_kf);
        for (int k = 0; k < n_kf; ++k) tposes[k] = pose_from7(&x7t[7 * k]);
        double new_cost = eval_cost(pr, tposes, pwt.data());
        double pred = 0.5 * (lambda * dx2 - gdx);
        double dcost = cost - new_cost;
        double rho = dcost / pred;
        if (std::isfinite(new_cost) && std::fabs(dcost) <= cfg->cost_tolerance * cost) {
            // converged: |change| within the tolerance whatever its sign; the candidate is not
            // applied (DESIGN.md section 5 -- a rounding-level change decides nothing).  This
            // build's rule, a deliberate departure: apex-solver's is absent offline (unpinned)
            status = LM_COST_TOL;
            break;
        }
        if (std::isfinite(new_cost) && rho > 0.0) {
            x7.swap(x7t);
            pw.swap(pwt);
            poses.swap(tposes);
            double f = 2.0 * rho - 1.0;
            lambda *= std::max(1.0 / 3.0, 1.0 - f * f * f);
            nu = 2.0;
            cost = new_cost;
        } else {
            lambda *= nu;
            nu *= 2.0;
            if (lambda > 1e32) {
                status = LM_TRUST_REGION;
                break;
            }
        }
    }
    res->status = status;
    res->final_cost = cost;
    memcpy(pose7, x7.data(), sizeof(double) * x7.size());
    memcpy(p_W, pw.data(), sizeof(double) * pw.size());
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// B8: SlidingWindow::track_motion (sliding_window.rs:490-587) + keyframe rule
// (estimator.rs:195-234).  PnPFactor::linearize (factors.rs:527-578): no cheirality guard.
static void pnp_linearize(const double* pW, const Pose& P, const double* TCB, const double* uv, double r[2],
                          double J[2][6]) {
    double RCB[3][3] = {{TCB[0], TCB[1], TCB[2]}, {TCB[4], TCB[5], TCB[6]}, {TCB[8], TCB[9], TCB[10]}};
    double pB[3], pC[3], tmp[3];
    mat3vec(P.R, pW, tmp);
    for (int i = 0; i < 3; ++i) pB[i] = tmp[i] + P.t[i];
    mat3vec(RCB, pB, tmp);
    pC[0] = tmp[0] + TCB[3];
    pC[1] = tmp[1] + TCB[7];
    pC[2] = tmp[2] + TCB[11];
    r[0] = pC[0] / pC[2] - uv[0];
    r[1] = pC[1] / pC[2] - uv[1];
    double iz = 1.0 / pC[2];
    double iz2 = iz * iz;
    double Jp[2][3] = {{iz, 0.0, -pC[0] * iz2}, {0.0, iz, -pC[1] * iz2}};
    double A[2][3], M[3][3];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) A[i][j] = (Jp[i][0] * RCB[0][j] + Jp[i][1] * RCB[1][j]) + Jp[i][2] * RCB[2][j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) J[i][j] = (A[i][0] * P.R[0][j] + A[i][1] * P.R[1][j]) + A[i][2] * P.R[2][j];
    double S[3][3] = {{0.0, -pW[2], pW[1]}, {pW[2], 0.0, -pW[0]}, {-pW[1], pW[0], 0.0}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            M[i][j] = ((-P.R[i][0]) * S[0][j] + (-P.R[i][1]) * S[1][j]) + (-P.R[i][2]) * S[2][j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) J[i][3 + j] = (A[i][0] * M[0][j] + A[i][1] * M[1][j]) + A[i][2] * M[2][j];
}

struct PnpObs {
    double pW[3], uv[2];
    int cam;
};

// H (6x6), g, cost over the factor list, sequentially in factor order
static void pnp_system(const std::vector<PnpObs>& obs, const Pose& P, const double* TCB2, double delta, double H[36],
                       double g[6], double* cost) {
    for (int k = 0; k < 36; ++k) H[k] = 0.0;
    for (int k = 0; k < 6; ++k) g[k] = 0.0;
    *cost = 0.0;
    for (const PnpObs& o : obs) {
        double r[2], J[2][6];
        pnp_linearize(o.pW, P, TCB2 + 16 * o.cam, o.uv, r, J);
        double s = r[0] * r[0] + r[1] * r[1], rho, w;
        huber(s, delta, &rho, &w);
        *cost += 0.5 * rho;
        double wr[2] = {w * r[0], w * r[1]};
        for (int a = 0; a < 6; ++a) {
            for (int c = 0; c < 6; ++c) H[a * 6 + c] += w * (J[0][a] * J[0][c] + J[1][a] * J[1][c]);
            g[a] += J[0][a] * wr[0] + J[1][a] * wr[1];
        }
    }
}

static void rigid_inverse(const double* T, double* Ti) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Ti[4 * i + j] = T[4 * j + i];
        Ti[4 * i + 3] = -((T[i] * T[3] + T[4 + i] * T[7]) + T[8 + i] * T[11]);
    }
    Ti[12] = 0.0; Ti[13] = 0.0; Ti[14] = 0.0; Ti[15] = 1.0;
}

// nalgebra Rotation3::euler_angles -> (roll, pitch, yaw), returned as its Euclidean norm
static double euler_norm(const double R[3][3]) {
    double roll, pitch, yaw;
    if (std::fabs(R[2][0]) < 1.0) {
        pitch = -std::asin(R[2][0]);
        double c = std::cos(pitch);
        roll = std::atan2(R[2][1] / c, R[2][2] / c);
        yaw = std::atan2(R[1][0] / c, R[0][0] / c);
    } else if (R[2][0] <= -1.0) {
        roll = std::atan2(R[0][1], R[0][2]);
        pitch = M_PI_2;
        yaw = 0.0;
    } else {
        roll = -std::atan2(-R[0][1], -R[0][2]);
        pitch = -M_PI_2;
        yaw = 0.0;
    }
    return std::sqrt((roll * roll + pitch * pitch) + yaw * yaw);
}

extern "C" int orc_track_motion(const uint64_t* ids_l, const float* uv_l, int n_l, const uint64_t* ids_r,
                                const float* uv_r, int n_r, const uint64_t* map_ids, const float* map_pw, int n_map,
                                const double* T_last, const double* TCB2, const orc_lm_cfg* cfg, double thr_t,
                                double thr_r, orc_motion_result* res) {
    // the factor list (sliding_window.rs:519-547): left then right, features with a map point;
    // map_points.get(id) restated as a search of the ascending id list
    std::vector<PnpObs> obs;
    for (int c = 0; c < 2; ++c) {
        const uint64_t* ids = c == 0 ? ids_l : ids_r;
        const float* uv = c == 0 ? uv_l : uv_r;
        int n = c == 0 ? n_l : n_r;
        for (int i = 0; i < n; ++i) {
            const uint64_t* it = std::lower_bound(map_ids, map_ids + n_map, ids[i]);
            if (it == map_ids + n_map || *it != ids[i]) continue;
            size_t k = (size_t)(it - map_ids);
            PnpObs o;
            for (int a = 0; a < 3; ++a) o.pW[a] = (double)map_pw[3 * k + a];  // point[a] as f64 (:530-535)
            o.uv[0] = (double)uv[2 * i];                                       // undistorted_coord cast (:529)
            o.uv[1] = (double)uv[2 * i + 1];
            o.cam = c;
            obs.push_back(o);
        }
    }
    res->n_observations = (int)obs.size();
    res->iterations = 0;
    res->initial_cost = res->final_cost = 0.0;
    res->translation_norm = res->rotation_norm = 0.0;
    // initial pose: the last keyframe's T_B_W (:506-517)
    double TBW0[16], x[7], xt[7];
    rigid_inverse(T_last, TBW0);
    double R0[9] = {TBW0[0], TBW0[1], TBW0[2], TBW0[4], TBW0[5], TBW0[6], TBW0[8], TBW0[9], TBW0[10]};
    x[0] = TBW0[3]; x[1] = TBW0[7]; x[2] = TBW0[11];
    orc_quat_from_matrix(R0, x + 3);  // UnitQuaternion::from_matrix (:511)
    int status = LM_MAX_ITERS;
    if (obs.empty()) {
        status = LM_SKIPPED;
    } else {
        double H[36], g[6], cost;
        pnp_system(obs, pose_from7(x), TCB2, cfg->huber_delta, H, g, &cost);
        res->initial_cost = cost;
        double lambda = cfg->lambda_init, nu = 2.0;
        for (int it = 0; it < cfg->max_iterations; ++it) {
            res->iterations = it + 1;
            if (!std::isfinite(cost)) {
                status = LM_NUMERICAL_FAILURE;
                break;
            }
            std::vector<double> A(H, H + 36), b(6), dx;
            for (int a = 0; a < 6; ++a) {
                A[a * 6 + a] += lambda;
                b[a] = -g[a];
            }
            if (!chol_solve(A, 6, b, dx)) {  // Err(LinearSolveFailed) -> Ok(None) (:554-560)
                status = LM_LINEAR_SOLVE_FAILED;
                break;
            }
            double dx2 = 0.0, gdx = 0.0, x2 = 0.0;
            for (int a = 0; a < 6; ++a) {
                dx2 += dx[a] * dx[a];
                gdx += g[a] * dx[a];
            }
            for (int a = 0; a < 7; ++a) x2 += x[a] * x[a];
            if (std::sqrt(dx2) <= cfg->parameter_tolerance * (std::sqrt(x2) + cfg->parameter_tolerance)) {
                status = LM_PARAM_TOL;
                break;
            }
            orc_se3_plus(x, dx.data(), xt);
            double Ht[36], gt[6], new_cost;
            pnp_system(obs, pose_from7(xt), TCB2, cfg->huber_delta, Ht, gt, &new_cost);
            double pred = 0.5 * (lambda * dx2 - gdx);
            double dcost = cost - new_cost;
            double rho = dcost / pred;
            if (std::isfinite(new_cost) && std::fabs(dcost) <= cfg->cost_tolerance * cost) {
                status = LM_COST_TOL;  // converged, the candidate not applied (as the BA above)
                break;
            }
            if (std::isfinite(new_cost) && rho > 0.0) {
                memcpy(x, xt, sizeof(x));
                memcpy(H, Ht, sizeof(H));
                memcpy(g, gt, sizeof(g));
                double f = 2.0 * rho - 1.0;
                lambda *= std::max(1.0 / 3.0, 1.0 - f * f * f);
                nu = 2.0;
                cost = new_cost;
            } else {
                lambda *= nu;
                nu *= 2.0;
                if (lambda > 1e32) {
                    status = LM_TRUST_REGION;
                    break;
                }
            }
        }
        res->final_cost = cost;
    }
    res->status = status;
    memcpy(res->pose7, x, sizeof(x));
    if (status > 0) {  // is_optimization_successful (:384-395)
        Pose P = pose_from7(x);
        double TBW[16], Tl_inv[16], Tr[16];
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) TBW[4 * i + j] = P.R[i][j];
            TBW[4 * i + 3] = P.t[i];
        }
        TBW[12] = 0.0; TBW[13] = 0.0; TBW[14] = 0.0; TBW[15] = 1.0;
        rigid_inverse(TBW, res->T_W_B);
        rigid_inverse(T_last, Tl_inv);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double s = 0.0;
                for (int k = 0; k < 4; ++k) s += res->T_W_B[4 * i + k] * Tl_inv[4 * k + j];
                Tr[4 * i + j] = s;
            }
        res->translation_norm = std::sqrt((Tr[3] * Tr[3] + Tr[7] * Tr[7]) + Tr[11] * Tr[11]);
        double Rr[9] = {Tr[0], Tr[1], Tr[2], Tr[4], Tr[5], Tr[6], Tr[8], Tr[9], Tr[10]};
        // UnitQuaternion::from_matrix(&R_rel).euler_angles() (estimator.rs:207-212): the unit
        // quaternion's to_rotation_matrix, no renormalisation
        double q[4];
        orc_quat_from_matrix(Rr, q);
        const double w = q[0], i = q[1], j = q[2], k = q[3];
        Pose Q;
        Q.R[0][0] = w * w + i * i - j * j - k * k; Q.R[0][1] = i * j * 2.0 - w * k * 2.0; Q.R[0][2] = w * j * 2.0 + i * k * 2.0;
        Q.R[1][0] = w * k * 2.0 + i * j * 2.0; Q.R[1][1] = w * w - i * i + j * j - k * k; Q.R[1][2] = j * k * 2.0 - w * i * 2.0;
        Q.R[2][0] = i * k * 2.0 - w * j * 2.0; Q.R[2][1] = w * i * 2.0 + j * k * 2.0; Q.R[2][2] = w * w - i * i - j * j + k * k;
        res->rotation_norm = euler_norm(Q.R);
        res->is_keyframe = (res->translation_norm > thr_t || res->rotation_norm > thr_r) ? 1 : 0;
    } else {  // estimator.rs:228-234: the frame stays a keyframe with T_W_B = I
        for (int k = 0; k < 16; ++k) res->T_W_B[k] = (k % 5 == 0) ? 1.0 : 0.0;
        res->is_keyframe = 1;
    }
    return 0;
}

