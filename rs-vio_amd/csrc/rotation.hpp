// rotation.hpp -- host-side restatement of nalgebra 0.33's rotation extraction as the reference
// calls it: UnitQuaternion::from_matrix(&m) (src/estimator/sliding_window.rs:221,511 and
// src/estimator/estimator.rs:209-211) = UnitQuaternion::from_rotation_matrix(
// &Rotation3::from_matrix_eps(m, f64::EPSILON, 0, identity)).  from_matrix_eps is the iterative
// method of Mueller et al. ("A Robust Method to Extract the Rotational Part of Deformations"),
// including nalgebra's perturbation test for a stationary point that is a maximum.  Evaluation
// order follows nalgebra (gemv column accumulation, left-to-right sums, division by the norm);
// the library is compiled with -ffp-contract=off.  nalgebra is not vendored in the reference,
// so this restates its published source (parity unpinned against its bits).
#pragma once
#include <cmath>
#include <cstring>

namespace rsvio {
namespace rot {

constexpr double kEps = 2.220446049250313e-16;  // f64::EPSILON (nalgebra default_epsilon)

// row-major 3x3 helpers: m[3 * r + c]
inline double col(const double* m, int r, int c) { return m[3 * r + c]; }

// nalgebra Matrix3 * Matrix3: C[:, j] = A[:, 0] b0j, then += A[:, k] bkj (gemv / axpy order)
inline void mul(const double* A, const double* B, double* C) {
    double T[9];
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) {
            double s = A[3 * i] * B[j];
            s = s + A[3 * i + 1] * B[3 + j];
            s = s + A[3 * i + 2] * B[6 + j];
            T[3 * i + j] = s;
        }
    std::memcpy(C, T, sizeof T);
}

// Rotation3::from_axis_angle (unit axis u, angle a != 0)
inline void axis_angle(const double u[3], double a, double* R) {
    const double ux = u[0], uy = u[1], uz = u[2];
    const double sqx = ux * ux, sqy = uy * uy, sqz = uz * uz;
    const double s = std::sin(a), c = std::cos(a);
    const double omc = 1.0 - c;
    R[0] = sqx + (1.0 - sqx) * c;
    R[1] = ux * uy * omc - uz * s;
    R[2] = ux * uz * omc + uy * s;
    R[3] = ux * uy * omc + uz * s;
    R[4] = sqy + (1.0 - sqy) * c;
    R[5] = uy * uz * omc - ux * s;
    R[6] = ux * uz * omc - uy * s;
    R[7] = uy * uz * omc + ux * s;
    R[8] = sqz + (1.0 - sqz) * c;
}

// (m - r).norm_squared(): column-major sequential sum of squares
inline double diff_norm2(const double* m, const double* r) {
    double s = 0.0;
    for (int c = 0; c < 3; ++c)
        for (int i = 0; i < 3; ++i) {
            const double d = m[3 * i + c] - r[3 * i + c];
            s = s + d * d;
        }
    return s;
}

// Rotation3::from_matrix_eps(m, f64::EPSILON, max_iter = 0 (unbounded), identity)
inline void from_matrix(const double* m, double* rot) {
    constexpr int kMaxIter = 100000;  // nalgebra loops until convergence; a guard, never reached
    const double eps_dist = std::fmax(std::sqrt(kEps), kEps * kEps);
    double r[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double pax[3] = {1.0, 0.0, 0.0};  // perturbation axis (x, then .yzx() swizzles)
    for (int it = 0; it < kMaxIter; ++it) {
        double axis[3] = {0.0, 0.0, 0.0}, denom = 0.0;
        for (int c = 0; c < 3; ++c) {
            const double ax = col(r, 0, c), ay = col(r, 1, c), az = col(r, 2, c);
            const double bx = col(m, 0, c), by = col(m, 1, c), bz = col(m, 2, c);
            const double cr[3] = {ay * bz - az * by, az * bx - ax * bz, ax * by - ay * bx};
            const double dt = (ax * bx + ay * by) + az * bz;
            if (c == 0) {
                axis[0] = cr[0]; axis[1] = cr[1]; axis[2] = cr[2];
                denom = dt;
            } else {
                axis[0] = axis[0] + cr[0]; axis[1] = axis[1] + cr[1]; axis[2] = axis[2] + cr[2];
                denom = denom + dt;
            }
        }
        const double dd = std::fabs(denom) + kEps;
        const double aa[3] = {axis[0] / dd, axis[1] / dd, axis[2] / dd};
        // Unit::try_new_and_get(aa, eps): norm^2 > eps^2
        const double n2 = (aa[0] * aa[0] + aa[1] * aa[1]) + aa[2] * aa[2];
        if (n2 > kEps * kEps) {
            const double n = std::sqrt(n2);
            const double u[3] = {aa[0] / n, aa[1] / n, aa[2] / n};
            double A[9];
            axis_angle(u, n, A);
            mul(A, r, r);
            continue;
        }
        // stationary: a minimum of ||m - r|| unless a small perturbation lowers it
        double p[9];
        std::memcpy(p, r, sizeof p);
        const double nsq = diff_norm2(m, r);
        double nnew = nsq;
        for (int k = 0; k < kMaxIter; ++k) {
            double P[9];
            axis_angle(pax, eps_dist, P);
            mul(p, P, p);
            nnew = diff_norm2(m, p);
            if (std::fabs(nsq - nnew) > kEps) break;
        }
        if (nsq < nnew) break;
        const double t0 = pax[0];
        pax[0] = pax[1]; pax[1] = pax[2]; pax[2] = t0;  // yzx()
        std::memcpy(r, p, sizeof r);
    }
    std::memcpy(rot, r, sizeof r);
}

// UnitQuaternion::from_rotation_matrix -> (w, i, j, k)
inline void quat_from_rotation(const double* R, double* q) {
    auto m = [&](int i, int j) { return R[3 * i + j]; };
    const double tr = (m(0, 0) + m(1, 1)) + m(2, 2);
    double w, x, y, z;
    if (tr > 0.0) {
        const double d = std::sqrt(tr + 1.0) * 2.0;
        w = d * 0.25; x = (m(2, 1) - m(1, 2)) / d; y = (m(0, 2) - m(2, 0)) / d; z = (m(1, 0) - m(0, 1)) / d;
    } else if (m(0, 0) > m(1, 1) && m(0, 0) > m(2, 2)) {
        const double d = std::sqrt(((1.0 + m(0, 0)) - m(1, 1)) - m(2, 2)) * 2.0;
        w = (m(2, 1) - m(1, 2)) / d; x = d * 0.25; y = (m(0, 1) + m(1, 0)) / d; z = (m(0, 2) + m(2, 0)) / d;
    } else if (m(1, 1) > m(2, 2)) {
        const double d = std::sqrt(((1.0 + m(1, 1)) - m(0, 0)) - m(2, 2)) * 2.0;
        w = (m(0, 2) - m(2, 0)) / d; x = (m(0, 1) + m(1, 0)) / d; y = d * 0.25; z = (m(1, 2) + m(2, 1)) / d;
    } else {
        const double d = std::sqrt(((1.0 + m(2, 2)) - m(0, 0)) - m(1, 1)) * 2.0;
        w = (m(1, 0) - m(0, 1)) / d; x = (m(0, 2) + m(2, 0)) / d; y = (m(1, 2) + m(2, 1)) / d; z = d * 0.25;
    }
    q[0] = w; q[1] = x; q[2] = y; q[3] = z;
}

// UnitQuaternion::from_matrix (w, i, j, k)
inline void quat_from_matrix(const double* m, double* q) {
    double r[9];
    from_matrix(m, r);
    quat_from_rotation(r, q);
}

// UnitQuaternion::to_rotation_matrix (no renormalisation), q = (w, i, j, k)
inline void rotation_of_quat(const double* q, double* R) {
    const double w = q[0], i = q[1], j = q[2], k = q[3];
    const double ww = w * w, ii = i * i, jj = j * j, kk = k * k;
    const double ij = i * j * 2.0, wk = w * k * 2.0, wj = w * j * 2.0;
    const double ik = i * k * 2.0, jk = j * k * 2.0, wi = w * i * 2.0;
    R[0] = ((ww + ii) - jj) - kk; R[1] = ij - wk;                 R[2] = wj + ik;
    R[3] = wk + ij;               R[4] = ((ww - ii) + jj) - kk;   R[5] = jk - wi;
    R[6] = ik - wj;               R[7] = wi + jk;                 R[8] = ((ww - ii) - jj) + kk;
}

// Rotation3::euler_angles (roll, pitch, yaw) -> |(roll, pitch, yaw)| (estimator.rs:207-212,216)
inline double euler_norm(const double* R) {
    double roll, pitch, yaw;
    if (std::fabs(R[6]) < 1.0) {
        pitch = -std::asin(R[6]);
        const double c = std::cos(pitch);
        roll = std::atan2(R[7] / c, R[8] / c);
        yaw = std::atan2(R[3] / c, R[0] / c);
    } else if (R[6] <= -1.0) {
        roll = std::atan2(R[1], R[2]);
        pitch = M_PI_2;
        yaw = 0.0;
    } else {
        roll = -std::atan2(-R[1], -R[2]);
        pitch = -M_PI_2;
        yaw = 0.0;
    }
    return std::sqrt((roll * roll + pitch * pitch) + yaw * yaw);
}

}  // namespace rot
}  // namespace rsvio
