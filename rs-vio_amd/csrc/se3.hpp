// se3.hpp -- device helpers shared by the BA (ba.hip) and the PnP motion tracker (pnp.hip):
// apex SE3 7-vector parsing, the LM's SE3 right-plus, Huber weights, and the deterministic
// wave reduction.  f64; the oracle (oracle/ba_oracle.cpp) states the same formulas.
#pragma once
#include <hip/hip_runtime.h>

namespace rsvio {

struct Pose {
    double R[3][3];
    double t[3];
};

// nalgebra UnitQuaternion::to_rotation_matrix after normalisation (apex SE3::from)
__device__ __forceinline__ Pose pose_from7(const double* p7) {
    double w = p7[3], x = p7[4], y = p7[5], z = p7[6];
    const double in = 1.0 / sqrt(w * w + x * x + y * y + z * z);  // one division, 4 products
    w *= in; x *= in; y *= in; z *= in;
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

// Coefficient k of the even power series in u = theta^2 used by se3_plus: (-1)^k / (4^k (2k)!)
// for cos(theta/2), (-1)^k / (2 4^k (2k+1)!) for sin(theta/2)/theta, (-1)^k / (2k+2)! for
// (1 - cos theta)/theta^2 and (-1)^k / (2k+3)! for (theta - sin theta)/theta^3.
constexpr double se3_series_coef(int which, int k) {
    double f = 1.0;  // the factorial
    const int n = which == 0 ? 2 * k : which == 1 ? 2 * k + 1 : which == 2 ? 2 * k + 2 : 2 * k + 3;
    for (int i = 2; i <= n; ++i) f *= (double)i;
    double q = 1.0;
    if (which <= 1)
        for (int i = 0; i < k; ++i) q *= 4.0;
    const double v = 1.0 / (f * q * (which == 1 ? 2.0 : 1.0));
    return (k & 1) ? -v : v;
}

template <int W>
__device__ __forceinline__ double se3_series(double u) {
    constexpr int kTerms = 8;  // u <= 1/16: the first omitted term is < 1e-24 of the sum
    double p = se3_series_coef(W, kTerms - 1);
#pragma unroll
    for (int k = kTerms - 2; k >= 0; --k) p = fma(p, u, se3_series_coef(W, k));
    return p;
}

// T (+) delta = T * Exp([rho; theta]) (same formula as oracle orc_se3_plus).  An LM step's
// rotation is small: for |theta| < 1/4 the four functions of theta it needs are even power
// series in theta^2 (no square root, sin/cos or division on the chain; within an ulp or two of
// the closed forms -- tolerance parity), and the product quaternion is normalised by a
// reciprocal square root refined by two Newton steps.
__device__ inline void se3_plus(const double* p7, const double* d, double* out) {
    const double* rho = d;
    const double* om = d + 3;
    double th2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
    double qd[4], A, Bc;
    if (th2 < 0.0625) {
        const double s = se3_series<1>(th2);  // sin(theta/2) / theta
        qd[0] = se3_series<0>(th2);           // cos(theta/2)
        qd[1] = s * om[0]; qd[2] = s * om[1]; qd[3] = s * om[2];
        A = se3_series<2>(th2);
        Bc = se3_series<3>(th2);
    } else {
        // one sincos of theta/2: sin(th) = 2 s c, 1 - cos(th) = 2 s^2 (same values as the
        // oracle's libm calls to within an ulp; tolerance parity)
        const double th = sqrt(th2);
        double sh, ch;
        sincos(0.5 * th, &sh, &ch);
        const double ith = 1.0 / th;
        const double s = sh * ith;
        qd[0] = ch; qd[1] = s * om[0]; qd[2] = s * om[1]; qd[3] = s * om[2];
        const double ith2 = ith * ith;
        A = 2.0 * sh * sh * ith2;
        Bc = (th - 2.0 * sh * ch) * ith2 * ith;
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
    const double n2 = qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3];
    const double h = 0.5 * n2;
    double inn = __builtin_amdgcn_rsq(n2);
    inn = inn * fma(-h * inn, inn, 1.5);
    inn = inn * fma(-h * inn, inn, 1.5);
    for (int i = 0; i < 4; ++i) out[3 + i] = qn[i] * inn;
}

__device__ __forceinline__ double rl64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Row-local DPP move of a double (both halves through the same lane permutation).
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Deterministic sum over the 64 lanes (all lanes active), returned to every lane: a fixed
// pairing inside each row of 16 (quad_perm xor 1, xor 2, half-row mirror, row mirror -- each
// step adds the same two values on both partners, so all 16 lanes agree bitwise), then the four
// row totals in row order.
__device__ __forceinline__ double wave_sum_det(double v) {
    v += dpp64<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp64<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp64<0x141>(v);  // row_half_mirror
    v += dpp64<0x140>(v);  // row_mirror
    return ((rl64(v, 0) + rl64(v, 16)) + rl64(v, 32)) + rl64(v, 48);
}

// 1/d, f64: hardware estimate (v_rcp_f64, ~2^-23 relative) + two Newton steps, the second
// folded into the correction: y1 = y0 + y0 e, e = 1 - d y0; y2 = y1 + y1 (1 - d y1) with
// 1 - d y1 = e^2 exactly up to rounding, so y2 = y0 (1 + e + e^2) -- full f64 precision with
// one fewer dependent step.
__device__ __forceinline__ double rcp_f64(double d) {
    const double y = __builtin_amdgcn_rcp(d);
    const double e = fma(-d, y, 1.0);
    return fma(y, fma(e, e, e), y);
}

// The correctly rounded f32 quotient a / b as RN_f32(a * (1/b)) in f64, 1/b = rcp_f64 (~2^-52
// relative): the f64 product is within 2^-51 of a / b, and a NORMAL f32 quotient of two f32 values
// is never a rounding midpoint nor within 2^-49 (relative) of one (|A 2^k - M B| >= 1 for the
// 24-bit significands A, B and a 25-bit midpoint M), so rounding the product to f32 gives exactly
// a / b (tests/test_div_rcp_cpu.py) -- with the reciprocal off the chain when b is known before a
// (the trackers: theta before its sine, a patch sum before the samples' products).
// Domain: |a / b| >= FLT_MIN (or 0).  A subnormal quotient has a shorter midpoint and CAN be an
// exact tie (e.g. (9 * 2^-149) / 6 = 1.5 * 2^-149), which RN(a * rcp(b)) may round the wrong way;
// the trackers' quotients (sin(theta) / theta, (1 - cos theta) / theta, nv v / sum over a patch of
// 8-bit intensities) never come near that range, so no guard sits on their chains.
__device__ __forceinline__ float div_rcp(float a, double rb) { return (float)((double)a * rb); }

// 1/sqrt(d), f64: hardware estimate + two Newton steps (y <- y (3 - d y^2) / 2)
__device__ __forceinline__ double rsqrt_f64(double d) {
    double y = __builtin_amdgcn_rsq(d);
    y = y * fma(-0.5 * d, y * y, 1.5);
    y = y * fma(-0.5 * d, y * y, 1.5);
    return y;
}

// Rigid inverse [R^T | -R^T t] of a row-major 4x4 transform (nalgebra try_inverse of a rigid
// T up to rounding; the oracle uses the same formula).
__host__ __device__ __forceinline__ void rigid_inverse(const double* T, double* Ti) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) Ti[4 * i + j] = T[4 * j + i];
        Ti[4 * i + 3] = -((T[i] * T[3] + T[4 + i] * T[7]) + T[8 + i] * T[11]);
    }
    Ti[12] = 0.0; Ti[13] = 0.0; Ti[14] = 0.0; Ti[15] = 1.0;
}

// UnitQuaternion::from_matrix for an orthonormal R (sliding_window.rs:221,511; same branch
// structure as oracle orc_quat_from_rotation), q = (w, x, y, z)
__device__ __forceinline__ void quat_from_rot(const double* R, double* q) {
    auto m = [&](int i, int j) { return R[3 * i + j]; };
    const double tr = m(0, 0) + m(1, 1) + m(2, 2);
    double w, x, y, z;
    if (tr > 0.0) {
        const double d = sqrt(tr + 1.0) * 2.0;
        w = 0.25 * d; x = (m(2, 1) - m(1, 2)) / d; y = (m(0, 2) - m(2, 0)) / d; z = (m(1, 0) - m(0, 1)) / d;
    } else if (m(0, 0) > m(1, 1) && m(0, 0) > m(2, 2)) {
        const double d = sqrt(1.0 + m(0, 0) - m(1, 1) - m(2, 2)) * 2.0;
        w = (m(2, 1) - m(1, 2)) / d; x = 0.25 * d; y = (m(0, 1) + m(1, 0)) / d; z = (m(0, 2) + m(2, 0)) / d;
    } else if (m(1, 1) > m(2, 2)) {
        const double d = sqrt(1.0 + m(1, 1) - m(0, 0) - m(2, 2)) * 2.0;
        w = (m(0, 2) - m(2, 0)) / d; x = (m(0, 1) + m(1, 0)) / d; y = 0.25 * d; z = (m(1, 2) + m(2, 1)) / d;
    } else {
        const double d = sqrt(1.0 + m(2, 2) - m(0, 0) - m(1, 1)) * 2.0;
        w = (m(1, 0) - m(0, 1)) / d; x = (m(0, 2) + m(2, 0)) / d; y = (m(1, 2) + m(2, 1)) / d; z = 0.25 * d;
    }
    q[0] = w; q[1] = x; q[2] = y; q[3] = z;
}

}  // namespace rsvio
