// camera_oracle.cpp -- TEST INFRASTRUCTURE, NOT PRODUCT CODE (see rsvio_oracle.h).
//
// CPU restatement of T12: `CameraModel::unproject_one` of camera-intrinsic-model 0.7.2
// (Cargo.toml:20; not available offline) as called by Frame::add_left_feature /
// add_right_feature (src/estimator/frame.rs:107-134), for the two models built by
// create_camera_models_from_config (src/datasets/mod.rs:93-163):
//   OpenCVModel5 params [fx, fy, cx, cy, k1, k2, p1, p2, k3] (mod.rs:118-128, k3 defaults 0)
//   EUCM         params [fx, fy, cx, cy, alpha, beta]        (mod.rs:102-110)
// plus the matching forward projections (used to build round-trip and config-5 inputs).
//
// Parity unpinned: the crate's unproject_one is not on disk and no reference test or fixture
// exercises it.  The restatement is the published algorithm:
//   radtan  -- Newton iterations on the 2x2 distortion Jacobian, started at the distorted
//              normalised point, stop when |step|^2 < 1e-28 or after max_iterations;
//   EUCM    -- Khomutenko, Garcia, Martinet (2016) closed form with the alpha > 1/2 cone.
// The return convention (plane x/z, y/z vs unit ray) is a parameter (rsvio_gpu.h).
// f64, -ffp-contract=off, IEEE division and sqrt; outputs narrowed to f32 like frame.rs:119.
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <limits>

#include "rsvio_oracle.h"

namespace {

bool unproject(const orc_camera& cam, float u_f, float v_f, float* ox_f, float* oy_f) {
    const double u = (double)u_f, v = (double)v_f;
    const double* p = cam.params;
    const double mx = (u - p[2]) / p[0];
    const double my = (v - p[3]) / p[1];
    double x, y, z;
    bool ok;
    if (cam.model == 1) {  // EUCM
        const double alpha = p[4], beta = p[5];
        const double r2 = mx * mx + my * my;
        const double s = 1.0 - (2.0 * alpha - 1.0) * beta * r2;
        ok = !(alpha > 0.5 && s < 0.0);
        const double mz = (1.0 - beta * alpha * alpha * r2) / (alpha * std::sqrt(s) + (1.0 - alpha));
        x = mx;
        y = my;
        z = mz;
    } else {  // OpenCVModel5
        const double k1 = p[4], k2 = p[5], p1 = p[6], p2 = p[7], k3 = p[8];
        const int max_it = cam.max_iterations > 0 ? cam.max_iterations : 20;
        x = mx;
        y = my;
        z = 1.0;
        ok = false;
        for (int it = 0; it < max_it; ++it) {
            const double x2 = x * x, y2 = y * y, xy = x * y;
            const double r2 = x2 + y2;
            const double rad = 1.0 + r2 * (k1 + r2 * (k2 + r2 * k3));
            const double drad = k1 + r2 * (2.0 * k2 + r2 * (3.0 * k3));  // d rad / d r2
            // residual of distort(x, y) - (mx, my)
            const double ex = x * rad + 2.0 * p1 * xy + p2 * (r2 + 2.0 * x2) - mx;
            const double ey = y * rad + p1 * (r2 + 2.0 * y2) + 2.0 * p2 * xy - my;
            // its Jacobian (symmetric off-diagonal)
            const double j00 = rad + 2.0 * x2 * drad + 2.0 * p1 * y + 6.0 * p2 * x;
            const double j01 = 2.0 * xy * drad + 2.0 * p1 * x + 2.0 * p2 * y;
            const double j11 = rad + 2.0 * y2 * drad + 6.0 * p1 * y + 2.0 * p2 * x;
            const double det = j00 * j11 - j01 * j01;
            const double dx = (j11 * ex - j01 * ey) / det;
            const double dy = (j00 * ey - j01 * ex) / det;
            x = x - dx;
            y = y - dy;
            if (dx * dx + dy * dy < 1e-28) {
                ok = true;
                break;
            }
        }
    }
    double ox, oy;
    if (cam.convention == 1) {  // unit ray
        const double n = std::sqrt(x * x + y * y + z * z);
        ox = x / n;
        oy = y / n;
    } else {  // normalised image plane
        ok = ok && z > 0.0;
        ox = x / z;
        oy = y / z;
    }
    ok = ok && std::isfinite(ox) && std::isfinite(oy);
    const float nan = std::numeric_limits<float>::quiet_NaN();
    *ox_f = ok ? (float)ox : nan;
    *oy_f = ok ? (float)oy : nan;
    return ok;
}

bool project(const orc_camera& cam, const double* P, double* uv) {
    const double* p = cam.params;
    const double X = P[0], Y = P[1], Z = P[2];
    if (cam.model == 1) {
        const double alpha = p[4], beta = p[5];
        const double d = std::sqrt(beta * (X * X + Y * Y) + Z * Z);
        const double den = alpha * d + (1.0 - alpha) * Z;
        if (!(den > 0.0)) return false;
        uv[0] = p[0] * (X / den) + p[2];
        uv[1] = p[1] * (Y / den) + p[3];
        return true;
    }
    if (!(Z > 0.0)) return false;
    const double x = X / Z, y = Y / Z;
    const double k1 = p[4], k2 = p[5], p1 = p[6], p2 = p[7], k3 = p[8];
    const double x2 = x * x, y2 = y * y, xy = x * y, r2 = x2 + y2;
    const double rad = 1.0 + r2 * (k1 + r2 * (k2 + r2 * k3));
    const double xd = x * rad + 2.0 * p1 * xy + p2 * (r2 + 2.0 * x2);
    const double yd = y * rad + p1 * (r2 + 2.0 * y2) + 2.0 * p2 * xy;
    uv[0] = p[0] * xd + p[2];
    uv[1] = p[1] * yd + p[3];
    return true;
}

}  // namespace

extern "C" {

int orc_unproject(const orc_camera* cam, const float* px, size_t n, float* out_xy, uint8_t* valid) {
    int n_ok = 0;
    for (size_t i = 0; i < n; ++i) {
        const bool ok = unproject(*cam, px[2 * i], px[2 * i + 1], out_xy + 2 * i, out_xy + 2 * i + 1);
        if (valid) valid[i] = ok ? 1 : 0;
        n_ok += ok ? 1 : 0;
    }
    return n_ok;
}

int orc_project(const orc_camera* cam, const double* pts, size_t n, double* out_uv, uint8_t* valid) {
    int n_ok = 0;
    for (size_t i = 0; i < n; ++i) {
        const bool ok = project(*cam, pts + 3 * i, out_uv + 2 * i);
        if (valid) valid[i] = ok ? 1 : 0;
        n_ok += ok ? 1 : 0;
    }
    return n_ok;
}

}  // extern "C"
