// camera.hpp -- T12: Frame::add_left_feature / add_right_feature unprojection on device.
//
// Replaces camera_intrinsic_model 0.7.2 `CameraModel::unproject_one` as called from
// src/estimator/frame.rs:118-119 (left) and :131-132 (right), for the two models
// src/datasets/mod.rs:93-163 builds (OpenCVModel5 pinhole-radtan, EUCM).  The crate's source is
// not available offline; the algorithm restated here is the published one:
//   * OpenCVModel5: Newton iterations on the 2x2 radtan Jacobian from the distorted normalised
//     point, until the squared step drops below 1e-28 (<= max_iterations);
//   * EUCM: the closed form of Khomutenko et al. (2016), with the model's validity cone.
// Arithmetic is f64 with IEEE division / sqrt and no contraction (-ffp-contract=off), so the
// result is bit-exact with oracle/camera_oracle.cpp; the outputs are narrowed to f32 exactly as
// frame.rs:119 narrows them.
#pragma once
#include <hip/hip_runtime.h>

#include "rsvio_gpu.h"

namespace rsvio {

bool camera_ok(const rsvio_camera* c);  // camera.hip: model/convention/focal checks

struct Undist {
    float x, y;
    bool ok;
};

__device__ __forceinline__ Undist unproject_one(const rsvio_camera& cam, float u_f, float v_f) {
    const double u = (double)u_f, v = (double)v_f;
    const double* p = cam.params;
    const double mx = (u - p[2]) / p[0];
    const double my = (v - p[3]) / p[1];
    double x, y, z;
    bool ok;
    if (cam.model == RSVIO_CAM_EUCM) {
        const double alpha = p[4], beta = p[5];
        const double r2 = mx * mx + my * my;
        const double s = 1.0 - (2.0 * alpha - 1.0) * beta * r2;
        ok = !(alpha > 0.5 && s < 0.0);
        const double mz = (1.0 - beta * alpha * alpha * r2) / (alpha * sqrt(s) + (1.0 - alpha));
        x = mx;
        y = my;
        z = mz;
    } else {
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
            const double drad = k1 + r2 * (2.0 * k2 + r2 * (3.0 * k3));
            const double ex = x * rad + 2.0 * p1 * xy + p2 * (r2 + 2.0 * x2) - mx;
            const double ey = y * rad + p1 * (r2 + 2.0 * y2) + 2.0 * p2 * xy - my;
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
    if (cam.convention == RSVIO_UNPROJ_RAY) {
        const double n = sqrt(x * x + y * y + z * z);
        ox = x / n;
        oy = y / n;
    } else {
        ok = ok && z > 0.0;
        ox = x / z;
        oy = y / z;
    }
    ok = ok && isfinite(ox) && isfinite(oy);
    Undist r;
    r.x = ok ? (float)ox : __builtin_nanf("");
    r.y = ok ? (float)oy : __builtin_nanf("");
    r.ok = ok;
    return r;
}

}  // namespace rsvio
