// trig.hpp -- f32 sin/cos as the trackers use them (shared by lk_track.hip and ft_track.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace rsvio {

// sin / cos of an f32 angle evaluated in f64 and rounded once to f32 (Rust's f32::sin_cos goes
// to libm; the oracle's trig mode 1 is the same rounding).  The trackers'
// increments are tiny, so |theta| < 1/16 takes a Taylor path (truncation < 1e-19 relative, i.e.
// the f64 value is within a few f64 ulp of the true one, as OCML's sin/cos are -- exhaustively
// checked equal to (float)sin((double)x) over that range); larger angles use OCML.
__device__ __forceinline__ void sincos_f64_rounded(float theta, float* s, float* c) {
    const double t = (double)theta;
    if (fabs(t) < 0.0625) {
        const double t2 = t * t;
        const double sp = -1.0 / 6.0 + t2 * (1.0 / 120.0 + t2 * (-1.0 / 5040.0 + t2 * (1.0 / 362880.0)));
        const double cp = -0.5 + t2 * (1.0 / 24.0 + t2 * (-1.0 / 720.0 + t2 * (1.0 / 40320.0 + t2 * (-1.0 / 3628800.0))));
        *s = (float)(t + t * (t2 * sp));
        *c = (float)(1.0 + t2 * cp);
    } else {
        *s = (float)sin(t);
        *c = (float)cos(t);
    }
}

}  // namespace rsvio
