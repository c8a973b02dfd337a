// trig.hpp -- f32 sin/cos exactly as the reference's trackers get them (shared by lk_track.hip and
// ft_track.hip; also compiled on the host by tools/trig_exhaustive.cpp).
//
// Rust's f32::sin / f32::cos / f32::sin_cos lower to calls of glibc's sinf / cosf (or sincosf,
// when LLVM pairs them -- same bits, checked exhaustively) on x86-64 Linux.  The reference takes
// them in se2_exp_matrix through nalgebra's Rotation2::new (src/feature_tracker/
// image_utilities.rs:82-106) and in the crate's exp_se2 (feature_tracker/src/feature_tracker/
// feature_tracking.rs:195-219).  This header restates glibc 2.35's algorithm
// (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, s_sincosf.h, s_sincosf_data.c; the x86-64 ifunc
// picks the variant built with -mfma, whose GCC contraction turns every `a + b * c` of the
// polynomials and of the fast reduction into one fused multiply-add):
//   |y| < 2^-12           sin = y, cos = 1
//   |y| < pi/4            degree-7 odd / degree-8 even f64 polynomials in x = y
//   |y| < 120             n = round(y * 2/pi) by a 2^24-scaled truncation, x = y - n*pi/2 (fma)
//   finite |y| >= 120     Payne-Hanek with the 4/pi bit table (reduce_large), x = r * pi/2^62
// then the quadrant picks sin or cos polynomial and the signs.  Proven equal to this container's
// libm.so.6 (glibc 2.35, FMA host) for all 2^32 f32 inputs by tools/trig_exhaustive.cpp
// (profiles/r03_trig_exhaustive.txt; NaN payloads excepted), and the device build against libm by
// tests/test_trig_gpu.py (per-chunk digests over all 2^32 inputs).  The non-FMA variant differs
// from libm on 34 inputs (all |y| > 50), so the fused forms below are load-bearing.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RSVIO_TRIG_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define RSVIO_TRIG_HD static inline
#endif

namespace rsvio {
namespace libm_trig {

// s_sincosf_data.c: the first table; the second differs only by the sign of c0..c4, applied
// below as an exact negation of the cosine polynomial.
constexpr double kHpiInv = 0x1.45F306DC9C883p+23;  // 2/pi * 2^24
constexpr double kHpi = 0x1.921FB54442D18p0;       // pi/2
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
                 kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7,
                 kS3 = -0x1.994eb3774cf24p-13;
constexpr double kPi63 = 0x1.921FB54442D18p-62;  // pi/2 * 2^-62

RSVIO_TRIG_HD uint32_t f32_bits(float f) {
#if defined(__HIPCC__)
    return __float_as_uint(f);
#else
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
#endif
}

RSVIO_TRIG_HD double fmad(double a, double b, double c) {
#if defined(__HIPCC__)
    return __fma_rn(a, b, c);
#else
    return fma(a, b, c);
#endif
}

// 4/pi to 192 bits, 8 new bits per entry (s_sincosf_data.c __inv_pio4; the digits of 2/pi).
RSVIO_TRIG_HD uint32_t inv_pio4(int i) {
    switch (i) {
        case 0: return 0xa2u;          case 1: return 0xa2f9u;        case 2: return 0xa2f983u;
        case 3: return 0xa2f9836eu;    case 4: return 0xf9836e4eu;    case 5: return 0x836e4e44u;
        case 6: return 0x6e4e4415u;    case 7: return 0x4e441529u;    case 8: return 0x441529fcu;
        case 9: return 0x1529fc27u;    case 10: return 0x29fc2757u;   case 11: return 0xfc2757d1u;
        case 12: return 0x2757d1f5u;   case 13: return 0x57d1f534u;   case 14: return 0xd1f534ddu;
        case 15: return 0xf534ddc0u;   case 16: return 0x34ddc0dbu;   case 17: return 0xddc0db62u;
        case 18: return 0xc0db6295u;   case 19: return 0xdb629599u;   case 20: return 0x6295993cu;
        case 21: return 0x95993c43u;   case 22: return 0x993c4390u;   default: return 0x3c439041u;
    }
}

// s_sincosf.h reduce_large: |y| >= 120 (rare on the trackers' paths; kept for exactness).
RSVIO_TRIG_HD double reduce_large(uint32_t xi, int* np) {
    const int base = (int)((xi >> 26) & 15);
    const int shift = (int)((xi >> 23) & 7);
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * inv_pio4(base));
    const uint64_t res1 = (uint64_t)xi * inv_pio4(base + 4);
    const uint64_t res2 = (uint64_t)xi * inv_pio4(base + 8);
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * kPi63;
}

// sin and cos of y, bit-equal to glibc sinf(y) / cosf(y).
RSVIO_TRIG_HD void sincosf(float y, float* sinp, float* cosp) {
    const uint32_t top = (f32_bits(y) >> 20) & 0x7ffu;  // abstop12
    if (top < 0x398u) {                                   // |y| < 2^-12
        *sinp = y;
        *cosp = 1.0f;
        return;
    }
    double x = (double)y;
    int n = 0, q = 0;  // n: quadrant (picks the polynomial), q: quadrant for the signs / table
    if (top >= 0x3f4u) {      // |y| >= pi/4 (abstop12(0x1.921FB6p-1f))
        if (top < 0x42fu) {   // |y| < 120: reduce_fast
            const double r = x * kHpiInv;
            n = ((int32_t)r + 0x800000) >> 24;
            x = fmad(-(double)n, kHpi, x);
            q = n;
        } else if (top < 0x7f8u) {
            const uint32_t xi = f32_bits(y);
            const int sign = (int)(xi >> 31);
            x = reduce_large(xi, &n);
            q = n + sign;  // signs and table include y's sign; the polynomial choice does not
        } else {
            const float nan = y - y;
            *sinp = *cosp = nan / nan;
            return;
        }
        double sgn = (q & 1) ? -1.0 : 1.0;  // sign[q & 3] = {1, -1, -1, 1}
        sgn = (q & 2) ? -sgn : sgn;
        x = x * sgn;
    }
    const double x2 = x * x;
    // sin polynomial (sinf_poly, n even)
    const double x3 = x * x2;
    const double s1 = fmad(x2, kS3, kS2);
    const double x7 = x3 * x2;
    const double s = fmad(x3, kS1, x);
    const float sp = (float)fmad(x7, s1, s);
    // cos polynomial (sinf_poly, n odd); the second table (n & 2) negates c0..c4
    const double x4 = x2 * x2;
    const double c2 = fmad(x2, kC4, kC3);
    const double c1 = fmad(x2, kC1, kC0);
    const double x6 = x4 * x2;
    const double c = fmad(x4, kC2, c1);
    float cp = (float)fmad(x6, c2, c);
    cp = (q & 2) ? -cp : cp;
    *sinp = (n & 1) ? cp : sp;
    *cosp = (n & 1) ? sp : cp;
}

}  // namespace libm_trig
}  // namespace rsvio
