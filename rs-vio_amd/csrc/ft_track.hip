// ft_track.hip -- feature_tracker/ crate variant: f32 pyramid and bicubic SE(2) LK (gfx950).
//
// Replaces build_image_pyramid (feature_tracker/src/image_operations.rs:47-78), track_points /
// track_point / track_point_at_level / exp_se2 (feature_tracking.rs:16-219) and Patch52
// (patch.rs:57-255).  Bit-exact with oracle/ft_oracle.cpp: same f32 operations in the same
// order (-ffp-contract=off, correctly rounded divide/sqrt), sin/cos = glibc sinf/cosf restated (trig.hpp).
//
// Pyramid: one launch per level (each level is resized from the previous one); a workgroup owns
// a 64 x 8 output tile, the vertical pass over the tile's source-column span is staged in LDS
// (coalesced reads along x), the horizontal pass reads it back and clamps to [0, 1].
//
// LK: one 64-lane workgroup per feature runs forward and backward tracking.  Lane i < 52 owns
// pattern point i (its bicubic sample, template intensity and Jacobian row); every sum over
// the 52 points runs in the reference's order as a lane-ordered chain staged in LDS.
#include <cmath>
#include <stdexcept>

#include "ft.hpp"
#include "se3.hpp"
#include "trig.hpp"

namespace rsvio {
namespace ft {

namespace {

constexpr int NP = 52;
constexpr int TX = 64;
constexpr int TY = 8;

// ------------------------------------------------------------------------------------------
// host: level geometry and tap tables
// ------------------------------------------------------------------------------------------

// Rust f64::powi with a runtime exponent (compiler-rt __powidf2: square-and-multiply)
double powi_f64(double a, int b) {
    const bool recip = b < 0;
    double r = 1.0;
    for (;;) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1.0 / r : r;
}

inline float triangle_kernel(float x) {
    const float ax = std::fabs(x);
    return ax < 1.0f ? 1.0f - ax : 0.0f;
}

// image 0.25 sample.rs gaussian(x, r) = (sqrt(2 pi) r)^-1 exp(-x^2 / (2 r^2))
inline float gaussian_kernel(float x, float r) {
    const float a = 1.0f / (std::sqrt(2.0f * 3.14159265358979323846f) * r);
    return a * std::exp(-(x * x) / (2.0f * (r * r)));
}

// image 0.25 sample.rs {vertical,horizontal}_sample: taps of every output index of one pass
template <class K>
void build_taps(uint32_t in_len, uint32_t out_len, float support, K kernel, std::vector<int>& L,
                std::vector<int>& C, std::vector<int>& O, std::vector<float>& Wt) {
    const float ratio = (float)in_len / (float)out_len;
    const float sratio = ratio < 1.0f ? 1.0f : ratio;
    const float src_support = support * sratio;
    for (uint32_t o = 0; o < out_len; ++o) {
        float inputc = ((float)o + 0.5f) * ratio;
        long long left = (long long)std::floor(inputc - src_support);
        left = std::max<long long>(0, std::min<long long>(left, (long long)in_len - 1));
        long long right = (long long)std::ceil(inputc + src_support);
        right = std::max<long long>(left + 1, std::min<long long>(right, (long long)in_len));
        inputc = inputc - 0.5f;
        const size_t w0 = Wt.size();
        float sum = 0.0f;
        for (long long i = left; i < right; ++i) {
            const float wv = kernel(((float)i - inputc) / sratio);
            Wt.push_back(wv);
            sum += wv;
        }
        for (size_t k = w0; k < Wt.size(); ++k) Wt[k] /= sum;
        L.push_back((int)left);
        C.push_back((int)(right - left));
        O.push_back((int)w0);
    }
}

// ------------------------------------------------------------------------------------------
// device: resampling
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ft_resample_kernel(const float* __restrict__ src, int sw, int sh,
                                                          float* __restrict__ dst, int dw, int dh, TapsDev tv,
                                                          TapsDev th, int span) {
    extern __shared__ float tmp[];
    const int tiles_x = (dw + TX - 1) / TX;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int ox0 = tx * TX, ox1 = min(ox0 + TX, dw);
    const int oy0 = ty * TY, oy1 = min(oy0 + TY, dh);
    const int rows = oy1 - oy0, cols = ox1 - ox0;
    const int xl = th.left[ox0];
    const int ncols = th.left[ox1 - 1] + th.cnt[ox1 - 1] - xl;  // right edge is non-decreasing in o
    // vertical pass (no clamp): tmp[r][c] = sum_k src[vl + k][xl + c] * w_k, taps in order
    for (int idx = threadIdx.x; idx < rows * ncols; idx += blockDim.x) {
        const int r = idx / ncols, c = idx - r * ncols;
        const int oy = oy0 + r;
        const int vl = tv.left[oy], vc = tv.cnt[oy];
        const float* __restrict__ wv = tv.w + tv.woff[oy];
        const float* __restrict__ col = src + (size_t)vl * sw + xl + c;
        float acc = 0.0f;
        for (int k0 = 0; k0 < vc; k0 += 8) {
            float px[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) px[u] = (k0 + u < vc) ? col[(size_t)(k0 + u) * sw] : 0.0f;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (k0 + u < vc) acc += px[u] * wv[k0 + u];
        }
        tmp[r * span + c] = acc;
    }
    __syncthreads();
    // horizontal pass, clamped to [0, 1] (Primitive::DEFAULT_{MIN,MAX}_VALUE of f32)
    for (int idx = threadIdx.x; idx < rows * cols; idx += blockDim.x) {
        const int r = idx / cols, c = idx - r * cols;
        const int ox = ox0 + c;
        const int hl = th.left[ox] - xl, hc = th.cnt[ox];
        const float* __restrict__ wh = th.w + th.woff[ox];
        const float* row = tmp + r * span + hl;
        float acc = 0.0f;
        for (int k = 0; k < hc; ++k) acc += row[k] * wh[k];
        dst[(size_t)(oy0 + r) * dw + ox] = acc < 0.0f ? 0.0f : (acc > 1.0f ? 1.0f : acc);
    }
}

// ------------------------------------------------------------------------------------------
// device: LK
// ------------------------------------------------------------------------------------------

// patch.rs:258-278 -- Patch52::PATTERN_RAW (pixel offsets, unscaled)
__constant__ int8_t kPat[64][2] = {
    {-3, 7},  {-1, 7},  {1, 7},   {3, 7},   {-5, 5},  {-3, 5},  {-1, 5},  {1, 5},   {3, 5},
    {5, 5},   {-7, 3},  {-5, 3},  {-3, 3},  {-1, 3},  {1, 3},   {3, 3},   {5, 3},   {7, 3},
    {-7, 1},  {-5, 1},  {-3, 1},  {-1, 1},  {1, 1},   {3, 1},   {5, 1},   {7, 1},   {-7, -1},
    {-5, -1}, {-3, -1}, {-1, -1}, {1, -1},  {3, -1},  {5, -1},  {7, -1},  {-7, -3}, {-5, -3},
    {-3, -3}, {-1, -3}, {1, -3},  {3, -3},  {5, -3},  {7, -3},  {-5, -5}, {-3, -5}, {-1, -5},
    {1, -5},  {3, -5},  {5, -5},  {-3, -7}, {-1, -7}, {1, -7},  {3, -7}};

constexpr int kLd = 68;  // LDS row stride (floats) of the chain staging

// N sequential f32 sums over lanes 0..51 in lane order, chain i starting from init[i]
// (+0: `acc += x` from zero; -0: nalgebra gemv, whose first term is the bare product;
// lambda: the damped Hessian diagonal).  Lane i runs chain i alone from LDS; sums are broadcast
// by readlane, so every lane ends with the same values.
template <int N>
__device__ __forceinline__ void chains(const float (&v)[N], const float (&init)[N], float (&out)[N], float* sh,
                                       int lane) {
#pragma unroll
    for (int i = 0; i < N; ++i) sh[i * kLd + lane] = v[i];
    // chain i's start value rides in its row's padding column 64 (a per-lane select of init[]
    // was lowered to a scratch-memory array index, a spill round trip on every chain)
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) sh[i * kLd + 64] = init[i];
    }
    __builtin_amdgcn_wave_barrier();
    const int c = lane < N ? lane : 0;
    float acc = sh[c * kLd + 64];
    const float4* row = reinterpret_cast<const float4*>(sh + c * kLd);
    float4 xs[NP / 4];
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) xs[q] = row[q];
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) {
        const float4 x = xs[q];
        acc = acc + x.x;
        acc = acc + x.y;
        acc = acc + x.z;
        acc = acc + x.w;
    }
    // every row read issued before the first add (one LDS latency per chain, as lk_track.hip)
    __builtin_amdgcn_sched_group_barrier(0x100, NP / 4 + 1, 0);  // DS reads (+ the start value)
    __builtin_amdgcn_sched_group_barrier(0x002, NP, 0);          // the chain's VALU adds
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), i));
}

// image_operations.rs:231-282
__device__ __forceinline__ float bicubic_1d(float f0, float f1, float f2, float f3, float t) {
    const float a0 = f1;
    const float a1 = f2 - f0;
    const float a2 = 2.0f * f0 - 5.0f * f1 + 4.0f * f2 - f3;
    const float a3 = 3.0f * (f1 - f2) + f3 - f0;
    return a0 + 0.5f * (t * (a1 + t * (a2 + t * a3)));
}

__device__ __forceinline__ float d_bicubic_1d(float f0, float f1, float f2, float f3, float t, float& dt) {
    const float a0 = f1;
    const float a1 = f2 - f0;
    const float a2 = 2.0f * f0 - 5.0f * f1 + 4.0f * f2 - f3;
    const float a3 = 3.0f * (f1 - f2) + f3 - f0;
    dt = 0.5f * ((a1 + t * (2.0f * a2 + t * 3.0f * a3)));
    return a0 + 0.5f * (t * (a1 + t * (a2 + t * a3)));
}

// (1..=w.saturating_sub(3)).contains(&floor(x) as u32), same for y (image_operations.rs:150-154)
__device__ __forceinline__ bool bicubic_cell(float x, float y, uint32_t w, uint32_t h, uint32_t& xf, uint32_t& yf) {
    xf = sat_u32(floorf(x));
    yf = sat_u32(floorf(y));
    const uint32_t wm = w >= 3 ? w - 3 : 0, hm = h >= 3 ? h - 3 : 0;
    return xf >= 1 && xf <= wm && yf >= 1 && yf <= hm;
}

// interpolate_bicubic (image_operations.rs:140-176)
__device__ __forceinline__ bool bicubic(const float* __restrict__ im, uint32_t w, uint32_t h, float x, float y,
                                        float& out) {
    uint32_t xf, yf;
    if (!bicubic_cell(x, y, w, h, xf, yf)) return false;
    const float tx = x - (float)xf, ty = y - (float)yf;
    const float* p = im + (size_t)(yf - 1) * w + (xf - 1);
    float f[16];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) f[4 * r + c] = p[(size_t)r * w + c];
    const float y0 = bicubic_1d(f[0], f[1], f[2], f[3], tx);
    const float y1 = bicubic_1d(f[4], f[5], f[6], f[7], tx);
    const float y2 = bicubic_1d(f[8], f[9], f[10], f[11], tx);
    const float y3 = bicubic_1d(f[12], f[13], f[14], f[15], tx);
    out = bicubic_1d(y0, y1, y2, y3, ty);
    return true;
}

// d_interpolate_bicubic (image_operations.rs:181-229): value and (d/dx, d/dy)
__device__ __forceinline__ bool d_bicubic(const float* __restrict__ im, uint32_t w, uint32_t h, float x, float y,
                                          float& out, float& gx, float& gy) {
    uint32_t xf, yf;
    if (!bicubic_cell(x, y, w, h, xf, yf)) return false;
    const float tx = x - (float)xf, ty = y - (float)yf;
    const float* p = im + (size_t)(yf - 1) * w + (xf - 1);
    float fy[4], dfy[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float* q = p + (size_t)r * w;
        fy[r] = d_bicubic_1d(q[0], q[1], q[2], q[3], tx, dfy[r]);
    }
    float dty;
    out = d_bicubic_1d(fy[0], fy[1], fy[2], fy[3], ty, dty);
    const float d0 = 0.5f * (ty * (-1.0f + ty * (2.0f + ty * -1.0f)));
    const float d1 = 1.0f + 0.5f * (ty * (ty * (-5.0f + ty * 3.0f)));
    const float d2 = 0.5f * (ty * (1.0f + ty * (4.0f + ty * -3.0f)));
    const float d3 = 0.5f * (ty * (ty * (-1.0f + ty)));
    gx = d0 * dfy[0] + d1 * dfy[1] + d2 * dfy[2] + d3 * dfy[3];
    gy = dty;
    return true;
}

// image_operations.rs:4-7: x.is_positive() (sign bit clear) && y.is_positive() && in the image
__device__ __forceinline__ bool in_bounds(uint32_t w, uint32_t h, float x, float y) {
    return !signbit(x) && !signbit(y) && sat_u32(roundf(x)) < w && sat_u32(roundf(y)) < h;
}

// nalgebra Isometry2<f32>: UnitComplex (re, im) + translation
struct Iso {
    float re, im, tx, ty;
};

__device__ __forceinline__ Iso iso_identity() { return Iso{1.0f, 0.0f, 0.0f, 0.0f}; }

// Isometry * Isometry: t = t_a + R_a t_b, R = R_a R_b (complex product)
__device__ __forceinline__ Iso iso_mul(const Iso& a, const Iso& b) {
    Iso c;
    c.tx = a.tx + (a.re * b.tx - a.im * b.ty);
    c.ty = a.ty + (a.im * b.tx + a.re * b.ty);
    c.re = a.re * b.re - a.im * b.im;
    c.im = a.re * b.im + a.im * b.re;
    return c;
}

__device__ __forceinline__ void iso_apply(const Iso& a, float x, float y, float& ox, float& oy) {
    ox = (a.re * x - a.im * y) + a.tx;
    oy = (a.im * x + a.re * y) + a.ty;
}

// feature_tracking.rs:195-219, twist [theta, vx, vy]
__device__ __forceinline__ Iso exp_se2(float theta, float v0, float v1) {
    const double rth = rcp_f64((double)theta);  // beside sincosf (the quotients' divisor, se3.hpp div_rcp)
    float s, c;
    libm_trig::sincosf(theta, &s, &c);
    float diag, cross;
    if (fabsf(theta) > 1e-4f) {
        diag = div_rcp(s, rth);         // s / theta
        cross = div_rcp(1.0f - c, rth);  // (1 - c) / theta
    } else {
        const float th2 = theta * theta;
        diag = 1.0f - (theta * theta) / 6.0f;
        cross = (0.5f - th2 / 24.0f) * theta;
    }
    Iso e;
    e.tx = diag * v0 - cross * v1;
    e.ty = cross * v0 + diag * v1;
    e.re = c;
    e.im = s;
    return e;
}

// nalgebra Matrix3::try_inverse_mut (cofactor form)
__device__ __forceinline__ bool inverse3(const float m[3][3], float o[3][3]) {
    const float m11 = m[0][0], m12 = m[0][1], m13 = m[0][2];
    const float m21 = m[1][0], m22 = m[1][1], m23 = m[1][2];
    const float m31 = m[2][0], m32 = m[2][1], m33 = m[2][2];
    const float minor_m12_m23 = m22 * m33 - m32 * m23;
    const float minor_m11_m23 = m21 * m33 - m31 * m23;
    const float minor_m11_m22 = m21 * m32 - m31 * m22;
    const float det = m11 * minor_m12_m23 - m12 * minor_m11_m23 + m13 * minor_m11_m22;
    if (det == 0.0f) return false;
    o[0][0] = minor_m12_m23 / det;
    o[0][1] = (m13 * m32 - m33 * m12) / det;
    o[0][2] = (m12 * m23 - m22 * m13) / det;
    o[1][0] = -minor_m11_m23 / det;
    o[1][1] = (m11 * m33 - m31 * m13) / det;
    o[1][2] = (m13 * m21 - m23 * m11) / det;
    o[2][0] = minor_m11_m22 / det;
    o[2][1] = (m12 * m31 - m32 * m11) / det;
    o[2][2] = (m11 * m22 - m21 * m12) / det;
    return true;
}

struct Patch {
    float data;            // this lane's template intensity
    float J0, J1, J2;      // this lane's row of dr/dtwist
    float Hi[3][3];        // (lambda I + J^T J)^-1, uniform
};

// Patch52::new (patch.rs:240-255) with compute_intensities_and_jacobian_{ssd,lssd} (:119-216).
// When d_interpolate_bicubic misses (None) the reference keeps the previous point's gradient
// (dimg_dpixel is reused across the loop): such a lane takes the gradient of the nearest lower
// lane that hit, or zero.
__device__ bool make_patch(const float* __restrict__ im, uint32_t w, uint32_t h, float cx, float cy, int lane,
                           float lambda, int cost, Patch& P, float* sh) {
    const bool act = lane < NP;
    const float px = cx + (act ? (float)kPat[lane][0] : 0.0f);
    const float py = cy + (act ? (float)kPat[lane][1] : 0.0f);
    float v = 0.0f, g0 = 0.0f, g1 = 0.0f;
    const bool in = act && d_bicubic(im, w, h, px, py, v, g0, g1);
    if (!in) v = 0.0f;
    const unsigned long long hit = __ballot(in);
    const unsigned long long lower = hit & ((1ull << lane) - 1ull);
    const int src = lower ? 63 - __clzll((long long)lower) : 0;
    const float s0 = __shfl(g0, src), s1 = __shfl(g1, src);
    if (!in) {
        g0 = lower ? s0 : 0.0f;
        g1 = lower ? s1 : 0.0f;
    }
    float J0, J1, J2;
    if (cost == kSSD) {
        // (1x2) [[-py, 1, 0], [px, 0, 1]] by columns (gemv: g0 m0j, then g1 m1j + acc)
        J0 = g1 * px + g0 * (-py);
        J1 = g1 * 0.0f + g0 * 1.0f;
        J2 = g1 * 1.0f + g0 * 0.0f;
    } else {
        const float x3[3] = {act ? v : 0.0f, act ? g0 : 0.0f, act ? g1 : 0.0f};
        const float z3[3] = {0.0f, 0.0f, 0.0f};
        float s3[3];
        chains<3>(x3, z3, s3, sh, lane);
        const float mi = s3[0] / (float)NP, m0 = s3[1] / (float)NP, m1 = s3[2] / (float)NP;
        const float m2 = mi * mi;
        const float d0 = (g0 * mi - v * m0) / m2;
        const float d1 = (g1 * mi - v * m1) / m2;
        J0 = d1 * px + d0 * (-py);
        J1 = d1 * 0.0f + d0 * 1.0f;
        J2 = d1 * 1.0f + d0 * 0.0f;
    }
    if (!act) J0 = J1 = J2 = 0.0f;
    P.data = v;
    P.J0 = J0;
    P.J1 = J1;
    P.J2 = J2;
    // H = lambda I + J^T J: gemm accumulation k-ascending onto lambda I
    const float x6[6] = {J0 * J0, J0 * J1, J0 * J2, J1 * J1, J1 * J2, J2 * J2};
    const float i6[6] = {lambda, 0.0f, 0.0f, lambda, 0.0f, lambda};
    float h6[6];
    chains<6>(x6, i6, h6, sh, lane);
    const float H[3][3] = {{h6[0], h6[1], h6[2]}, {h6[1], h6[3], h6[4]}, {h6[2], h6[4], h6[5]}};
    return inverse3(H, P.Hi);
}

// track_point_at_level (feature_tracking.rs:129-192) with residuals_{ssd,lssd} (patch.rs:65-105)
__device__ bool track_level(const float* __restrict__ im1, uint32_t w, uint32_t h, const Patch& P, float cx,
                            float cy, int lane, Iso& X, int max_iter, int cost, float* sh) {
    const bool act = lane < NP;
    const float px = cx + (act ? (float)kPat[lane][0] : 0.0f);
    const float py = cy + (act ? (float)kPat[lane][1] : 0.0f);
    for (int it = 0; it < max_iter; ++it) {
        float x, y;
        iso_apply(X, px, py, x, y);
        float v = 0.0f;
        if (!(act && bicubic(im1, w, h, x, y, v))) v = 0.0f;
        float r;
        if (cost == kSSD) {
            r = v - P.data;
        } else {
            const float x1[1] = {act ? v : 0.0f};
            const float z1[1] = {0.0f};
            float s1[1];
            chains<1>(x1, z1, s1, sh, lane);
            const float mean = div_rcp(s1[0], 1.0 / NP);  // s1 / 52 (se3.hpp div_rcp)
            r = div_rcp(v, rcp_f64((double)mean)) - P.data;  // v / mean
        }
        if (!act) r = 0.0f;
        // b = J^T r (gemv: first term is the bare product -> chains start at -0)
        const float x3[3] = {P.J0 * r, P.J1 * r, P.J2 * r};
        const float z3[3] = {-0.0f, -0.0f, -0.0f};
        float b[3];
        chains<3>(x3, z3, b, sh, lane);
        float tw[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float acc = P.Hi[a][0] * b[0];
            acc = P.Hi[a][1] * b[1] + acc;
            acc = P.Hi[a][2] * b[2] + acc;
            tw[a] = acc;
        }
        X = iso_mul(X, exp_se2(-tw[0], -tw[1], -tw[2]));
        float ix, iy;
        iso_apply(X, cx, cy, ix, iy);
        if (!in_bounds(w, h, ix, iy)) return false;
        if (sqrtf(tw[0] * tw[0] + tw[1] * tw[1] + tw[2] * tw[2]) < 1e-3f) break;
    }
    return true;
}

// track_point (feature_tracking.rs:70-125): coarse to fine, pixel-centre level mapping
__device__ bool track_point(const float* __restrict__ p0, const float* __restrict__ p1, const PyrGeom& g, float fx,
                            float fy, int lane, int max_iter, float lambda, int cost, Iso& out, float* sh) {
    const float w = (float)g.w[0], h = (float)g.h[0];
    Iso X = iso_identity();
    for (int level = g.n - 1; level >= 0; --level) {
        const uint32_t lw = (uint32_t)g.w[level], lh = (uint32_t)g.h[level];
        const float sx = (float)lw / w, sy = (float)lh / h;
        const float lx = sx * (fx + 0.5f) - 0.5f, ly = sy * (fy + 0.5f) - 0.5f;
        Patch P;
        if (!make_patch(p0 + g.off[level], lw, lh, lx, ly, lane, lambda, cost, P, sh)) return false;
        if (!track_level(p1 + g.off[level], lw, lh, P, lx, ly, lane, X, max_iter, cost, sh)) return false;
        if (level > 0) {
            X.tx *= (float)g.w[level - 1] / (float)lw;
            X.ty *= (float)g.h[level - 1] / (float)lh;
        }
    }
    out = X;
    return true;
}

// track_points (feature_tracking.rs:16-61): forward, backward, ||centre - return|| < 2.0
__global__ __launch_bounds__(64) void ft_lk_kernel(LkLaunch L) {
    const int i = blockIdx.x;
    if (i >= L.n) return;
    __shared__ __attribute__((aligned(16))) float sh[6 * kLd];
    const int lane = threadIdx.x;
    const float fx = L.xy[i].x, fy = L.xy[i].y;
    Iso f;
    bool ok = track_point(L.pyr0, L.pyr1, L.g, fx, fy, lane, L.max_iter, L.lambda, L.cost, f, sh);
    float x1 = fx, y1 = fy;
    if (ok) {
        iso_apply(f, fx, fy, x1, y1);
        Iso b;
        ok = track_point(L.pyr1, L.pyr0, L.g, x1, y1, lane, L.max_iter, L.lambda, L.cost, b, sh);
        if (ok) {
            float xr, yr;
            iso_apply(b, x1, y1, xr, yr);
            const float dx = fx - xr, dy = fy - yr;
            ok = sqrtf(dx * dx + dy * dy) < 2.0f;
        }
    }
    if (lane == 0) {
        L.valid[i] = ok ? 1 : 0;
        L.xy_out[i] = ok ? make_float2(x1, y1) : make_float2(fx, fy);
        if (L.iso_out) L.iso_out[i] = ok ? make_float4(f.re, f.im, f.tx, f.ty) : make_float4(1.0f, 0.0f, 0.0f, 0.0f);
    }
}

}  // namespace

PyrGeom make_geom(int w, int h, int nlevels, double ratio) {
    if (nlevels < 1 || nlevels > kMaxLevels) throw std::invalid_argument("nlevels must be in [1, 8]");
    if (w < 4 || h < 4 || w > 65535 || h > 65535) throw std::invalid_argument("image size out of range");
    if (!(ratio > 0.0)) throw std::invalid_argument("ratio must be > 0");
    PyrGeom g{};
    g.n = nlevels;
    long off = 0;
    for (int l = 0; l < nlevels; ++l) {
        if (l == 0) {
            g.w[0] = w;
            g.h[0] = h;
        } else {
            const double p = powi_f64(ratio, l);
            g.w[l] = (int)std::round((double)w / p);
            g.h[l] = (int)std::round((double)h / p);
        }
        if (g.w[l] < 1 || g.h[l] < 1) throw std::invalid_argument("too many pyramid levels for the image size");
        g.off[l] = off;
        off += (long)g.w[l] * g.h[l];
    }
    g.total = off;
    return g;
}

void PyrPlan::init(int w, int h, int nlevels, double ratio, bool blur_on, float sigma) {
    g = make_geom(w, h, nlevels, ratio);
    blur = blur_on;
    std::vector<int> L, C, O;
    std::vector<float> Wt;
    auto tile_span = [&](int pass, int out_len) {
        int s = 0;
        for (int o0 = 0; o0 < out_len; o0 += TX) {
            const int o1 = std::min(o0 + TX, out_len) - 1;
            s = std::max(s, L[moff[pass] + o1] + C[moff[pass] + o1] - L[moff[pass] + o0]);
        }
        return s;
    };
    if (blur) {
        // imageops::blur: the resampler at the same size, Gaussian of support 2 sigma (sigma <= 0 -> 1)
        const float sg = sigma <= 0.0f ? 1.0f : sigma;
        auto gk = [sg](float x) { return gaussian_kernel(x, sg); };
        moff[0] = (int)L.size();
        build_taps((uint32_t)h, (uint32_t)h, 2.0f * sg, gk, L, C, O, Wt);
        moff[1] = (int)L.size();
        build_taps((uint32_t)w, (uint32_t)w, 2.0f * sg, gk, L, C, O, Wt);
        span[0] = tile_span(1, w);
    }
    for (int l = 1; l < g.n; ++l) {
        copy[l] = g.w[l] == g.w[l - 1] && g.h[l] == g.h[l - 1];
        if (copy[l]) continue;
        moff[2 * l] = (int)L.size();
        build_taps((uint32_t)g.h[l - 1], (uint32_t)g.h[l], 1.0f, triangle_kernel, L, C, O, Wt);
        moff[2 * l + 1] = (int)L.size();
        build_taps((uint32_t)g.w[l - 1], (uint32_t)g.w[l], 1.0f, triangle_kernel, L, C, O, Wt);
        span[l] = tile_span(2 * l + 1, g.w[l]);
    }
    n_meta = (int)L.size();
    for (int l = 0; l < g.n; ++l)
        if ((size_t)span[l] * TY * sizeof(float) > 64 * 1024) throw std::invalid_argument("resampling tile too wide");
    if (n_meta) {
        std::vector<int> m(3 * (size_t)n_meta);
        std::copy(L.begin(), L.end(), m.begin());
        std::copy(C.begin(), C.end(), m.begin() + n_meta);
        std::copy(O.begin(), O.end(), m.begin() + 2 * (size_t)n_meta);
        meta.alloc(m.size());
        wts.alloc(Wt.size());
        RSVIO_HIP(hipMemcpy(meta.p, m.data(), sizeof(int) * m.size(), hipMemcpyHostToDevice));
        RSVIO_HIP(hipMemcpy(wts.p, Wt.data(), sizeof(float) * Wt.size(), hipMemcpyHostToDevice));
    }
}

TapsDev PyrPlan::taps(int pass) const {
    TapsDev t;
    t.left = meta.p + moff[pass];
    t.cnt = meta.p + n_meta + moff[pass];
    t.woff = meta.p + 2 * (size_t)n_meta + moff[pass];
    t.w = wts.p;
    return t;
}

void enqueue_pyramid(const PyrPlan& P, const float* img, float* pyr, hipStream_t s) {
    const PyrGeom& g = P.g;
    auto resample = [&](const float* src, int sw, int sh, float* dst, int l) {
        const int dw = g.w[l], dh = g.h[l];
        const int tiles = ((dw + TX - 1) / TX) * ((dh + TY - 1) / TY);
        hipLaunchKernelGGL(ft_resample_kernel, dim3(tiles), dim3(256), sizeof(float) * TY * P.span[l], s, src, sw, sh,
                           dst, dw, dh, P.taps(2 * l), P.taps(2 * l + 1), P.span[l]);
        RSVIO_HIP(hipGetLastError());
    };
    if (P.blur)
        resample(img, g.w[0], g.h[0], pyr, 0);
    else
        RSVIO_HIP(hipMemcpyAsync(pyr, img, sizeof(float) * g.w[0] * g.h[0], hipMemcpyDeviceToDevice, s));
    for (int l = 1; l < g.n; ++l) {
        const float* src = pyr + g.off[l - 1];
        if (P.copy[l])
            RSVIO_HIP(hipMemcpyAsync(pyr + g.off[l], src, sizeof(float) * g.w[l] * g.h[l], hipMemcpyDeviceToDevice, s));
        else
            resample(src, g.w[l - 1], g.h[l - 1], pyr + g.off[l], l);
    }
}

void enqueue_lk(const LkLaunch& L, hipStream_t s) {
    if (L.n <= 0) return;
    hipLaunchKernelGGL(ft_lk_kernel, dim3(L.n), dim3(64), 0, s, L);
    RSVIO_HIP(hipGetLastError());
}

}  // namespace ft
}  // namespace rsvio
