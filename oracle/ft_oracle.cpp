// ft_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see rsvio_oracle.h).
//
// Scalar C++ restatement of the standalone `feature_tracker/` crate of EthanD11/RS-VIO (the
// secondary tracker variant): f32 image pyramid with optional
// Gaussian pre-blur, bicubic inverse-compositional SE(2) LK with an LM-damped 3x3 system (SSD or
// LSSD cost), and Shi-Tomasi detection with non-maximum suppression.  Every floating-point
// expression keeps the reference's evaluation order; build with -ffp-contract=off.
//
// Third-party arithmetic restated from the published crates (no source offline -> parity
// unpinned):
//   image 0.25.9  imageops::resize(Triangle) / blur (separable resampler, f32 output clamped to
//                 [0, 1] = Primitive::DEFAULT_{MIN,MAX}_VALUE for f32), fast_blur (3 box passes)
//   imageproc 0.26 filter::{horizontal,vertical}_filter, suppress::local_maxima
//   nalgebra 0.34  Isometry2 / UnitComplex products, gemv/gemm accumulation order, 3x3 inverse
#include "rsvio_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

namespace {

constexpr int NP = 52;
constexpr float kPi = 3.14159265358979323846f;

// feature_tracker/src/patch.rs:258-278 -- Patch52::PATTERN_RAW (pixel offsets, unscaled :282)
const float PAT[NP][2] = {
    {-3, 7},  {-1, 7},  {1, 7},   {3, 7},   {-5, 5},  {-3, 5},  {-1, 5},  {1, 5},   {3, 5},
    {5, 5},   {-7, 3},  {-5, 3},  {-3, 3},  {-1, 3},  {1, 3},   {3, 3},   {5, 3},   {7, 3},
    {-7, 1},  {-5, 1},  {-3, 1},  {-1, 1},  {1, 1},   {3, 1},   {5, 1},   {7, 1},   {-7, -1},
    {-5, -1}, {-3, -1}, {-1, -1}, {1, -1},  {3, -1},  {5, -1},  {7, -1},  {-7, -3}, {-5, -3},
    {-3, -3}, {-1, -3}, {1, -3},  {3, -3},  {5, -3},  {7, -3},  {-5, -5}, {-3, -5}, {-1, -5},
    {1, -5},  {3, -5},  {5, -5},  {-3, -7}, {-1, -7}, {1, -7},  {3, -7}};

// Rust f32::sin / f32::cos (feature_tracking.rs:199-203) -> glibc sinf / cosf on x86-64 Linux.
inline void sin_cos(float th, float* s, float* c) {
    *s = sinf(th);
    *c = cosf(th);
}

// Rust `f32 as u32` saturates (NaN and negatives -> 0).
inline uint32_t sat_u32(float v) {
    if (!(v > 0.0f)) return 0u;
    if (v >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)v;
}

struct FImg {
    const float* p;
    uint32_t w, h;
    float at(uint32_t x, uint32_t y) const { return p[(size_t)y * w + x]; }
};

// ------------------------------------------------------------------------------------------
// Pyramid (image_operations.rs:47-78)
// ------------------------------------------------------------------------------------------

// Rust f64::powi with a runtime exponent (compiler-rt __powidf2: square-and-multiply).
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

// image_operations.rs:69-70: level l is round(w0 / ratio^l) x round(h0 / ratio^l)
void level_dims(int w0, int h0, int nlevels, double ratio, int* dims) {
    for (int l = 0; l < nlevels; ++l) {
        if (l == 0) {
            dims[0] = w0;
            dims[1] = h0;
            continue;
        }
        const double p = powi_f64(ratio, l);
        dims[2 * l] = (int)std::round((double)w0 / p);
        dims[2 * l + 1] = (int)std::round((double)h0 / p);
    }
}

// image 0.25 sample.rs filter taps for one output index (support already in kernel units).
struct Taps {
    int64_t left;
    std::vector<float> w;
};

template <class K>
Taps make_taps(int out_i, uint32_t in_len, uint32_t out_len, float support, K kernel) {
    const float ratio = (float)in_len / (float)out_len;
    const float sratio = ratio < 1.0f ? 1.0f : ratio;
    const float src_support = support * sratio;
    float inputc = ((float)out_i + 0.5f) * ratio;
    int64_t left = (int64_t)std::floor(inputc - src_support);
    left = std::max<int64_t>(0, std::min<int64_t>(left, (int64_t)in_len - 1));
    int64_t right = (int64_t)std::ceil(inputc + src_support);
    right = std::max<int64_t>(left + 1, std::min<int64_t>(right, (int64_t)in_len));
    inputc = inputc - 0.5f;
    Taps t;
    t.left = left;
    float sum = 0.0f;
    for (int64_t i = left; i < right; ++i) {
        const float wv = kernel(((float)i - inputc) / sratio);
        t.w.push_back(wv);
        sum += wv;
    }
    for (auto& wv : t.w) wv /= sum;
    return t;
}

inline float triangle_kernel(float x) {
    const float ax = std::fabs(x);
    return ax < 1.0f ? 1.0f - ax : 0.0f;
}

// image 0.25 sample.rs gaussian(x, r)
inline float gaussian_kernel(float x, float r) {
    const float a = 1.0f / (std::sqrt(2.0f * kPi) * r);
    return a * std::exp(-(x * x) / (2.0f * (r * r)));
}

// vertical_sample into an f32 buffer (no clamp), then horizontal_sample with the f32 clamp to
// [0, 1]; t += v * w in tap order.
template <class K>
void resample(const float* src, uint32_t w, uint32_t h, float* dst, uint32_t nw, uint32_t nh, float support,
              K kernel) {
    std::vector<float> tmp((size_t)w * nh);
    for (uint32_t oy = 0; oy < nh; ++oy) {
        const Taps t = make_taps((int)oy, h, nh, support, kernel);
        for (uint32_t x = 0; x < w; ++x) {
            float acc = 0.0f;
            for (size_t i = 0; i < t.w.size(); ++i) acc += src[(size_t)(t.left + (int64_t)i) * w + x] * t.w[i];
            tmp[(size_t)oy * w + x] = acc;
        }
    }
    for (uint32_t ox = 0; ox < nw; ++ox) {
        const Taps t = make_taps((int)ox, w, nw, support, kernel);
        for (uint32_t y = 0; y < nh; ++y) {
            float acc = 0.0f;
            for (size_t i = 0; i < t.w.size(); ++i) acc += tmp[(size_t)y * w + (size_t)(t.left + (int64_t)i)] * t.w[i];
            dst[(size_t)y * nw + ox] = acc < 0.0f ? 0.0f : (acc > 1.0f ? 1.0f : acc);
        }
    }
}

// imageops::resize(.., Triangle): a same-size resize is a copy.
void resize_triangle_f32(const float* src, uint32_t w, uint32_t h, float* dst, uint32_t nw, uint32_t nh) {
    if (nw == w && nh == h) {
        std::memcpy(dst, src, sizeof(float) * w * h);
        return;
    }
    resample(src, w, h, dst, nw, nh, 1.0f, triangle_kernel);
}

// imageops::blur(image, sigma): the resampler at the same size with a Gaussian of support 2 sigma.
void gaussian_blur_f32(const float* src, uint32_t w, uint32_t h, float sigma, float* dst) {
    if (!(sigma > 0.0f)) sigma = 1.0f;
    resample(src, w, h, dst, w, h, 2.0f * sigma, [sigma](float x) { return gaussian_kernel(x, sigma); });
}

// ------------------------------------------------------------------------------------------
// fast_blur (image 0.25 imageops::fast_blur; feature_detection.rs:122-124)
// ------------------------------------------------------------------------------------------
void boxes_for_gauss(float sigma, int n, int* out) {
    const float w_ideal = std::sqrt((12.0f * (sigma * sigma) / (float)n) + 1.0f);
    float w_l = std::floor(w_ideal);
    if (std::fmod(w_l, 2.0f) == 0.0f) w_l -= 1.0f;
    const float w_u = w_l + 2.0f;
    const float m_ideal = 0.25f * (float)n * (w_l + 3.0f) - 3.0f * (sigma * sigma) * (1.0f / (w_l + 1.0f));
    const int m = (int)std::round(m_ideal);
    for (int i = 0; i < n; ++i) out[i] = i < m ? (int)w_l : (int)w_u;
}

// One "horizontal_fast_blur_half": running box sum along each row, output transposed (h x w -> w x h).
void fast_blur_half(const float* s, size_t width, size_t height, size_t r, float* out) {
    auto ext = [&](long x, size_t row) {
        const long xc = std::max<long>(0, std::min<long>(x, (long)width - 1));
        return s[row * width + (size_t)xc];
    };
    const float den = 2.0f * (float)r + 1.0f;
    for (size_t row = 0; row < height; ++row) {
        float val = -0.0f;  // Rust float Sum starts from -0.0
        for (long x = -(long)r; x < (long)r + 1; ++x) val = val + ext(x, row);
        for (size_t col = 0; col < width; ++col) {
            float v = val / den;
            v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
            out[col * height + row] = v;
            val = val - ext((long)col - (long)r, row) + ext((long)(col + r + 1), row);
        }
    }
}

void fast_blur_f32(const float* src, uint32_t w, uint32_t h, float sigma, float* dst) {
    std::vector<float> a(src, src + (size_t)w * h), t((size_t)w * h);
    int boxes[3];
    boxes_for_gauss(sigma, 3, boxes);
    for (int k = 0; k < 3; ++k) {
        const size_t r = (size_t)(boxes[k] - 1) / 2;
        fast_blur_half(a.data(), w, h, r, t.data());
        fast_blur_half(t.data(), h, w, r, a.data());
    }
    std::memcpy(dst, a.data(), sizeof(float) * w * h);
}

// ------------------------------------------------------------------------------------------
// Bicubic interpolation (image_operations.rs:140-282)
// ------------------------------------------------------------------------------------------
inline float bicubic_1d(const float f[4], float t) {
    const float a0 = f[1];
    const float a1 = f[2] - f[0];
    const float a2 = 2.0f * f[0] - 5.0f * f[1] + 4.0f * f[2] - f[3];
    const float a3 = 3.0f * (f[1] - f[2]) + f[3] - f[0];
    return a0 + 0.5f * (t * (a1 + t * (a2 + t * a3)));
}

inline float d_bicubic_1d(const float f[4], float t, float* dt) {
    const float a0 = f[1];
    const float a1 = f[2] - f[0];
    const float a2 = 2.0f * f[0] - 5.0f * f[1] + 4.0f * f[2] - f[3];
    const float a3 = 3.0f * (f[1] - f[2]) + f[3] - f[0];
    *dt = 0.5f * ((a1 + t * (2.0f * a2 + t * 3.0f * a3)));
    return a0 + 0.5f * (t * (a1 + t * (a2 + t * a3)));
}

inline float d_bicubic_1d_full(const float f[4], float df[4], float t, float* dt) {
    const float r = d_bicubic_1d(f, t, dt);
    df[0] = 0.5f * (t * (-1.0f + t * (2.0f + t * -1.0f)));
    df[1] = 1.0f + 0.5f * (t * (t * (-5.0f + t * 3.0f)));
    df[2] = 0.5f * (t * (1.0f + t * (4.0f + t * -3.0f)));
    df[3] = 0.5f * (t * (t * (-1.0f + t)));
    return r;
}

// (1..=w.saturating_sub(3)).contains(&xf)
inline bool bicubic_inside(uint32_t xf, uint32_t yf, uint32_t w, uint32_t h) {
    const uint32_t wm = w >= 3 ? w - 3 : 0, hm = h >= 3 ? h - 3 : 0;
    return xf >= 1 && xf <= wm && yf >= 1 && yf <= hm;
}

bool interpolate_bicubic(const FImg& im, float x, float y, float* out) {
    const uint32_t xf = sat_u32(std::floor(x)), yf = sat_u32(std::floor(y));
    if (!bicubic_inside(xf, yf, im.w, im.h)) return false;
    const uint32_t xl = xf - 1, yl = yf - 1;
    const float tx = x - (float)xf, ty = y - (float)yf;
    float fy[4];
    for (uint32_t dy = 0; dy < 4; ++dy) {
        const float fx[4] = {im.at(xl, yl + dy), im.at(xl + 1, yl + dy), im.at(xl + 2, yl + dy), im.at(xl + 3, yl + dy)};
        fy[dy] = bicubic_1d(fx, tx);
    }
    *out = bicubic_1d(fy, ty);
    return true;
}

bool d_interpolate_bicubic(const FImg& im, float x, float y, float* out, float grad[2]) {
    const uint32_t xf = sat_u32(std::floor(x)), yf = sat_u32(std::floor(y));
    if (!bicubic_inside(xf, yf, im.w, im.h)) return false;
    const uint32_t xl = xf - 1, yl = yf - 1;
    const float tx = x - (float)xf, ty = y - (float)yf;
    float fy[4], dfy[4];
    for (uint32_t dy = 0; dy < 4; ++dy) {
        const float fx[4] = {im.at(xl, yl + dy), im.at(xl + 1, yl + dy), im.at(xl + 2, yl + dy), im.at(xl + 3, yl + dy)};
        fy[dy] = d_bicubic_1d(fx, tx, &dfy[dy]);
    }
    float dty, df[4];
    *out = d_bicubic_1d_full(fy, df, ty, &dty);
    grad[0] = df[0] * dfy[0] + df[1] * dfy[1] + df[2] * dfy[2] + df[3] * dfy[3];
    grad[1] = dty;
    return true;
}

// image_operations.rs:4-7: x.is_positive() (sign bit clear) && y.is_positive() && in image
inline bool in_bounds(uint32_t w, uint32_t h, float x, float y) {
    return !std::signbit(x) && !std::signbit(y) && sat_u32(std::round(x)) < w && sat_u32(std::round(y)) < h;
}

// ------------------------------------------------------------------------------------------
// SE(2) as nalgebra Isometry2<f32> {UnitComplex (re, im), translation}
// ------------------------------------------------------------------------------------------
struct Iso {
    float re = 1.0f, im = 0.0f, tx = 0.0f, ty = 0.0f;
};

// Isometry * Isometry: t = t_a + R_a t_b, R = R_a R_b (complex product)
inline Iso iso_mul(const Iso& a, const Iso& b) {
    Iso c;
    c.tx = a.tx + (a.re * b.tx - a.im * b.ty);
    c.ty = a.ty + (a.im * b.tx + a.re * b.ty);
    c.re = a.re * b.re - a.im * b.im;
    c.im = a.re * b.im + a.im * b.re;
    return c;
}

inline void iso_apply(const Iso& a, float x, float y, float* ox, float* oy) {
    *ox = (a.re * x - a.im * y) + a.tx;
    *oy = (a.im * x + a.re * y) + a.ty;
}

// feature_tracking.rs:195-219 -- exp_se2([theta, vx, vy])
Iso exp_se2(float theta, float v0, float v1) {
    float s, c;
    sin_cos(theta, &s, &c);
    float diag, cross;
    if (std::fabs(theta) > 1e-4f) {
        diag = s / theta;
        cross = (1.0f - c) / theta;
    } else {
        const float th2 = theta * theta;
        diag = 1.0f - (theta * theta) / 6.0f;
        cross = (0.5f - th2 / 24.0f) * theta;
    }
    Iso e;
    e.tx = diag * v0 - cross * v1;
    e.ty = cross * v0 + diag * v1;
    e.re = c;  // Isometry2::new -> UnitComplex::new(theta) = (cos, sin)
    e.im = s;
    return e;
}

// feature_tracking.rs:221-244 (test-only in the reference: the exp/log round trip KAT)
void log_se2(const Iso& T, float out[3]) {
    const float theta = std::atan2(T.im, T.re);
    float diag;
    if (std::fabs(theta) > 1e-3f) {
        float s, c;
        sin_cos(theta, &s, &c);
        diag = theta * s / (2.0f * (1.0f - c));
    } else {
        const float th2 = theta * theta;
        diag = (1.0f - th2 / 6.0f) / (1.0f - th2 / 12.0f);
    }
    const float cross = 0.5f * theta;
    out[0] = theta;
    out[1] = diag * T.tx + cross * T.ty;
    out[2] = -cross * T.tx + diag * T.ty;
}

// nalgebra Matrix3::try_inverse_mut (cofactor form); false when the determinant is zero.
bool inverse3(const float m[3][3], float o[3][3]) {
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

// ------------------------------------------------------------------------------------------
// Patch52 (patch.rs:107-255)
// ------------------------------------------------------------------------------------------
struct Patch {
    float cx, cy;
    float data[NP];
    float J[NP][3];
    float Hinv[3][3];
};

// patch.rs:119-216 (SSD / LSSD intensities and dr/dtwist); the gradient row keeps its previous
// value when d_interpolate_bicubic returns None (:154-158, :184-186).
void intensities_and_jacobian(const FImg& im, float cx, float cy, int cost, float data[NP], float J[NP][3]) {
    float g[2] = {0.0f, 0.0f};
    if (cost == 0) {
        for (int i = 0; i < NP; ++i) {
            const float px = cx + PAT[i][0], py = cy + PAT[i][1];
            float v;
            if (!d_interpolate_bicubic(im, px, py, &v, g)) v = 0.0f;
            data[i] = v;
            // (1x2) * [[-py, 1, 0], [px, 0, 1]] column by column (gemv: g0*m0j, then g1*m1j + acc)
            J[i][0] = g[1] * px + g[0] * (-py);
            J[i][1] = g[1] * 0.0f + g[0] * 1.0f;
            J[i][2] = g[1] * 1.0f + g[0] * 0.0f;
        }
        return;
    }
    float gi[NP][2];
    float mean_i = 0.0f, mg0 = 0.0f, mg1 = 0.0f;
    for (int i = 0; i < NP; ++i) {
        const float px = cx + PAT[i][0], py = cy + PAT[i][1];
        float v;
        if (!d_interpolate_bicubic(im, px, py, &v, g)) v = 0.0f;
        data[i] = v;
        gi[i][0] = g[0];
        gi[i][1] = g[1];
        mean_i += v;
        mg0 += g[0];
        mg1 += g[1];
    }
    mean_i /= (float)NP;
    mg0 /= (float)NP;
    mg1 /= (float)NP;
    const float m2 = mean_i * mean_i;
    for (int i = 0; i < NP; ++i) {
        const float px = cx + PAT[i][0], py = cy + PAT[i][1];
        const float d0 = (gi[i][0] * mean_i - data[i] * mg0) / m2;
        const float d1 = (gi[i][1] * mean_i - data[i] * mg1) / m2;
        J[i][0] = d1 * px + d0 * (-py);
        J[i][1] = d1 * 0.0f + d0 * 1.0f;
        J[i][2] = d1 * 1.0f + d0 * 0.0f;
    }
}

// patch.rs:240-255: H = lambda I + J^T J (gemm, k ascending from lambda I), then try_inverse.
bool patch_new(const FImg& im, float cx, float cy, float lambda, int cost, Patch& P) {
    P.cx = cx;
    P.cy = cy;
    intensities_and_jacobian(im, cx, cy, cost, P.data, P.J);
    float H[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            float acc = a == b ? lambda : 0.0f;
            for (int k = 0; k < NP; ++k) acc = P.J[k][a] * P.J[k][b] + acc;
            H[a][b] = acc;
        }
    return inverse3(H, P.Hinv);
}

// patch.rs:57-105
void residuals(const Patch& P, const FImg& im, const Iso& T, int cost, float r[NP]) {
    for (int i = 0; i < NP; ++i) {
        float x, y, v;
        iso_apply(T, P.cx + PAT[i][0], P.cy + PAT[i][1], &x, &y);
        if (!interpolate_bicubic(im, x, y, &v)) v = 0.0f;
        r[i] = v;
    }
    if (cost == 0) {
        for (int i = 0; i < NP; ++i) r[i] = r[i] - P.data[i];
        return;
    }
    float sum = 0.0f;
    for (int i = 0; i < NP; ++i) sum = sum + r[i];
    const float mean = sum / (float)NP;
    for (int i = 0; i < NP; ++i) r[i] = r[i] / mean - P.data[i];
}

// feature_tracking.rs:129-192
bool track_point_at_level(const FImg& im0, const FImg& im1, float fx, float fy, Iso& T, int max_iter,
                          float lambda, int cost) {
    Patch P;
    if (!patch_new(im0, fx, fy, lambda, cost, P)) return false;  // reference panics (:248-250)
    float r[NP];
    for (int it = 0; it < max_iter; ++it) {
        residuals(P, im1, T, cost, r);
        float b[3];
        for (int a = 0; a < 3; ++a) {
            float acc = P.J[0][a] * r[0];
            for (int k = 1; k < NP; ++k) acc = P.J[k][a] * r[k] + acc;
            b[a] = acc;
        }
        float tw[3];
        for (int a = 0; a < 3; ++a) {
            float acc = P.Hinv[a][0] * b[0];
            acc = P.Hinv[a][1] * b[1] + acc;
            acc = P.Hinv[a][2] * b[2] + acc;
            tw[a] = acc;
        }
        T = iso_mul(T, exp_se2(-tw[0], -tw[1], -tw[2]));
        float ix, iy;
        iso_apply(T, fx, fy, &ix, &iy);
        if (!in_bounds(im0.w, im0.h, ix, iy)) return false;
        const float n2 = tw[0] * tw[0] + tw[1] * tw[1] + tw[2] * tw[2];
        if (std::sqrt(n2) < 1e-3f) break;
    }
    return true;
}

struct Pyr {
    const float* base;
    std::vector<int> dims;  // 2 per level
    std::vector<size_t> off;
    FImg level(int l) const { return FImg{base + off[l], (uint32_t)dims[2 * l], (uint32_t)dims[2 * l + 1]}; }
    int levels() const { return (int)off.size(); }
};

Pyr make_pyr(const float* base, int w, int h, int nlevels, double ratio) {
    Pyr p;
    p.base = base;
    p.dims.resize(2 * nlevels);
    level_dims(w, h, nlevels, ratio, p.dims.data());
    size_t o = 0;
    for (int l = 0; l < nlevels; ++l) {
        p.off.push_back(o);
        o += (size_t)p.dims[2 * l] * p.dims[2 * l + 1];
    }
    return p;
}

// feature_tracking.rs:70-125
bool track_point(const Pyr& p0, const Pyr& p1, float fx, float fy, int max_iter, float lambda, int cost, Iso& out) {
    const float w = (float)p0.dims[0], h = (float)p0.dims[1];
    Iso T;
    for (int level = p0.levels() - 1; level >= 0; --level) {
        const FImg i0 = p0.level(level), i1 = p1.level(level);
        const float sx = (float)i0.w / w, sy = (float)i0.h / h;
        const float lx = sx * (fx + 0.5f) - 0.5f, ly = sy * (fy + 0.5f) - 0.5f;
        if (!track_point_at_level(i0, i1, lx, ly, T, max_iter, lambda, cost)) return false;
        if (level > 0) {
            const FImg n = p0.level(level - 1);
            T.tx *= (float)n.w / (float)i0.w;
            T.ty *= (float)n.h / (float)i0.h;
        }
    }
    out = T;
    return true;
}

// feature_tracking.rs:16-61 -- forward, backward, ||center - return|| < 2.0
bool track_feature(const Pyr& p0, const Pyr& p1, float fx, float fy, int max_iter, float lambda, int cost,
                   Iso& fwd) {
    if (!track_point(p0, p1, fx, fy, max_iter, lambda, cost, fwd)) return false;
    float x1, y1;
    iso_apply(fwd, fx, fy, &x1, &y1);
    Iso bwd;
    if (!track_point(p1, p0, x1, y1, max_iter, lambda, cost, bwd)) return false;
    float xr, yr;
    iso_apply(bwd, x1, y1, &xr, &yr);
    const float dx = fx - xr, dy = fy - yr;
    return std::sqrt(dx * dx + dy * dy) < 2.0f;
}

// ------------------------------------------------------------------------------------------
// Shi-Tomasi detection (feature_detection.rs:48-285)
// ------------------------------------------------------------------------------------------
void shi_tomasi_score(const FImg& im, float blur, float* score) {
    const uint32_t w = im.w, h = im.h;
    const size_t n = (size_t)w * h;
    std::vector<float> dxx(n), dyy(n), dxy(n);
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            // imageproc horizontal_filter / vertical_filter, kernel [-1, 0, 1], correlation with
            // clamp-to-edge: acc = 0 + p(-1)*(-1); acc += p(0)*0; acc += p(+1)*1
            const uint32_t xm = x > 0 ? x - 1 : 0, xp = x + 1 < w ? x + 1 : w - 1;
            const uint32_t ym = y > 0 ? y - 1 : 0, yp = y + 1 < h ? y + 1 : h - 1;
            float gx = 0.0f + im.at(xm, y) * -1.0f;
            gx = gx + im.at(x, y) * 0.0f;
            gx = gx + im.at(xp, y) * 1.0f;
            float gy = 0.0f + im.at(x, ym) * -1.0f;
            gy = gy + im.at(x, y) * 0.0f;
            gy = gy + im.at(x, yp) * 1.0f;
            const size_t i = (size_t)y * w + x;
            dxx[i] = gx * gx;
            dyy[i] = gy * gy;
            dxy[i] = gx * gy;
        }
    std::vector<float> bxx(n), byy(n), bxy(n);
    fast_blur_f32(dxx.data(), w, h, blur, bxx.data());
    fast_blur_f32(dyy.data(), w, h, blur, byy.data());
    fast_blur_f32(dxy.data(), w, h, blur, bxy.data());
    for (size_t i = 0; i < n; ++i) {
        const float trace = bxx[i] + byy[i];
        const float det = bxx[i] * byy[i] - bxy[i] * bxy[i];
        float delta = trace * trace - 4.0f * det;
        delta = delta > 0.0f ? delta : 0.0f;  // f32::max(x, 0.0) (NaN -> 0)
        score[i] = 500.0f * std::fabs(trace - std::sqrt(delta));
    }
}

struct Corner {
    uint32_t x, y;
    float score;
    bool past;
};

inline bool lex_less(uint32_t ax, uint32_t ay, uint32_t bx, uint32_t by) { return ax < bx || (ax == bx && ay < by); }

bool contains_greater(const float* s, uint32_t w, uint32_t x, uint32_t y, float v, uint32_t y0, uint32_t y1,
                      uint32_t x0, uint32_t x1) {
    for (uint32_t cy = y0; cy < y1; ++cy)
        for (uint32_t cx = x0; cx < x1; ++cx) {
            const float ci = s[(size_t)cy * w + cx];
            if (ci < v) continue;
            if (ci > v || lex_less(cx, cy, x, y)) return true;
        }
    return false;
}

// feature_detection.rs:171-253 (imageproc suppress_non_maximum adapted), radius r
std::vector<Corner> suppress_non_maximum(const float* s, uint32_t w, uint32_t h, uint32_t r, float thr) {
    std::vector<Corner> out;
    for (uint32_t y = 0; y < h; y += r + 1)
        for (uint32_t x = 0; x < w; x += r + 1) {
            uint32_t bx = x, by = y;
            float best = s[(size_t)y * w + x];
            for (uint32_t cy = y; cy < std::min(h, y + r + 1); ++cy)
                for (uint32_t cx = x; cx < std::min(w, x + r + 1); ++cx) {
                    const float ci = s[(size_t)cy * w + cx];
                    if (ci < best) continue;
                    if (ci > best || lex_less(cx, cy, bx, by)) {
                        bx = cx;
                        by = cy;
                        best = ci;
                    }
                }
            if (best >= thr) {
                const uint32_t x0 = bx >= r ? bx - r : 0, x1 = x, x2 = std::min(w, x + r + 1),
                               x3 = std::min(w, bx + r + 1);
                const uint32_t y0 = by >= r ? by - r : 0, y1 = y, y2 = std::min(h, y + r + 1),
                               y3 = std::min(h, by + r + 1);
                bool failed = contains_greater(s, w, bx, by, best, y0, y1, x0, x3);
                failed |= contains_greater(s, w, bx, by, best, y1, y2, x0, x1);
                failed |= contains_greater(s, w, bx, by, best, y1, y2, x2, x3);
                failed |= contains_greater(s, w, bx, by, best, y2, y3, x0, x3);
                if (!failed) out.push_back(Corner{bx, by, best, false});
            }
        }
    return out;
}

// imageproc 0.26 suppress::local_maxima: stable sort by (y, x); a point survives unless a point
// in rows [y-r, min(y+r+1, height)) and columns [x-r, x+r] has a greater score, or an equal score
// at a lexicographically smaller (y, x).  height = y of the last sorted point.
std::vector<Corner> local_maxima(const std::vector<Corner>& ts, uint32_t r) {
    std::vector<Corner> o(ts);
    std::stable_sort(o.begin(), o.end(), [](const Corner& a, const Corner& b) {
        return a.y < b.y || (a.y == b.y && a.x < b.x);
    });
    const uint32_t height = o.empty() ? 0 : o.back().y;
    std::vector<std::vector<const Corner*>> rows(height + 1);
    for (const auto& t : o) rows[t.y].push_back(&t);
    std::vector<Corner> out;
    for (const auto& t : o) {
        const uint32_t cx = t.x, cy = t.y;
        const float cs = t.score;
        bool is_max = true;
        const uint32_t lo = r > cy ? 0 : cy - r;
        const uint32_t hi = cy + r + 1 > height ? height : cy + r + 1;
        for (uint32_t y = lo; y < hi && is_max; ++y)
            for (const Corner* c : rows[y]) {
                if (c->x + r < cx) continue;
                if (c->x > cx + r) break;
                if (c->score > cs) { is_max = false; break; }
                if (c->score < cs) continue;
                if (c->y < cy || (c->y == cy && c->x < cx)) { is_max = false; break; }
            }
        if (is_max) out.push_back(t);
    }
    return out;
}

// feature_detection.rs:48-80 -> new corners (x, y) in (y, x) order
std::vector<Corner> add_points(const FImg& fine, const float* tracked_xy, int n_tracked, float threshold,
                               uint32_t min_dist, float blur) {
    std::vector<float> score((size_t)fine.w * fine.h);
    shi_tomasi_score(fine, blur, score.data());
    std::vector<Corner> corners = suppress_non_maximum(score.data(), fine.w, fine.h, 1, threshold);
    if (n_tracked > 0) {
        float mx = -std::numeric_limits<float>::infinity();
        for (const auto& c : corners) mx = std::fmax(mx, c.score);
        for (int i = 0; i < n_tracked; ++i)
            corners.push_back(Corner{sat_u32(std::round(tracked_xy[2 * i])), sat_u32(std::round(tracked_xy[2 * i + 1])),
                                     mx + 1.0f, true});
    }
    const std::vector<Corner> lm = local_maxima(corners, min_dist);
    std::vector<Corner> out;
    for (const auto& c : lm)
        if (!c.past && c.x >= min_dist && c.x < fine.w - min_dist && c.y >= min_dist && c.y < fine.h - min_dist)
            out.push_back(c);
    return out;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// FeatureTracker (feature_tracker.rs:51-185)
// ------------------------------------------------------------------------------------------
struct orc_ft {
    orc_ft_config cfg;
    int w, h;
    std::vector<int> dims;
    size_t pyr_floats = 0;
    bool has_prev = false;
    std::vector<float> prev_pyr;
    std::vector<uint64_t> ids;
    std::vector<float> xy;
    uint64_t last_id = 0;
};

extern "C" {

void orc_ft_level_dims(int w, int h, int nlevels, double ratio, int* dims) { level_dims(w, h, nlevels, ratio, dims); }

size_t orc_ft_pyramid_floats(int w, int h, int nlevels, double ratio) {
    std::vector<int> d(2 * nlevels);
    level_dims(w, h, nlevels, ratio, d.data());
    size_t n = 0;
    for (int l = 0; l < nlevels; ++l) n += (size_t)d[2 * l] * d[2 * l + 1];
    return n;
}

void orc_ft_resize_triangle(const float* src, int w, int h, float* dst, int nw, int nh) {
    resize_triangle_f32(src, w, h, dst, nw, nh);
}

void orc_ft_gaussian_blur(const float* src, int w, int h, float sigma, float* dst) {
    gaussian_blur_f32(src, w, h, sigma, dst);
}

void orc_ft_fast_blur(const float* src, int w, int h, float sigma, float* dst) { fast_blur_f32(src, w, h, sigma, dst); }

void orc_ft_boxes_for_gauss(float sigma, int n, int* out) { boxes_for_gauss(sigma, n, out); }

void orc_ft_build_pyramid(const float* img, int w, int h, int nlevels, double ratio, int blur, float sigma,
                          float* out) {
    Pyr p = make_pyr(out, w, h, nlevels, ratio);
    if (blur)
        gaussian_blur_f32(img, w, h, sigma, out);
    else
        std::memcpy(out, img, sizeof(float) * w * h);
    for (int l = 1; l < nlevels; ++l) {
        const FImg prev = p.level(l - 1);
        resize_triangle_f32(prev.p, prev.w, prev.h, out + p.off[l], p.dims[2 * l], p.dims[2 * l + 1]);
    }
}

int orc_ft_bicubic(const float* img, int w, int h, float x, float y, float* out3) {
    FImg im{img, (uint32_t)w, (uint32_t)h};
    float v, g[2] = {0.0f, 0.0f};
    if (!d_interpolate_bicubic(im, x, y, &v, g)) return 0;
    float v2;
    interpolate_bicubic(im, x, y, &v2);
    out3[0] = v2;
    out3[1] = g[0];
    out3[2] = g[1];
    return 1;
}

void orc_ft_exp_se2(const float* twist, float* out4) {
    const Iso e = exp_se2(twist[0], twist[1], twist[2]);
    out4[0] = e.re;
    out4[1] = e.im;
    out4[2] = e.tx;
    out4[3] = e.ty;
}

void orc_ft_log_se2(const float* iso4, float* out3) {
    Iso t;
    t.re = iso4[0];
    t.im = iso4[1];
    t.tx = iso4[2];
    t.ty = iso4[3];
    log_se2(t, out3);
}

int orc_ft_patch_new(const float* img, int w, int h, float cx, float cy, float lambda, int cost, float* data,
                     float* jac, float* hinv) {
    Patch P;
    FImg im{img, (uint32_t)w, (uint32_t)h};
    const bool ok = patch_new(im, cx, cy, lambda, cost, P);
    std::memcpy(data, P.data, sizeof(P.data));
    std::memcpy(jac, P.J, sizeof(P.J));
    std::memcpy(hinv, P.Hinv, sizeof(P.Hinv));
    return ok ? 1 : 0;
}

void orc_ft_track_points(const float* pyr0, const float* pyr1, int w, int h, int nlevels, double ratio,
                         const float* xy, int n, int max_iter, float lambda, int cost, float* iso_out,
                         uint8_t* valid) {
    const Pyr p0 = make_pyr(pyr0, w, h, nlevels, ratio), p1 = make_pyr(pyr1, w, h, nlevels, ratio);
    for (int i = 0; i < n; ++i) {
        Iso f;
        const bool ok = track_feature(p0, p1, xy[2 * i], xy[2 * i + 1], max_iter, lambda, cost, f);
        valid[i] = ok ? 1 : 0;
        iso_out[4 * i + 0] = ok ? f.re : 1.0f;
        iso_out[4 * i + 1] = ok ? f.im : 0.0f;
        iso_out[4 * i + 2] = ok ? f.tx : 0.0f;
        iso_out[4 * i + 3] = ok ? f.ty : 0.0f;
    }
}

void orc_ft_shi_tomasi_score(const float* img, int w, int h, float blur, float* score) {
    shi_tomasi_score(FImg{img, (uint32_t)w, (uint32_t)h}, blur, score);
}

int orc_ft_suppress_non_maximum(const float* score, int w, int h, int radius, float threshold, uint32_t* out_xy,
                                float* out_score, int cap) {
    const auto c = suppress_non_maximum(score, w, h, radius, threshold);
    const int n = (int)std::min<size_t>(c.size(), (size_t)cap);
    for (int i = 0; i < n; ++i) {
        out_xy[2 * i] = c[i].x;
        out_xy[2 * i + 1] = c[i].y;
        out_score[i] = c[i].score;
    }
    return (int)c.size();
}

int orc_ft_add_points(const float* fine, int w, int h, const float* tracked_xy, int n_tracked, float threshold,
                      int min_dist, float blur, uint32_t* out_xy, int cap) {
    const auto c = add_points(FImg{fine, (uint32_t)w, (uint32_t)h}, tracked_xy, n_tracked, threshold,
                              (uint32_t)min_dist, blur);
    const int n = (int)std::min<size_t>(c.size(), (size_t)cap);
    for (int i = 0; i < n; ++i) {
        out_xy[2 * i] = c[i].x;
        out_xy[2 * i + 1] = c[i].y;
    }
    return (int)c.size();
}

orc_ft* orc_ft_create(const orc_ft_config* cfg, int w, int h) {
    orc_ft* t = new orc_ft();
    t->cfg = *cfg;
    t->w = w;
    t->h = h;
    t->pyr_floats = orc_ft_pyramid_floats(w, h, cfg->nlevels, cfg->ratio);
    return t;
}

void orc_ft_destroy(orc_ft* t) { delete t; }

// feature_tracker.rs:77-185.  Features of the frame: the previous frame's features that track
// (previous order), then the new corners (detection order) with consecutive ids.
int orc_ft_process_frame(orc_ft* t, const float* img, uint64_t* ids_out, float* xy_out, int cap, int* n_out) {
    const orc_ft_config& c = t->cfg;
    std::vector<float> pyr(t->pyr_floats);
    orc_ft_build_pyramid(img, t->w, t->h, c.nlevels, c.ratio, c.preprocessing_blur, c.preprocessing_blur_sigma,
                         pyr.data());
    std::vector<uint64_t> ids;
    std::vector<float> xy;
    if (t->has_prev) {
        const Pyr p0 = make_pyr(t->prev_pyr.data(), t->w, t->h, c.nlevels, c.ratio);
        const Pyr p1 = make_pyr(pyr.data(), t->w, t->h, c.nlevels, c.ratio);
        for (size_t i = 0; i < t->ids.size(); ++i) {
            Iso f;
            const float fx = t->xy[2 * i], fy = t->xy[2 * i + 1];
            if (track_feature(p0, p1, fx, fy, c.optical_flow_max_iter, c.optical_flow_lm_lambda, c.matching_cost, f)) {
                float x1, y1;
                iso_apply(f, fx, fy, &x1, &y1);
                ids.push_back(t->ids[i]);
                xy.push_back(x1);
                xy.push_back(y1);
            }
        }
    }
    const auto nc = add_points(FImg{pyr.data(), (uint32_t)t->w, (uint32_t)t->h}, xy.data(), (int)ids.size(),
                               c.detection_threshold, c.detection_min_dist, c.detection_blur);
    for (const auto& k : nc) {
        ids.push_back(t->last_id++);
        xy.push_back((float)k.x);
        xy.push_back((float)k.y);
    }
    t->ids = ids;
    t->xy = xy;
    t->prev_pyr.swap(pyr);
    t->has_prev = true;
    const int n = (int)ids.size();
    *n_out = n;
    for (int i = 0; i < n && i < cap; ++i) {
        ids_out[i] = ids[i];
        xy_out[2 * i] = xy[2 * i];
        xy_out[2 * i + 1] = xy[2 * i + 1];
    }
    return n <= cap ? 0 : -4;
}

}  // extern "C"
