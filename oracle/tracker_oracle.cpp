// tracker_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see rsvio_oracle.h).
//
// Scalar C++ restatement of the reference patch tracker, src/feature_tracker/ of
// EthanD11/RS-VIO.  Every floating-point expression keeps the reference's
// evaluation order (Rust never contracts a*b+c, nalgebra accumulates small
// products sequentially in k); build with -ffp-contract=off.
#include "pool.hpp"
#include "rsvio_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

namespace {

// Rust f32::sin / f32::cos (reached through nalgebra Rotation2::new, image_utilities.rs:84) call
// glibc sinf / cosf on x86-64 Linux: the oracle calls the same libm.
inline void sin_cos_f32(float th, float* s, float* c) {
    *s = sinf(th);
    *c = cosf(th);
}

// Rust `f32 as u32` saturates (NaN -> 0, negative -> 0).
inline uint32_t sat_u32(float v) {
    if (!(v > 0.0f)) return 0u;
    if (v >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)v;
}

// ---------------------------------------------------------------------------------
// image 0.25 imageops::resize(.., Triangle)  (call site feature_tracker.rs:217)
// Vertical pass into an f32 buffer, then horizontal pass with clamp + round.
// ---------------------------------------------------------------------------------
inline float triangle_kernel(float x) {
    float ax = std::fabs(x);
    return ax < 1.0f ? 1.0f - ax : 0.0f;
}

struct Taps {
    int64_t left;
    std::vector<float> w;
};

Taps make_taps(int out_i, uint32_t in_len, uint32_t out_len) {
    float ratio = (float)in_len / (float)out_len;
    float sratio = ratio < 1.0f ? 1.0f : ratio;
    float support = 1.0f * sratio;
    float inputc = ((float)out_i + 0.5f) * ratio;
    int64_t left = (int64_t)std::floor(inputc - support);
    if (left < 0) left = 0;
    if (left > (int64_t)in_len - 1) left = (int64_t)in_len - 1;
    int64_t right = (int64_t)std::ceil(inputc + support);
    if (right < left + 1) right = left + 1;
    if (right > (int64_t)in_len) right = (int64_t)in_len;
    inputc = inputc - 0.5f;
    Taps t;
    t.left = left;
    float sum = 0.0f;
    for (int64_t i = left; i < right; ++i) {
        float wv = triangle_kernel(((float)i - inputc) / sratio);
        t.w.push_back(wv);
        sum += wv;
    }
    for (auto& wv : t.w) wv /= sum;
    return t;
}

// ---------------------------------------------------------------------------------
// Pattern52 (patch.rs:8-233)
// ---------------------------------------------------------------------------------
constexpr int NP = 52;
// patch.rs:19-72 -- the 52-point sampling pattern (x, y), pixel units before the 1/2 scale.
const float PATTERN_RAW[NP][2] = {
    {-3, 7},  {-1, 7},  {1, 7},   {3, 7},   {-5, 5},  {-3, 5},  {-1, 5},  {1, 5},   {3, 5},
    {5, 5},   {-7, 3},  {-5, 3},  {-3, 3},  {-1, 3},  {1, 3},   {3, 3},   {5, 3},   {7, 3},
    {-7, 1},  {-5, 1},  {-3, 1},  {-1, 1},  {1, 1},   {3, 1},   {5, 1},   {7, 1},   {-7, -1},
    {-5, -1}, {-3, -1}, {-1, -1}, {1, -1},  {3, -1},  {5, -1},  {7, -1},  {-7, -3}, {-5, -3},
    {-3, -3}, {-1, -3}, {1, -3},  {3, -3},  {5, -3},  {7, -3},  {-5, -5}, {-3, -5}, {-1, -5},
    {1, -5},  {3, -5},  {5, -5},  {-3, -7}, {-1, -7}, {1, -7},  {3, -7}};

struct Img {
    const uint8_t* p;
    uint32_t w, h;
};

// image_utilities.rs:75-80
inline bool inbound(const Img& im, float x, float y, uint32_t r) {
    uint32_t xi = sat_u32(std::round(x));
    uint32_t yi = sat_u32(std::round(y));
    return xi >= r && yi >= r && xi < im.w - r && yi < im.h - r;
}

// image_utilities.rs:5-66 -- bilinear value and central-difference gradient.
inline void image_grad(const Img& im, float x, float y, float out[3]) {
    uint32_t ix = (uint32_t)std::floor(x);
    uint32_t iy = (uint32_t)std::floor(y);
    float dx = x - (float)ix;
    float dy = y - (float)iy;
    float ddx = 1.0f - dx;
    float ddy = 1.0f - dy;
    uint32_t w = im.w;
    const uint8_t* P = im.p;
    auto px = [&](uint32_t xx, uint32_t yy) { return (float)P[(size_t)yy * w + xx]; };
    float p00 = px(ix, iy), p10 = px(ix + 1, iy), p01 = px(ix, iy + 1), p11 = px(ix + 1, iy + 1);
    float res0 = ddx * ddy * p00 + ddx * dy * p01 + dx * ddy * p10 + dx * dy * p11;
    float pm0 = px(ix - 1, iy), pm1 = px(ix - 1, iy + 1);
    float res_mx = ddx * ddy * pm0 + ddx * dy * pm1 + dx * ddy * p00 + dx * dy * p01;
    float p20 = px(ix + 2, iy), p21 = px(ix + 2, iy + 1);
    float res_px = ddx * ddy * p10 + ddx * dy * p11 + dx * ddy * p20 + dx * dy * p21;
    float res1 = 0.5f * (res_px - res_mx);
    float p0m = px(ix, iy - 1), p1m = px(ix + 1, iy - 1);
    float res_my = ddx * ddy * p0m + ddx * dy * p00 + dx * ddy * p1m + dx * dy * p10;
    float p02 = px(ix, iy + 2), p12 = px(ix + 1, iy + 2);
    float res_py = ddx * ddy * p01 + ddx * dy * p02 + dx * ddy * p11 + dx * dy * p12;
    float res2 = 0.5f * (res_py - res_my);
    out[0] = res0;
    out[1] = res1;
    out[2] = res2;
}

struct Pattern52 {
    bool valid = false;
    float mean = 1.0f;
    float posx = 0, posy = 0;
    float data[NP];
    float hinvjt[3][NP];  // h_se2_inv_j_se2_t
    float pat[2][NP];     // pattern_matrix (PATTERN_RAW / 2)
};

// nalgebra Cholesky::new on a 3x3 (lower triangle, column j: axpy updates then sqrt, divide)
bool cholesky3(float A[3][3]) {
    for (int j = 0; j < 3; ++j) {
        for (int k = 0; k < j; ++k) {
            float factor = -A[j][k];
            for (int r = j; r < 3; ++r) A[r][j] = factor * A[r][k] + A[r][j];
        }
        float diag = A[j][j];
        if (diag != 0.0f && diag >= 0.0f) {
            float denom = std::sqrt(diag);
            A[j][j] = denom;
            for (int r = j + 1; r < 3; ++r) A[r][j] = A[r][j] / denom;
            continue;
        }
        return false;
    }
    return true;
}

// Cholesky::solve_mut(identity): forward L y = e, then backward L^T x = y (nalgebra solve.rs)
void chol_inverse3(const float L[3][3], float X[3][3]) {
    for (int c = 0; c < 3; ++c) {
        float b[3] = {0.0f, 0.0f, 0.0f};
        b[c] = 1.0f;
        for (int i = 0; i < 3; ++i) {
            float coeff = b[i] / L[i][i];
            b[i] = coeff;
            for (int r = i + 1; r < 3; ++r) b[r] = (-coeff) * L[r][i] + b[r];
        }
        for (int i = 2; i >= 0; --i) {
            float dot = 0.0f;
            for (int r = i + 1; r < 3; ++r) dot = dot + L[r][i] * b[r];
            b[i] = (b[i] - dot) / L[i][i];
        }
        for (int r = 0; r < 3; ++r) X[r][c] = b[r];
    }
}

// patch.rs:75-123
void set_data_jac_se2(Pattern52& P, const Img& im, float J[NP][3]) {
    int num_valid = 0;
    float sum = 0.0f;
    float gs[3] = {0.0f, 0.0f, 0.0f};
    const float sd = 2.0f;
    for (int i = 0; i < NP; ++i) {
        float ox = PATTERN_RAW[i][0], oy = PATTERN_RAW[i][1];
        float px = P.posx + ox / sd;
        float py = P.posy + oy / sd;
        float jw02 = -oy / sd;
        float jw12 = ox / sd;
        if (inbound(im, px, py, 2)) {
            float vg[3];
            image_grad(im, px, py, vg);
            P.data[i] = vg[0];
            sum += vg[0];
            // (1x2 grad) * (2x3 [[1,0,-oy/2],[0,1,ox/2]]), gemm column by column
            J[i][0] = vg[1] * 1.0f + vg[2] * 0.0f;
            J[i][1] = vg[1] * 0.0f + vg[2] * 1.0f;
            J[i][2] = vg[1] * jw02 + vg[2] * jw12;
            gs[0] = gs[0] + J[i][0];
            gs[1] = gs[1] + J[i][1];
            gs[2] = gs[2] + J[i][2];
            num_valid += 1;
        } else {
            P.data[i] = -1.0f;
        }
    }
    P.mean = sum / (float)num_valid;
    float mean_inv = (float)num_valid / sum;
    for (int i = 0; i < NP; ++i) {
        if (P.data[i] >= 0.0f) {
            for (int k = 0; k < 3; ++k) {
                float rhs = gs[k] * P.data[i] / sum;
                J[i][k] = J[i][k] + (-rhs);
            }
            P.data[i] *= mean_inv;
        } else {
            J[i][0] = J[i][1] = J[i][2] = 0.0f;
        }
    }
    for (int i = 0; i < NP; ++i)
        for (int k = 0; k < 3; ++k) J[i][k] *= mean_inv;
}

// patch.rs:124-162
Pattern52 pattern_new(const Img& im, float px, float py) {
    Pattern52 P;
    for (int j = 0; j < NP; ++j) {
        P.pat[0][j] = PATTERN_RAW[j][0] / 2.0f;
        P.pat[1][j] = PATTERN_RAW[j][1] / 2.0f;
        P.hinvjt[0][j] = P.hinvjt[1][j] = P.hinvjt[2][j] = 0.0f;
        P.data[j] = 0.0f;
    }
    P.posx = px;
    P.posy = py;
    float J[NP][3];
    for (int i = 0; i < NP; ++i) J[i][0] = J[i][1] = J[i][2] = 0.0f;
    set_data_jac_se2(P, im, J);
    // H = J^T J : column b of H = sum_k J_k,: * J_kb (k ascending)
    float H[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            float acc = J[0][a] * J[0][b];
            for (int k = 1; k < NP; ++k) acc = J[k][a] * J[k][b] + acc;
            H[a][b] = acc;
        }
    if (cholesky3(H)) {
        float Hi[3][3];
        chol_inverse3(H, Hi);
        for (int k = 0; k < NP; ++k)
            for (int a = 0; a < 3; ++a) {
                float acc = Hi[a][0] * J[k][0];
                acc = Hi[a][1] * J[k][1] + acc;
                acc = Hi[a][2] * J[k][2] + acc;
                P.hinvjt[a][k] = acc;
            }
        bool fin = true;
        for (int a = 0; a < 3; ++a)
            for (int k = 0; k < NP; ++k) fin = fin && std::isfinite(P.hinvjt[a][k]);
        for (int k = 0; k < NP; ++k) fin = fin && std::isfinite(P.data[k]);
        P.valid = (P.mean > __FLT_EPSILON__) && fin;
    }
    return P;
}

// patch.rs:163-232
bool pattern_residual(const Pattern52& P, const Img& im, const float tp[2][NP], float res[NP]) {
    float sum = 0.0f;
    int num_valid = 0;
    float wlim = (float)(im.w - 2), hlim = (float)(im.h - 2);
    for (int i = 0; i < NP; ++i) {
        float x = tp[0][i], y = tp[1][i];
        if (x >= 2.0f && y >= 2.0f && x < wlim && y < hlim) {
            uint32_t ix = (uint32_t)std::floor(x);
            uint32_t iy = (uint32_t)std::floor(y);
            float dx = x - (float)ix;
            float dy = y - (float)iy;
            float ddx = 1.0f - dx;
            float ddy = 1.0f - dy;
            const uint8_t* row0 = im.p + (size_t)iy * im.w;
            const uint8_t* row1 = row0 + im.w;
            float p00 = (float)row0[ix], p10 = (float)row0[ix + 1];
            float p01 = (float)row1[ix], p11 = (float)row1[ix + 1];
            res[i] = ddx * ddy * p00 + ddx * dy * p01 + dx * ddy * p10 + dx * dy * p11;
            sum += res[i];
            num_valid += 1;
        } else {
            res[i] = -1.0f;
        }
    }
    if (sum < __FLT_EPSILON__) return false;
    int num_res = 0;
    for (int i = 0; i < NP; ++i) {
        if (res[i] >= 0.0f && P.data[i] >= 0.0f) {
            float val = res[i];
            res[i] = (float)num_valid * val / sum - P.data[i];
            num_res += 1;
        } else {
            res[i] = 0.0f;
        }
    }
    return num_res > NP / 2;
}

// Affine2 as a 3x3 [[m11 m12 m13],[m21 m22 m23],[0 0 1]]
struct Aff {
    float m[3][3];
};
Aff aff_from6(const float* a) {
    Aff A;
    A.m[0][0] = a[0]; A.m[0][1] = a[1]; A.m[0][2] = a[4];
    A.m[1][0] = a[2]; A.m[1][1] = a[3]; A.m[1][2] = a[5];
    A.m[2][0] = 0.0f; A.m[2][1] = 0.0f; A.m[2][2] = 1.0f;
    return A;
}
void aff_to6(const Aff& A, float* a) {
    a[0] = A.m[0][0]; a[1] = A.m[0][1]; a[2] = A.m[1][0];
    a[3] = A.m[1][1]; a[4] = A.m[0][2]; a[5] = A.m[1][2];
}
// nalgebra 3x3 gemm: column j = sum_k A.col(k) * B[k][j], k ascending
Aff mat3_mul(const Aff& A, const Aff& B) {
    Aff C;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) {
            float acc = A.m[i][0] * B.m[0][j];
            acc = A.m[i][1] * B.m[1][j] + acc;
            acc = A.m[i][2] * B.m[2][j] + acc;
            C.m[i][j] = acc;
        }
    return C;
}

// image_utilities.rs:82-106 (twist order [vx, vy, theta])
Aff se2_exp(const float a[3]) {
    float theta = a[2];
    float s, c;
    sin_cos_f32(theta, &s, &c);
    float sin_by, omc_by;
    if (std::fabs(theta) < __FLT_EPSILON__) {
        float th2 = theta * theta;
        sin_by = 1.0f - (1.0f / 6.0f) * th2;
        omc_by = 0.5f * theta - (1.0f / 24.0f) * theta * th2;
    } else {
        sin_by = s / theta;
        omc_by = (1.0f - c) / theta;
    }
    Aff E;
    E.m[0][0] = c; E.m[0][1] = -s; E.m[1][0] = s; E.m[1][1] = c;
    E.m[0][2] = sin_by * a[0] - omc_by * a[1];
    E.m[1][2] = omc_by * a[0] + sin_by * a[1];
    E.m[2][0] = 0.0f; E.m[2][1] = 0.0f; E.m[2][2] = 1.0f;
    return E;
}

// feature_tracker.rs:344-395
bool track_point_at_level(const Img& im, const Pattern52& P, Aff& T, int max_iter, float thresh) {
    float tp[2][NP];
    float res[NP];
    for (int it = 0; it < max_iter; ++it) {
        for (int j = 0; j < NP; ++j) {
            float x = T.m[0][0] * P.pat[0][j];
            x = T.m[0][1] * P.pat[1][j] + x;
            float y = T.m[1][0] * P.pat[0][j];
            y = T.m[1][1] * P.pat[1][j] + y;
            tp[0][j] = x + T.m[0][2];
            tp[1][j] = y + T.m[1][2];
        }
        if (!pattern_residual(P, im, tp, res)) return false;
        float inc[3];
        for (int a = 0; a < 3; ++a) {
            float acc = (-P.hinvjt[a][0]) * res[0];
            for (int k = 1; k < NP; ++k) acc = (-P.hinvjt[a][k]) * res[k] + acc;
            inc[a] = acc;
        }
        if (!(std::isfinite(inc[0]) && std::isfinite(inc[1]) && std::isfinite(inc[2]))) return false;
        float nrm = std::sqrt(inc[0] * inc[0] + inc[1] * inc[1] + inc[2] * inc[2]);
        if (nrm > 1e6f) return false;
        if (nrm < thresh) break;
        T = mat3_mul(T, se2_exp(inc));
        if (!inbound(im, T.m[0][2], T.m[1][2], 2)) return false;
    }
    return true;
}

struct Pyr {
    const uint8_t* base;
    int w, h;
    Img level(int i) const {
        Img im;
        im.p = base + orc_pyramid_offset(w, h, i);
        im.w = (uint32_t)(w >> 0) / (1u << i);
        im.h = (uint32_t)(h >> 0) / (1u << i);
        return im;
    }
};

// feature_tracker.rs:292-342
bool track_one_point(const Pyr& p0, const Pyr& p1, int levels, const Aff& T0, int max_iter,
                     float thresh, Aff& out) {
    Aff T1;
    T1.m[0][0] = 1.0f; T1.m[0][1] = 0.0f; T1.m[1][0] = 0.0f; T1.m[1][1] = 1.0f;
    T1.m[2][0] = 0.0f; T1.m[2][1] = 0.0f; T1.m[2][2] = 1.0f;
    T1.m[0][2] = T0.m[0][2];
    T1.m[1][2] = T0.m[1][2];
    for (int i = levels - 1; i >= 0; --i) {
        float sdn = (float)(1 << i);
        T1.m[0][2] /= sdn;
        T1.m[1][2] /= sdn;
        Img im0 = p0.level(i), im1 = p1.level(i);
        Pattern52 P = pattern_new(im0, T0.m[0][2] / sdn, T0.m[1][2] / sdn);
        if (!P.valid) return false;
        if (!track_point_at_level(im1, P, T1, max_iter, thresh)) return false;
        T1.m[0][2] *= sdn;
        T1.m[1][2] *= sdn;
    }
    Aff R = mat3_mul(T0, T1);
    T1.m[0][0] = R.m[0][0];
    T1.m[0][1] = R.m[0][1];
    T1.m[1][0] = R.m[1][0];
    T1.m[1][1] = R.m[1][1];
    out = T1;
    return true;
}

bool track_fb(const Pyr& p0, const Pyr& p1, int levels, const float* ain, int max_iter,
              float thresh, float* aout) {
    Aff T0 = aff_from6(ain);
    Aff fwd, bwd;
    if (!track_one_point(p0, p1, levels, T0, max_iter, thresh, fwd)) return false;
    if (!track_one_point(p1, p0, levels, fwd, max_iter, thresh, bwd)) return false;
    float dx = T0.m[0][2] - bwd.m[0][2];
    float dy = T0.m[1][2] - bwd.m[1][2];
    if (!(dx * dx + dy * dy < 0.4f)) return false;
    aff_to6(fwd, aout);
    return true;
}

// ---------------------------------------------------------------------------------
// imageproc 0.25 corners_fast9 (call site image_utilities.rs:156)
// ---------------------------------------------------------------------------------
bool is_corner_fast9(const Img& im, uint8_t t, uint32_t x, uint32_t y) {
    if (x < 3 || y < 3 || im.w <= x + 3 || im.h <= y + 3) return false;
    auto px = [&](uint32_t xx, uint32_t yy) { return (int16_t)im.p[(size_t)yy * im.w + xx]; };
    int16_t c = px(x, y);
    int16_t lo = (int16_t)(c - (int16_t)t);
    int16_t hi = (int16_t)(c + (int16_t)t);
    // Bresenham circle of radius 3, clockwise from the top (labels 0..15)
    int16_t p[16] = {px(x, y - 3),     px(x + 1, y - 3), px(x + 2, y - 2), px(x + 3, y - 1),
                     px(x + 3, y),     px(x + 3, y + 1), px(x + 2, y + 2), px(x + 1, y + 3),
                     px(x, y + 3),     px(x - 1, y + 3), px(x - 2, y + 2), px(x - 3, y + 1),
                     px(x - 3, y),     px(x - 3, y - 1), px(x - 2, y - 2), px(x - 1, y - 3)};
    // quick rejection on the four cardinal points (adjacent pairs)
    int16_t c0 = p[0], c4 = p[4], c8 = p[8], c12 = p[12];
    bool above = (c0 > hi && c4 > hi) || (c4 > hi && c8 > hi) || (c8 > hi && c12 > hi) ||
                 (c12 > hi && c0 > hi);
    bool below = (c0 < lo && c4 < lo) || (c4 < lo && c8 < lo) || (c8 < lo && c12 < lo) ||
                 (c12 < lo && c0 < lo);
    if (!above && !below) return false;
    auto span = [&](bool bright) {
        int nb = 0, start = -1;
        for (int i = 0; i < 16; ++i) {
            bool ok = bright ? (p[i] > hi) : (p[i] < lo);
            if (ok) {
                if (++nb == 9) return true;
            } else {
                if (start < 0) start = nb;
                nb = 0;
            }
        }
        return nb + start >= 9;
    };
    return (above && span(true)) || (below && span(false));
}

// imageproc fast_corner_score: binary search for the largest threshold that is still a corner
uint8_t fast9_score(const Img& im, uint8_t threshold, uint32_t x, uint32_t y) {
    uint8_t mx = 255, mn = threshold;
    for (;;) {
        if (mx == mn) return mx;
        uint8_t mean = (uint8_t)(((uint16_t)mx + (uint16_t)mn) / 2u);
        uint8_t probe = (mx == (uint8_t)(mn + 1)) ? mx : mean;
        if (is_corner_fast9(im, probe, x, y))
            mn = probe;
        else
            mx = (uint8_t)(probe - 1);
    }
}

struct Corner {
    uint32_t x, y;
    float score;
};

std::vector<Corner> corners_fast9(const Img& im, uint8_t t) {
    std::vector<Corner> out;
    for (uint32_t y = 0; y < im.h; ++y)
        for (uint32_t x = 0; x < im.w; ++x)
            if (is_corner_fast9(im, t, x, y)) out.push_back({x, y, (float)fast9_score(im, t, x, y)});
    return out;
}

// image_utilities.rs:68-73 (note the inclusive upper bound)
inline bool point_in_bound(const Corner& k, uint32_t h, uint32_t w, uint32_t r) {
    return k.x >= r && k.x <= w - r && k.y >= r && k.y <= h - r;
}

// image_utilities.rs:108-175 with num_points_in_cell = 1 (feature_tracker.rs:227)
std::vector<Corner> detect_key_points(const Img& im, uint32_t grid,
                                      const std::vector<Corner>& current) {
    const uint32_t EDGE = 19;
    uint32_t h = im.h, w = im.w;
    std::vector<Corner> all;
    uint32_t gr = h / grid + 1, gc = w / grid + 1;
    std::vector<int> cells((size_t)gr * gc, 0);
    uint32_t xs = (w % grid) / 2, xe = xs + grid * (w / grid - 1) + 1;
    uint32_t ys = (h % grid) / 2, ye = ys + grid * (h / grid - 1) + 1;
    for (const auto& c : current) {
        if (c.x >= xs && c.y >= ys && c.x < xe + grid && c.y < ye + grid) {
            uint32_t cx = (c.x - xs) / grid, cy = (c.y - ys) / grid;
            cells[(size_t)cy * gc + cx] += 1;
        }
    }
    std::vector<uint8_t> crop((size_t)grid * grid);
    for (uint32_t x = xs; x < xe; x += grid) {
        for (uint32_t y = ys; y < ye; y += grid) {
            if (cells[(size_t)((y - ys) / grid) * gc + (x - xs) / grid] > 0) continue;
            for (uint32_t r = 0; r < grid; ++r)
                memcpy(&crop[(size_t)r * grid], im.p + (size_t)(y + r) * w + x, grid);
            Img cim{crop.data(), grid, grid};
            uint32_t added = 0;
            uint8_t thr = 40;
            while (added < 1 && thr >= 10) {
                auto fc = corners_fast9(cim, thr);
                std::stable_sort(fc.begin(), fc.end(),
                                 [](const Corner& a, const Corner& b) { return a.score < b.score; });
                for (auto pt : fc) {
                    if (added >= 1) break;
                    pt.x += x;
                    pt.y += y;
                    if (point_in_bound(pt, h, w, EDGE)) {
                        all.push_back(pt);
                        added += 1;
                    }
                }
                thr -= 5;
            }
        }
    }
    return all;
}

}  // namespace

// =====================================================================================
extern "C" {

// Per-chunk digests of libm's sinf/cosf over f32 bit patterns [first, first + count), the
// definition rsvio_sincosf_digest (include/rsvio_gpu.h) states, over nthreads threads.
void orc_libm_sincosf_digest(uint64_t first, uint64_t count, uint32_t chunk_log2, int nthreads,
                             uint64_t* digests) {
    const uint64_t n_chunks = (count + (1ull << chunk_log2) - 1) >> chunk_log2;
    for (uint64_t k = 0; k < n_chunks; ++k) digests[k] = 0;
    if (nthreads < 1) nthreads = 1;
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; ++t)
        pool.emplace_back([=] {
            for (uint64_t k = (uint64_t)t; k < n_chunks; k += (uint64_t)nthreads) {
                const uint64_t a = k << chunk_log2;
                const uint64_t b = std::min(count, (k + 1) << chunk_log2);
                uint64_t acc = 0;
                for (uint64_t off = a; off < b; ++off) {
                    const uint32_t u = (uint32_t)(first + off);
                    float y;
                    std::memcpy(&y, &u, 4);
                    const float sv = sinf(y), cv = cosf(y);
                    uint32_t sb, cb;
                    std::memcpy(&sb, &sv, 4);
                    std::memcpy(&cb, &cv, 4);
                    if (sv != sv) sb = 0x7fc00000u;
                    if (cv != cv) cb = 0x7fc00000u;
                    uint64_t z = (((uint64_t)sb << 32) | cb) + (uint64_t)u * 0x9E3779B97F4A7C15ull;
                    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                    acc += z ^ (z >> 31);
                }
                digests[k] = acc;
            }
        });
    for (auto& th : pool) th.join();
}
}  // extern "C"

extern "C" {

void orc_se2_exp(const float* twist, float* out9) {
    Aff E = se2_exp(twist);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out9[3 * i + j] = E.m[i][j];
}

size_t orc_pyramid_offset(int w, int h, int level) {
    size_t off = 0;
    for (int i = 0; i < level; ++i) off += (size_t)((uint32_t)w / (1u << i)) * ((uint32_t)h / (1u << i));
    return off;
}
size_t orc_pyramid_bytes(int w, int h, int levels) { return orc_pyramid_offset(w, h, levels); }

void orc_resize_triangle(const uint8_t* src, int w, int h, uint8_t* dst, int nw, int nh) {
    if (w == 0 || h == 0) {
        memset(dst, 0, (size_t)nw * nh);
        return;
    }
    if (nw == w && nh == h) {
        memcpy(dst, src, (size_t)w * h);
        return;
    }
    std::vector<float> tmp((size_t)w * nh);
    for (int oy = 0; oy < nh; ++oy) {
        Taps t = make_taps(oy, (uint32_t)h, (uint32_t)nh);
        for (int x = 0; x < w; ++x) {
            float acc = 0.0f;
            for (size_t k = 0; k < t.w.size(); ++k)
                acc += (float)src[(size_t)(t.left + (int64_t)k) * w + x] * t.w[k];
            tmp[(size_t)oy * w + x] = acc;
        }
    }
    for (int ox = 0; ox < nw; ++ox) {
        Taps t = make_taps(ox, (uint32_t)w, (uint32_t)nw);
        for (int y = 0; y < nh; ++y) {
            float acc = 0.0f;
            for (size_t k = 0; k < t.w.size(); ++k)
                acc += tmp[(size_t)y * w + (size_t)(t.left + (int64_t)k)] * t.w[k];
            float c = acc < 0.0f ? 0.0f : (acc > 255.0f ? 255.0f : acc);
            dst[(size_t)y * nw + ox] = (uint8_t)std::round(c);
        }
    }
}

void orc_build_pyramid(const uint8_t* img, int w, int h, int levels, uint8_t* out) {
    for (int i = 0; i < levels; ++i) {
        int nw = (int)((uint32_t)w / (1u << i)), nh = (int)((uint32_t)h / (1u << i));
        orc_resize_triangle(img, w, h, out + orc_pyramid_offset(w, h, i), nw, nh);
    }
}

// build_image_pyramid with rayon's par_iter over levels (feature_tracker.rs:213): the levels as
// tasks of the persistent pool (pool.hpp; the all-cores CPU baseline); the same bytes as
// orc_build_pyramid
void orc_build_pyramid_mt(const uint8_t* img, int w, int h, int levels, uint8_t* out, int n_threads) {
    if (n_threads <= 1 || levels < 2) {
        orc_build_pyramid(img, w, h, levels, out);
        return;
    }
    orc::Pool::get().run(levels, std::min(n_threads, levels), [=](int i) {
        int nw = (int)((uint32_t)w / (1u << i)), nh = (int)((uint32_t)h / (1u << i));
        orc_resize_triangle(img, w, h, out + orc_pyramid_offset(w, h, i), nw, nh);
    });
}

int orc_pattern52_new(const uint8_t* img, int w, int h, float px, float py, float* out_data,
                      float* out_hinvjt, float* out_mean) {
    Img im{img, (uint32_t)w, (uint32_t)h};
    Pattern52 P = pattern_new(im, px, py);
    for (int k = 0; k < NP; ++k) {
        out_data[k] = P.data[k];
        for (int a = 0; a < 3; ++a) out_hinvjt[a * NP + k] = P.hinvjt[a][k];
    }
    if (out_mean) *out_mean = P.mean;
    return P.valid ? 1 : 0;
}

int orc_track_point_at_level(const uint8_t* img, int w, int h, const uint8_t* tmpl_img, float px,
                             float py, float* aff, int max_iter, float thresh) {
    Img im{img, (uint32_t)w, (uint32_t)h};
    Img tm{tmpl_img, (uint32_t)w, (uint32_t)h};
    Pattern52 P = pattern_new(tm, px, py);
    if (!P.valid) return 0;
    Aff T = aff_from6(aff);
    bool ok = track_point_at_level(im, P, T, max_iter, thresh);
    aff_to6(T, aff);
    return ok ? 1 : 0;
}

int orc_track_one_point(const uint8_t* pyr0, const uint8_t* pyr1, int w, int h, int levels,
                        const float* aff_in, int max_iter, float thresh, float* aff_out) {
    Pyr p0{pyr0, w, h}, p1{pyr1, w, h};
    Aff out;
    if (!track_one_point(p0, p1, levels, aff_from6(aff_in), max_iter, thresh, out)) return 0;
    aff_to6(out, aff_out);
    return 1;
}

void orc_track_points(const uint8_t* pyr0, const uint8_t* pyr1, int w, int h, int levels,
                      const float* aff_in, int n, int max_iter, float thresh, float* aff_out,
                      uint8_t* valid_out, int n_threads) {
    Pyr p0{pyr0, w, h}, p1{pyr1, w, h};
    auto work = [&](int b, int e) {
        for (int i = b; i < e; ++i) {
            bool ok = track_fb(p0, p1, levels, aff_in + 6 * i, max_iter, thresh, aff_out + 6 * i);
            valid_out[i] = ok ? 1 : 0;
            if (!ok)
                for (int k = 0; k < 6; ++k) aff_out[6 * i + k] = aff_in[6 * i + k];
        }
    };
    if (n_threads <= 1 || n < 2) {
        work(0, n);
        return;
    }
    // rayon par_iter analogue (feature_tracker.rs:260): grains of 2 features claimed dynamically
    // by the persistent pool's threads (the chains' lengths vary by 10x, so static chunks idle)
    constexpr int kGrain = 2;
    orc::Pool::get().run((n + kGrain - 1) / kGrain, n_threads,
                         [&](int g) { work(g * kGrain, std::min(n, (g + 1) * kGrain)); });
}

int orc_fast9_scores(const uint8_t* img, int w, int h, int threshold, uint8_t* score_out) {
    Img im{img, (uint32_t)w, (uint32_t)h};
    int cnt = 0;
    for (uint32_t y = 0; y < (uint32_t)h; ++y)
        for (uint32_t x = 0; x < (uint32_t)w; ++x) {
            uint8_t s = 0;
            if (is_corner_fast9(im, (uint8_t)threshold, x, y)) {
                s = fast9_score(im, (uint8_t)threshold, x, y);
                ++cnt;
            }
            score_out[(size_t)y * w + x] = s;
        }
    return cnt;
}

int orc_detect_keypoints(const uint8_t* img, int w, int h, int grid, const float* existing_xy,
                         int n_existing, uint32_t* out_xy, float* out_score, int cap) {
    Img im{img, (uint32_t)w, (uint32_t)h};
    std::vector<Corner> cur;
    for (int i = 0; i < n_existing; ++i)
        cur.push_back({sat_u32(std::round(existing_xy[2 * i])),
                       sat_u32(std::round(existing_xy[2 * i + 1])), 0.0f});
    auto pts = detect_key_points(im, (uint32_t)grid, cur);
    int n = 0;
    for (const auto& c : pts) {
        if (n >= cap) break;
        out_xy[2 * n] = c.x;
        out_xy[2 * n + 1] = c.y;
        if (out_score) out_score[n] = c.score;
        ++n;
    }
    return n;
}

// ---------------------------------------------------------------------------------
// StereoPatchTracker (feature_tracker.rs:91-207), canonical order: ascending id.
// ---------------------------------------------------------------------------------
struct orc_tracker {
    int w, h, levels, grid, max_iter;
    float thresh;
    uint64_t last_id = 0;
    std::vector<orc_feature> map0, map1;
    std::vector<uint8_t> prev0, prev1;
    bool has_prev = false;
    int threads = 1;  // rayon analogue: pyramid levels and features in parallel (all-cores CPU leg)
};

orc_tracker* orc_tracker_create(int w, int h, int levels, int grid, int max_iter, float thresh) {
    auto* t = new orc_tracker();
    t->w = w; t->h = h; t->levels = levels; t->grid = grid; t->max_iter = max_iter;
    t->thresh = thresh;
    return t;
}
void orc_tracker_destroy(orc_tracker* t) { delete t; }
void orc_tracker_set_threads(orc_tracker* t, int threads) { t->threads = threads < 1 ? 1 : threads; }

static void track_map(const orc_tracker* t, const uint8_t* pa, const uint8_t* pb,
                      std::vector<orc_feature>& m) {
    int n = (int)m.size();
    std::vector<float> ain(6 * n), aout(6 * n);
    std::vector<uint8_t> v(n);
    for (int i = 0; i < n; ++i) memcpy(&ain[6 * i], m[i].aff, 24);
    orc_track_points(pa, pb, t->w, t->h, t->levels, ain.data(), n, t->max_iter, t->thresh,
                     aout.data(), v.data(), t->threads);
    std::vector<orc_feature> out;
    for (int i = 0; i < n; ++i)
        if (v[i]) {
            orc_feature f = m[i];
            memcpy(f.aff, &aout[6 * i], 24);
            f.x = f.aff[4];
            f.y = f.aff[5];
            out.push_back(f);
        }
    m.swap(out);
}

int orc_tracker_process_frame(orc_tracker* t, const uint8_t* left, const uint8_t* right,
                              orc_feature* out_l, int cap_l, int* n_l, orc_feature* out_r,
                              int cap_r, int* n_r) {
    size_t pb = orc_pyramid_bytes(t->w, t->h, t->levels);
    std::vector<uint8_t> cur0(pb), cur1(pb);
    orc_build_pyramid_mt(left, t->w, t->h, t->levels, cur0.data(), t->threads);
    orc_build_pyramid_mt(right, t->w, t->h, t->levels, cur1.data(), t->threads);
    if (t->has_prev) {
        track_map(t, t->prev0.data(), cur0.data(), t->map0);
        track_map(t, t->prev1.data(), cur1.data(), t->map1);
    }
    // add_points (feature_tracker.rs:222-251)
    std::vector<float> ex(2 * t->map0.size());
    for (size_t i = 0; i < t->map0.size(); ++i) {
        ex[2 * i] = t->map0[i].aff[4];
        ex[2 * i + 1] = t->map0[i].aff[5];
    }
    Img im{left, (uint32_t)t->w, (uint32_t)t->h};
    std::vector<Corner> cur;
    for (size_t i = 0; i < t->map0.size(); ++i)
        cur.push_back({sat_u32(std::round(ex[2 * i])), sat_u32(std::round(ex[2 * i + 1])), 0.0f});
    auto pts = detect_key_points(im, (uint32_t)t->grid, cur);
    int m = (int)pts.size();
    std::vector<float> a0(6 * m), a1(6 * m);
    std::vector<uint8_t> v(m);
    for (int i = 0; i < m; ++i) {
        float* a = &a0[6 * i];
        a[0] = 1.0f; a[1] = 0.0f; a[2] = 0.0f; a[3] = 1.0f;
        a[4] = (float)pts[i].x;
        a[5] = (float)pts[i].y;
    }
    orc_track_points(cur0.data(), cur1.data(), t->w, t->h, t->levels, a0.data(), m, t->max_iter,
                     t->thresh, a1.data(), v.data(), t->threads);
    // feature_tracker.rs:162-170, canonical order = ascending detection index
    for (int i = 0; i < m; ++i) {
        if (!v[i]) continue;
        orc_feature f0, f1;
        f0.id = f1.id = t->last_id;
        memcpy(f0.aff, &a0[6 * i], 24);
        memcpy(f1.aff, &a1[6 * i], 24);
        f0.x = f0.aff[4]; f0.y = f0.aff[5];
        f1.x = f1.aff[4]; f1.y = f1.aff[5];
        t->map0.push_back(f0);
        t->map1.push_back(f1);
        t->last_id += 1;
    }
    t->prev0.swap(cur0);
    t->prev1.swap(cur1);
    t->has_prev = true;
    int nl = 0, nr = 0;
    for (const auto& f : t->map0)
        if (nl < cap_l) out_l[nl++] = f;
    for (const auto& f : t->map1)
        if (nr < cap_r) out_r[nr++] = f;
    *n_l = nl;
    *n_r = nr;
    return 0;
}

void orc_tracker_remove_ids(orc_tracker* t, const uint64_t* ids, int n) {
    auto rm = [&](std::vector<orc_feature>& m) {
        std::vector<orc_feature> out;
        for (const auto& f : m) {
            bool drop = false;
            for (int i = 0; i < n; ++i) drop = drop || (ids[i] == f.id);
            if (!drop) out.push_back(f);
        }
        m.swap(out);
    };
    rm(t->map0);
    rm(t->map1);
}

}  // extern "C"
