// lk_track.hip -- K2: coarse-to-fine inverse-compositional SE(2) LK with the 52-point pattern,
// forward + backward + consistency check, one wavefront per feature (gfx950, wave64).
//
// Replaces track_points / track_one_point / track_point_at_level
// (src/feature_tracker/feature_tracker.rs:252-395) and Pattern52::{new, set_data_jac_se2,
// residual} (src/feature_tracker/patch.rs:75-232).
//
// Mapping: lane i < 52 owns pattern point i (its offset, template intensity, its column of
// H^-1 J^T, its bilinear sample).  Everything the reference sums over the 52 points is summed
// in the reference's order -- sequential add chains over lanes 0..51, staged through LDS and
// read back by broadcast ds_read_b128, several independent chains interleaved -- so
// the result is bit-identical to the scalar Rust/oracle arithmetic (no FMA contraction; the
// quotients exact through an f64 reciprocal, se3.hpp div_rcp; the norm tests exact against
// squared midpoints; sin/cos = glibc's sinf/cosf restated, trig.hpp).
#include "lk_track.hpp"
#include "se3.hpp"
#include "trig.hpp"

namespace rsvio {

namespace {

RSVIO_DBG_DECL

constexpr int NP = 52;

// diagnostic phase accumulators (stamps build only): cycles per phase summed over a block's
// iterations into g_dbg[block][16..20] (tools/lk_stamps.py)
#ifdef RSVIO_STAMPS
#define LK_CLK(v)                                  \
    __builtin_amdgcn_s_waitcnt(0);                 \
    const unsigned long long v = clock64()
#define LK_ACC(slot, a, b)                                                  \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_dbg[blockIdx.x * 32 + (slot)] += (b) - (a)
#else
#define LK_CLK(v)
#define LK_ACC(slot, a, b)
#endif
constexpr int kXcds = 8;  // MI355X: 8 XCDs, workgroups dispatched round-robin

// patch.rs:19-72 -- the 52-point pattern (pixel offsets before the 1/2 scale of :126)
__constant__ int8_t kPattern[64][2] = {
    {-3, 7},  {-1, 7},  {1, 7},   {3, 7},   {-5, 5},  {-3, 5},  {-1, 5},  {1, 5},   {3, 5},
    {5, 5},   {-7, 3},  {-5, 3},  {-3, 3},  {-1, 3},  {1, 3},   {3, 3},   {5, 3},   {7, 3},
    {-7, 1},  {-5, 1},  {-3, 1},  {-1, 1},  {1, 1},   {3, 1},   {5, 1},   {7, 1},   {-7, -1},
    {-5, -1}, {-3, -1}, {-1, -1}, {1, -1},  {3, -1},  {5, -1},  {7, -1},  {-7, -3}, {-5, -3},
    {-3, -3}, {-1, -3}, {1, -3},  {3, -3},  {5, -3},  {7, -3},  {-5, -5}, {-3, -5}, {-1, -5},
    {1, -5},  {3, -5},  {5, -5},  {-3, -7}, {-1, -7}, {1, -7},  {3, -7}};

// N independent sequential f32 sums over lanes 0..51, in lane order (the reference's loop order):
// every lane stages its N values in LDS (row i = value i, padded stride), lane i then runs chain
// i alone -- 52 dependent adds, the N chains side by side in N lanes -- and the sums are
// broadcast back by readlane.  FROM_ZERO: acc = 0; acc += v_k (Rust `sum += x` loops); otherwise
// acc = v_0; acc = v_k + acc (nalgebra gemv / gemm column accumulation).  All lanes end with
// the same sums.  sh: N * kChainLd floats of this wave's LDS.
constexpr int kChainLd = 68;  // row stride (floats): 16-B aligned rows on distinct banks

template <int N, bool FROM_ZERO>
__device__ __forceinline__ void lane_chains(const float (&v)[N], float (&out)[N], float* sh, int lane) {
#pragma unroll
    for (int i = 0; i < N; ++i) sh[i * kChainLd + lane] = v[i];
    __builtin_amdgcn_wave_barrier();
    const float4* row = reinterpret_cast<const float4*>(sh + (lane < N ? lane : 0) * kChainLd);
    float4 xs[NP / 4];
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) xs[q] = row[q];
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) {
        const float4 x = xs[q];
        if (!FROM_ZERO && q == 0)
            acc = x.x;
        else
            acc = acc + x.x;
        acc = acc + x.y;
        acc = acc + x.z;
        acc = acc + x.w;
    }
    // all 13 row reads issued before the first add, consumed in order as they land (the chain
    // then waits on LDS latency once, not once per row: the scheduler otherwise interleaves
    // reads and adds two rows deep when registers are tight)
    __builtin_amdgcn_sched_group_barrier(0x100, NP / 4, 0);  // DS reads
    __builtin_amdgcn_sched_group_barrier(0x002, NP, 0);      // the chain's VALU adds
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), i));
}

struct LevelImg {
    const uint8_t* __restrict__ p;
    uint32_t w, h;
};

// image_utilities.rs:75-80
__device__ __forceinline__ bool inbound(const LevelImg& im, float x, float y, uint32_t r) {
    uint32_t xi = sat_u32(roundf(x)), yi = sat_u32(roundf(y));
    return xi >= r && yi >= r && xi < im.w - r && yi < im.h - r;
}

__device__ __forceinline__ float px(const LevelImg& im, uint32_t x, uint32_t y) {
    return (float)im.p[(size_t)y * im.w + x];
}

// image_utilities.rs:5-66
__device__ __forceinline__ void image_grad(const LevelImg& im, float x, float y, float out[3]) {
    uint32_t ix = (uint32_t)floorf(x), iy = (uint32_t)floorf(y);
    float dx = x - (float)ix, dy = y - (float)iy;
    float ddx = 1.0f - dx, ddy = 1.0f - dy;
    float p00 = px(im, ix, iy), p10 = px(im, ix + 1, iy), p01 = px(im, ix, iy + 1), p11 = px(im, ix + 1, iy + 1);
    float pm0 = px(im, ix - 1, iy), pm1 = px(im, ix - 1, iy + 1);
    float p20 = px(im, ix + 2, iy), p21 = px(im, ix + 2, iy + 1);
    float p0m = px(im, ix, iy - 1), p1m = px(im, ix + 1, iy - 1);
    float p02 = px(im, ix, iy + 2), p12 = px(im, ix + 1, iy + 2);
    float res0 = ddx * ddy * p00 + ddx * dy * p01 + dx * ddy * p10 + dx * dy * p11;
    float res_mx = ddx * ddy * pm0 + ddx * dy * pm1 + dx * ddy * p00 + dx * dy * p01;
    float res_px = ddx * ddy * p10 + ddx * dy * p11 + dx * ddy * p20 + dx * dy * p21;
    float res_my = ddx * ddy * p0m + ddx * dy * p00 + dx * ddy * p1m + dx * dy * p10;
    float res_py = ddx * ddy * p01 + ddx * dy * p02 + dx * ddy * p11 + dx * dy * p12;
    out[0] = res0;
    out[1] = 0.5f * (res_px - res_mx);
    out[2] = 0.5f * (res_py - res_my);
}

// Affine2 as a 3x3 with implicit last row [0 0 1] kept explicitly for exact product order.
struct Aff {
    float m00, m01, m02, m10, m11, m12, m20, m21, m22;
};

// nalgebra 3x3 gemm: C[i][j] = (A[i][0] B[0][j] + A[i][1] B[1][j]) + A[i][2] B[2][j]
__device__ __forceinline__ Aff mul3(const Aff& A, const Aff& B) {
    Aff C;
#define RSV_EL(i, j) ((A.m##i##2 * B.m2##j) + ((A.m##i##1 * B.m1##j) + (A.m##i##0 * B.m0##j)))
    C.m00 = RSV_EL(0, 0); C.m01 = RSV_EL(0, 1); C.m02 = RSV_EL(0, 2);
    C.m10 = RSV_EL(1, 0); C.m11 = RSV_EL(1, 1); C.m12 = RSV_EL(1, 2);
    C.m20 = RSV_EL(2, 0); C.m21 = RSV_EL(2, 1); C.m22 = RSV_EL(2, 2);
#undef RSV_EL
    return C;
}

// image_utilities.rs:82-106, twist [vx, vy, theta]; sin/cos = glibc sinf/cosf (trig.hpp)
__device__ __forceinline__ Aff se2_exp(float a0, float a1, float theta) {
    double rth = rcp_f64((double)theta);  // beside sincosf (the quotients' divisor)
    // pinned here: the compiler otherwise sinks the reciprocal into the branch that uses it,
    // after sincosf, and its ~7 dependent f64 ops land on the chain instead of beside it
    __asm__ volatile("" : "+v"(rth));
    float s, c;
    libm_trig::sincosf(theta, &s, &c);
    // both forms, then a select (no branch between sincosf and the update)
    const float th2 = theta * theta;
    const float sin_small = 1.0f - (1.0f / 6.0f) * th2;
    const float omc_small = 0.5f * theta - (1.0f / 24.0f) * theta * th2;
    const bool small = fabsf(theta) < __FLT_EPSILON__;
    const float sin_by = small ? sin_small : div_rcp(s, rth);         // s / theta
    const float omc_by = small ? omc_small : div_rcp(1.0f - c, rth);  // (1 - c) / theta
    Aff E;
    E.m00 = c; E.m01 = -s; E.m10 = s; E.m11 = c;
    E.m02 = sin_by * a0 - omc_by * a1;
    E.m12 = omc_by * a0 + sin_by * a1;
    E.m20 = 0.0f; E.m21 = 0.0f; E.m22 = 1.0f;
    return E;
}

// nalgebra Cholesky (3x3, lower) + solve_mut(identity); uniform across lanes.
__device__ __forceinline__ bool chol_inv3(float A[3][3], float X[3][3]) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int k = 0; k < j; ++k) {
            float factor = -A[j][k];
#pragma unroll
            for (int r = j; r < 3; ++r) A[r][j] = factor * A[r][k] + A[r][j];
        }
        float diag = A[j][j];
        if (!(diag != 0.0f && diag >= 0.0f)) return false;
        float den = sqrtf(diag);
        A[j][j] = den;
#pragma unroll
        for (int r = j + 1; r < 3; ++r) A[r][j] = A[r][j] / den;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float b[3] = {0.0f, 0.0f, 0.0f};
        b[c] = 1.0f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            float coeff = b[i] / A[i][i];
            b[i] = coeff;
#pragma unroll
            for (int r = i + 1; r < 3; ++r) b[r] = (-coeff) * A[r][i] + b[r];
        }
#pragma unroll
        for (int i = 2; i >= 0; --i) {
            float dot = 0.0f;
#pragma unroll
            for (int r = i + 1; r < 3; ++r) dot = dot + A[r][i] * b[r];
            b[i] = (b[i] - dot) / A[i][i];
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) X[r][c] = b[r];
    }
    return true;
}

struct Template {
    float data;   // normalised intensity of this lane's point (-1 invalid)
    float h0, h1, h2;  // this lane's column of H^-1 J^T
};

__device__ __forceinline__ LevelImg level_of(const uint8_t* pyr, uint32_t w, uint32_t h, int i) {
    LevelImg L;
    L.p = pyr + level_offset(w, h, i);
    L.w = level_w(w, i);
    L.h = level_h(h, i);
    return L;
}

// Pattern52::new (patch.rs:124-162 + set_data_jac_se2 :75-123) for every level of a pyramid at
// once, level i at (posx, posy) / 2^i -- the templates track_one_point builds level by level
// (feature_tracker.rs:310-314).  They are independent, so one pass overlaps them: the 12-pixel
// image_grad crosses of all levels are in flight together, the 4L normalisation sums run as one
// lane_chains<4L> (chain j in lane j, each in the reference's order) and the 6L entries of H
// as one lane_chains<6L>; the L 3x3 Cholesky solves interleave.  Every value is the one the
// per-level build computes (same f32 operations), so tracks stay bit-exact.
// Levels [L0, L0 + K) of the L templates (K <= 4 keeps the chain values within the VGPR file).
template <int L, int L0, int K>
__device__ void make_templates_part(const uint8_t* pyr, uint32_t w, uint32_t h, float posx, float posy, int lane,
                                    Template (&T)[L], bool (&ok)[L], float* sh) {
    const bool act = lane < NP;
    const float ox = act ? (float)kPattern[lane][0] : 0.0f;
    const float oy = act ? (float)kPattern[lane][1] : 0.0f;
    const float jw02 = -oy / 2.0f, jw12 = ox / 2.0f;
    float v[K], J0[K], J1[K], J2[K];
    bool in[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const float sdn = (float)(1 << (L0 + i));
        const LevelImg im = level_of(pyr, w, h, L0 + i);
        const float qx = posx / sdn + ox / 2.0f, qy = posy / sdn + oy / 2.0f;
        in[i] = act && inbound(im, qx, qy, 2);
        // every lane samples (an out-of-bound one at a safe dummy spot, its values discarded):
        // no branch around the loads, so all levels' gathers are in flight together
        // (levels under 5 x 5 have no in-bound point and are not sampled at all)
        float vg[3] = {0.0f, 0.0f, 0.0f};
        if (im.w >= 5 && im.h >= 5) image_grad(im, in[i] ? qx : 2.0f, in[i] ? qy : 2.0f, vg);
        v[i] = in[i] ? vg[0] : 0.0f;
        J0[i] = in[i] ? vg[1] * 1.0f + vg[2] * 0.0f : 0.0f;
        J1[i] = in[i] ? vg[1] * 0.0f + vg[2] * 1.0f : 0.0f;
        J2[i] = in[i] ? vg[1] * jw02 + vg[2] * jw12 : 0.0f;
    }
    float x4[4 * K], s4[4 * K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        x4[4 * i] = in[i] ? v[i] : 0.0f;
        x4[4 * i + 1] = in[i] ? J0[i] : 0.0f;
        x4[4 * i + 2] = in[i] ? J1[i] : 0.0f;
        x4[4 * i + 3] = in[i] ? J2[i] : 0.0f;
    }
    lane_chains<4 * K, true>(x4, s4, sh, lane);
    float x6[6 * K], h6[6 * K], mean[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const float sum = s4[4 * i], gs0 = s4[4 * i + 1], gs1 = s4[4 * i + 2], gs2 = s4[4 * i + 3];
        const int nvalid = __popcll(__ballot(in[i]));
        mean[i] = sum / (float)nvalid;
        const float mean_inv = (float)nvalid / sum;
        float data = in[i] ? v[i] : -1.0f;
        float a0 = J0[i], a1 = J1[i], a2 = J2[i];
        if (data >= 0.0f) {
            a0 = a0 + (-(gs0 * data / sum));
            a1 = a1 + (-(gs1 * data / sum));
            a2 = a2 + (-(gs2 * data / sum));
            data *= mean_inv;
        } else {
            a0 = a1 = a2 = 0.0f;
        }
        J0[i] = a0 * mean_inv;
        J1[i] = a1 * mean_inv;
        J2[i] = a2 * mean_inv;
        T[L0 + i].data = data;
        x6[6 * i] = J0[i] * J0[i];
        x6[6 * i + 1] = J0[i] * J1[i];
        x6[6 * i + 2] = J0[i] * J2[i];
        x6[6 * i + 3] = J1[i] * J1[i];
        x6[6 * i + 4] = J1[i] * J2[i];
        x6[6 * i + 5] = J2[i] * J2[i];
    }
    lane_chains<6 * K, false>(x6, h6, sh, lane);
#pragma unroll
    for (int i = 0; i < K; ++i) {
        float H[3][3], Hi[3][3];
        H[0][0] = h6[6 * i]; H[0][1] = h6[6 * i + 1]; H[0][2] = h6[6 * i + 2];
        H[1][1] = h6[6 * i + 3]; H[1][2] = h6[6 * i + 4]; H[2][2] = h6[6 * i + 5];
        H[1][0] = H[0][1];
        H[2][0] = H[0][2];
        H[2][1] = H[1][2];
        Template& t = T[L0 + i];
        ok[L0 + i] = chol_inv3(H, Hi);
        if (!ok[L0 + i]) continue;
        t.h0 = Hi[0][2] * J2[i] + (Hi[0][1] * J1[i] + Hi[0][0] * J0[i]);
        t.h1 = Hi[1][2] * J2[i] + (Hi[1][1] * J1[i] + Hi[1][0] * J0[i]);
        t.h2 = Hi[2][2] * J2[i] + (Hi[2][1] * J1[i] + Hi[2][0] * J0[i]);
        const bool fin = !act || (isfinite(t.h0) && isfinite(t.h1) && isfinite(t.h2) && isfinite(t.data));
        const bool all_fin = __ballot(!fin) == 0ull;
        ok[L0 + i] = (mean[i] > __FLT_EPSILON__) && all_fin;
    }
}

template <int L>
__device__ void make_templates(const uint8_t* pyr, uint32_t w, uint32_t h, float posx, float posy, int lane,
                               Template (&T)[L], bool (&ok)[L], float* sh) {
    make_templates_part<L, 0, (L < 4 ? L : 4)>(pyr, w, h, posx, posy, lane, T, ok, sh);
    if constexpr (L > 4) make_templates_part<L, 4, L - 4>(pyr, w, h, posx, posy, lane, T, ok, sh);
}

// track_point_at_level (feature_tracker.rs:344-395) with Pattern52::residual (patch.rs:163-232).
// One iteration is a chain of dependent latencies (gather -> 52-add sum -> residual -> three
// 52-add increment chains -> exp/update), so it is written without branches until its end:
// out-of-bound lanes sample a safe pixel and discard it (no exec-masked region around the
// loads), the residual and increment are formed even when a check has already failed, and the
// norm, SE(2) exp, product and in-bound test of the trial run side by side.  The checks are then
// taken in the reference's order -- sum, residual count, finite increment, norm > 1e6 (all
// "return false"), convergence ("break" before the update), in-bound after it -- so every outcome
// and every kept value is the one the sequential code produces.
// The norm tests without the square root: for x = i0^2 + i1^2 + i2^2 (f32, the reference's order)
// and a positive normal f32 t, RN(sqrt(x)) < t  <=>  x < m^2 with m the midpoint of t and its
// predecessor (m has a 25-bit odd significand, so sqrt(x) == m is impossible and m^2 is exact in
// f64); likewise RN(sqrt(x)) > 1e6  <=>  x > m'^2, m' the midpoint of 1e6 and its successor.
__device__ __forceinline__ double sq_mid(float a, float b) {
    const double m = 0.5 * ((double)a + (double)b);
    return m * m;
}

__device__ bool track_at_level(const LevelImg& im, const Template& T, float patx, float paty, int lane,
                               Aff& A, int max_iter, float thresh, float* sh) {
    const bool act = lane < NP;
    const float wlim = (float)(im.w - 2), hlim = (float)(im.h - 2);
    const bool tval = T.data >= 0.0f;
    const float mh0 = -T.h0, mh1 = -T.h1, mh2 = -T.h2;
    const bool thr_mid = thresh >= __FLT_MIN__ && thresh <= __FLT_MAX__;  // (else the sqrt form)
    const double thr2 = thr_mid ? sq_mid(__int_as_float(__float_as_int(thresh) - 1), thresh) : 0.0;
    const double big2 = sq_mid(1e6f, __int_as_float(__float_as_int(1e6f) + 1));
    // the in-bound test of an update (image_utilities::inbound after transform *= exp) is taken
    // with the next iteration's first test (before any other outcome of that iteration), or after
    // the loop: no branch between the update and the next gather (the iteration computed on an
    // out-of-bound transform is discarded, as the reference never computes it)
    bool oob = false;
    for (int it = 0; it < max_iter; ++it) {
#ifdef RSVIO_STAMPS
        if (lane == 0 && blockIdx.x < 4096) g_dbg[blockIdx.x * 32 + 15] += 1;
#endif
        LK_CLK(t0);
        float x = A.m00 * patx;
        x = A.m01 * paty + x;
        float y = A.m10 * patx;
        y = A.m11 * paty + y;
        x = x + A.m02;
        y = y + A.m12;
        const bool inb = act && x >= 2.0f && y >= 2.0f && x < wlim && y < hlim;
        const float sx = inb ? x : 2.0f, sy = inb ? y : 2.0f;
        const uint32_t ix = (uint32_t)floorf(sx), iy = (uint32_t)floorf(sy);
        const float dx = sx - (float)ix, dy = sy - (float)iy;
        const float ddx = 1.0f - dx, ddy = 1.0f - dy;
        const uint8_t* r0 = im.p + (size_t)iy * im.w + ix;
        const uint8_t* r1 = r0 + im.w;
        const float p00 = (float)r0[0], p10 = (float)r0[1], p01 = (float)r1[0], p11 = (float)r1[1];
        const float v = ddx * ddy * p00 + ddx * dy * p01 + dx * ddy * p10 + dx * dy * p11;
        const int nv = __popcll(__ballot(inb));
        const bool use = inb && v >= 0.0f && tval;
        const int nres = __popcll(__ballot(use));
        LK_CLK(t1);
        LK_ACC(16, t0, t1);
        float sum;
        {
            const float x1[1] = {inb ? v : 0.0f};
            float s1[1];
            lane_chains<1, true>(x1, s1, sh, lane);
            sum = s1[0];
        }
        const float r = use ? (div_rcp((float)nv * v, rcp_f64((double)sum)) - T.data) : 0.0f;  // nv v / sum
        float inc[3];
        LK_CLK(t2);
        LK_ACC(17, t1, t2);
        {
            const float x3[3] = {mh0 * r, mh1 * r, mh2 * r};
            lane_chains<3, false>(x3, inc, sh, lane);
        }
        LK_CLK(t3);
        LK_ACC(18, t2, t3);
        const float i0 = inc[0], i1 = inc[1], i2 = inc[2];
        const bool fin = isfinite(i0) && isfinite(i1) && isfinite(i2);
        const float nx = i0 * i0 + i1 * i1 + i2 * i2;
#ifdef RSVIO_STAMPS
        if (lane == 0 && blockIdx.x < 4096 && !(fabsf(i2) < 0.0625f)) g_dbg[blockIdx.x * 32 + 21] += 1;
#endif
        const bool too_big = (double)nx > big2;  // nrm > 1e6 (nx = +inf included; NaN: false, as the sqrt)
        const bool conv = thr_mid ? (double)nx < thr2 : sqrtf(nx) < thresh;  // nrm < thresh
        const Aff An = mul3(A, se2_exp(i0, i1, i2));
        const bool inb2 = inbound(im, An.m02, An.m12, 2);
        LK_CLK(t4);
        LK_ACC(19, t3, t4);
        if (oob || sum < __FLT_EPSILON__ || !(nres > NP / 2) || !fin || too_big) return false;
        if (conv) break;
        A = An;
        oob = !inb2;
    }
    return !oob;
}

// track_one_point (feature_tracker.rs:292-342): the L templates first (make_templates), then
// the levels coarse to fine; an invalid template fails the call when its level is reached, as
// the reference's level-by-level build does.
template <int L>
__device__ bool track_one(const uint8_t* pyr0, const uint8_t* pyr1, uint32_t w, uint32_t h, const Aff& T0, int lane,
                          float patx, float paty, int max_iter, float thresh, Aff& out, float* sh, float* tsh) {
    uint32_t tok_mask = 0;
    {
        Template tp[L];
        bool tok[L];
        LK_CLK(m0);
        make_templates<L>(pyr0, w, h, T0.m02, T0.m12, lane, tp, tok, sh);
        LK_CLK(m1);
        LK_ACC(20, m0, m1);
        // park the templates in LDS so the level loop below is not unrolled (one inlined
        // track_at_level per direction; tsh: [level][4][64] floats of this wave)
#pragma unroll
        for (int i = 0; i < L; ++i) {
            tsh[(4 * i + 0) * 64 + lane] = tp[i].data;
            tsh[(4 * i + 1) * 64 + lane] = tp[i].h0;
            tsh[(4 * i + 2) * 64 + lane] = tp[i].h1;
            tsh[(4 * i + 3) * 64 + lane] = tp[i].h2;
            tok_mask |= tok[i] ? (1u << i) : 0u;
        }
    }
    Aff T1;
    T1.m00 = 1.0f; T1.m01 = 0.0f; T1.m10 = 0.0f; T1.m11 = 1.0f;
    T1.m20 = 0.0f; T1.m21 = 0.0f; T1.m22 = 1.0f;
    T1.m02 = T0.m02;
    T1.m12 = T0.m12;
#pragma unroll 1
    for (int i = L - 1; i >= 0; --i) {
        const float sdn = (float)(1 << i);
        T1.m02 /= sdn;
        T1.m12 /= sdn;
        if (!((tok_mask >> i) & 1u)) return false;
        Template tp;
        tp.data = tsh[(4 * i + 0) * 64 + lane];
        tp.h0 = tsh[(4 * i + 1) * 64 + lane];
        tp.h1 = tsh[(4 * i + 2) * 64 + lane];
        tp.h2 = tsh[(4 * i + 3) * 64 + lane];
        if (!track_at_level(level_of(pyr1, w, h, i), tp, patx, paty, lane, T1, max_iter, thresh, sh))
            return false;
        T1.m02 *= sdn;
        T1.m12 *= sdn;
    }
    Aff R = mul3(T0, T1);
    T1.m00 = R.m00;
    T1.m01 = R.m01;
    T1.m10 = R.m10;
    T1.m11 = R.m11;
    out = T1;
    return true;
}

template <int L>
__global__ __launch_bounds__(64) void lk_track_kernel(TrackLaunch P) {
    // XCD-aware: workgroup b runs on XCD b % 8; give each XCD a contiguous range of jobs (whole
    // batches, i.e. 2 of the 4 pyramids) so its L2 fetches only what its features read
    const int per = (P.njobs + kXcds - 1) / kXcds;
    const int job = (int)(blockIdx.x % kXcds) * per + (int)(blockIdx.x / kXcds);
    if (job >= P.njobs) return;
    const uint8_t* pyr0;
    const uint8_t* pyr1;
    const float* ain;
    float* aout;
    uint8_t* valid;
    int idx;
    if (P.table != nullptr) {
        // largest b with tstart[b] <= job (binary search over the device prefix)
        int lo = 0, hi = P.nb - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (P.tstart[mid] <= job) lo = mid; else hi = mid - 1;
        }
        const rsvio_track_batch& d = P.table[lo];
        idx = job - P.tstart[lo];
        if (idx < 0 || idx >= d.n) return;  // a malformed caller prefix never indexes out of a batch
        pyr0 = d.d_pyr0; pyr1 = d.d_pyr1; ain = d.d_aff_in; aout = d.d_aff_out; valid = d.d_valid;
    } else {
        int b = 0;
        while (b + 1 < P.nb && job >= P.start[b + 1]) ++b;
        idx = job - P.start[b];
        if (P.dcount[b] != nullptr && idx >= *P.dcount[b]) return;
        pyr0 = P.pyr0[b]; pyr1 = P.pyr1[b]; ain = P.ain[b]; aout = P.aout[b]; valid = P.valid[b];
        if (P.mask[b] != nullptr && P.mask[b][idx].w == 0) {  // an empty job (a cell without a corner)
            if (threadIdx.x == 0) valid[idx] = 0;
            return;
        }
    }
    __shared__ __attribute__((aligned(16))) float sh[6 * (L < 4 ? L : 4) * kChainLd];
    __shared__ float tsh[4 * L * 64];
    const int lane = threadIdx.x;
    const float patx = lane < NP ? (float)kPattern[lane][0] / 2.0f : 0.0f;
    const float paty = lane < NP ? (float)kPattern[lane][1] / 2.0f : 0.0f;
    const float* a = ain + 6 * (size_t)idx;
    Aff T0;
    T0.m00 = a[0]; T0.m01 = a[1]; T0.m10 = a[2]; T0.m11 = a[3]; T0.m02 = a[4]; T0.m12 = a[5];
    T0.m20 = 0.0f; T0.m21 = 0.0f; T0.m22 = 1.0f;
    Aff fwd, bwd;
#ifdef RSVIO_STAMPS
    if (lane == 0 && blockIdx.x < 4096)
        for (int k = 15; k <= 21; ++k) g_dbg[blockIdx.x * 32 + k] = 0;
#endif
    STAMP(0);
    bool ok = track_one<L>(pyr0, pyr1, P.w, P.h, T0, lane, patx, paty, P.max_iter, P.thresh, fwd, sh, tsh);
    STAMP(1);
    if (ok) ok = track_one<L>(pyr1, pyr0, P.w, P.h, fwd, lane, patx, paty, P.max_iter, P.thresh, bwd, sh, tsh);
    STAMP(2);
    if (ok) {
        // feature_tracker.rs:277-281: squared translation distance < 0.4
        float dx = T0.m02 - bwd.m02, dy = T0.m12 - bwd.m12;
        ok = (dx * dx + dy * dy) < 0.4f;
    }
    if (lane == 0) {
        float* o = aout + 6 * (size_t)idx;
        if (ok) {
            o[0] = fwd.m00; o[1] = fwd.m01; o[2] = fwd.m10; o[3] = fwd.m11; o[4] = fwd.m02; o[5] = fwd.m12;
        } else {
            for (int k = 0; k < 6; ++k) o[k] = a[k];
        }
        valid[idx] = ok ? 1 : 0;
    }
}

}  // namespace

RSVIO_DBG_READER(rsvio_dbg_lk_stamps)

void enqueue_track(const TrackLaunch& L0, hipStream_t s) {
    TrackLaunch L = L0;
    const int total = L.table != nullptr ? L.start[0] : L.start[L.nb];
    if (total <= 0) return;
    L.njobs = total;
    const int grid = ((total + kXcds - 1) / kXcds) * kXcds;
    switch (L.levels) {  // one instantiation per pyramid depth (make_templates<L>)
#define RSVIO_LK(NL) \
    case NL: hipLaunchKernelGGL(lk_track_kernel<NL>, dim3(grid), dim3(64), 0, s, L); break;
        RSVIO_LK(1) RSVIO_LK(2) RSVIO_LK(3) RSVIO_LK(4) RSVIO_LK(5) RSVIO_LK(6) RSVIO_LK(7) RSVIO_LK(8)
#undef RSVIO_LK
        default: throw std::invalid_argument("track_points: levels must be in [1, 8]");
    }
    RSVIO_HIP(hipGetLastError());
}

}  // namespace rsvio
