// ft_detect.hip -- feature_tracker/ crate variant: Shi-Tomasi detection (gfx950).
//
// Replaces add_points / shi_tomasi_score / suppress_non_maximum / contains_greater_value
// (feature_tracker/src/feature_tracker/feature_detection.rs:47-285) with imageproc 0.26's
// horizontal/vertical_filter and suppress::local_maxima and image 0.25's fast_blur restated as
// in oracle/ft_oracle.cpp.  Bit-exact with the oracle (same f32 operations, same order).
//
//   Kg  grad:      one lane per pixel, [-1, 0, 1] correlation (clamp to edge) -> dxx, dyy, dxy
//   Kb  box half:  fast_blur's running box sum, one lane per (plane, row) -- the reference's
//                  sequential f32 sum is kept -- output transposed (coalesced stores); 6 launches
//   Ks  score:     one lane per pixel
//   Kn  NMS:       one lane per (r+1) x (r+1) block (+ the tracked positions, rounded)
//   Kl  local max: one workgroup per block row; survivors ranked in (y, x) order in LDS
//   Ka  assemble:  one workgroup: surviving tracks, then new corners with consecutive ids
#include <cmath>
#include <stdexcept>

#include "ft.hpp"

namespace rsvio {
namespace ft {

namespace {

__device__ __forceinline__ uint32_t sat_u32(float v) {
    if (!(v > 0.0f)) return 0u;
    if (v >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)v;
}

// feature_detection.rs:90-119: dx, dy by imageproc horizontal/vertical_filter([-1, 0, 1]) --
// correlation, pads by continuity, acc = 0; acc = acc + p * k in kernel order -- then products.
__global__ __launch_bounds__(256) void ft_grad_kernel(const float* __restrict__ im, int w, int h,
                                                      float* __restrict__ planes) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = w * h;
    if (idx >= n) return;
    const int y = idx / w, x = idx - y * w;
    const int xm = x > 0 ? x - 1 : 0, xp = x + 1 < w ? x + 1 : w - 1;
    const int ym = y > 0 ? y - 1 : 0, yp = y + 1 < h ? y + 1 : h - 1;
    const float c = im[idx];
    float gx = 0.0f + im[(size_t)y * w + xm] * -1.0f;
    gx = gx + c * 0.0f;
    gx = gx + im[(size_t)y * w + xp] * 1.0f;
    float gy = 0.0f + im[(size_t)ym * w + x] * -1.0f;
    gy = gy + c * 0.0f;
    gy = gy + im[(size_t)yp * w + x] * 1.0f;
    planes[idx] = gx * gx;
    planes[(size_t)n + idx] = gy * gy;
    planes[2 * (size_t)n + idx] = gx * gy;
}

// image 0.25 fast_blur horizontal_fast_blur_half: per row a running sum over a (2r+1) window
// (clamp-to-edge), value = clamp(sum / (2r + 1), 0, 1), written transposed.  The running sum is
// the reference's sequential f32 recurrence, so each (plane, row) is one lane's serial loop.
__global__ __launch_bounds__(64) void ft_boxblur_half(const float* __restrict__ in, float* __restrict__ out,
                                                      int width, int rows, int r, long plane) {
    const int row = blockIdx.x * 64 + threadIdx.x;
    if (row >= rows) return;
    const float* __restrict__ s = in + blockIdx.y * plane + (size_t)row * width;
    float* __restrict__ d = out + blockIdx.y * plane + row;
    const int last = width - 1;
    float val = -0.0f;  // Rust's float Sum starts from -0.0
    for (int x = -r; x <= r; ++x) val = val + s[min(max(x, 0), last)];
    const float den = 2.0f * (float)r + 1.0f;
    // the window's trailing / leading samples are independent of the running sum: load ahead
    constexpr int U = 8;
    int col = 0;
    for (; col + U <= width; col += U) {
        float a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = s[max(col + u - r, 0)];
            b[u] = s[min(col + u + r + 1, last)];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float v = val / den;
            v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
            d[(size_t)(col + u) * rows] = v;
            val = val - a[u] + b[u];
        }
    }
    for (; col < width; ++col) {
        float v = val / den;
        v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
        d[(size_t)col * rows] = v;
        val = val - s[max(col - r, 0)] + s[min(col + r + 1, last)];
    }
}

// feature_detection.rs:134-155
__global__ __launch_bounds__(256) void ft_score_kernel(const float* __restrict__ planes, int n,
                                                       float* __restrict__ score) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float dxx = planes[i], dyy = planes[(size_t)n + i], dxy = planes[2 * (size_t)n + i];
    const float trace = dxx + dyy;
    const float det = dxx * dyy - dxy * dxy;
    float delta = trace * trace - 4.0f * det;
    delta = delta > 0.0f ? delta : 0.0f;  // f32::max(x, 0.0)
    score[i] = 500.0f * fabsf(trace - sqrtf(delta));
}

__device__ __forceinline__ bool lex_less(uint32_t ax, uint32_t ay, uint32_t bx, uint32_t by) {
    return ax < bx || (ax == bx && ay < by);
}

// contains_greater_value (feature_detection.rs:259-285)
__device__ __forceinline__ bool contains_greater(const float* __restrict__ s, int w, uint32_t x, uint32_t y, float v,
                                                 uint32_t y0, uint32_t y1, uint32_t x0, uint32_t x1) {
    for (uint32_t cy = y0; cy < y1; ++cy)
        for (uint32_t cx = x0; cx < x1; ++cx) {
            const float ci = s[(size_t)cy * w + cx];
            if (ci < v) continue;
            if (ci > v || lex_less(cx, cy, x, y)) return true;
        }
    return false;
}

// suppress_non_maximum (feature_detection.rs:171-253), one lane per (r+1) x (r+1) block; lanes
// past the blocks publish the tracked positions (add_points :61-66 rounds them to u32).
__global__ __launch_bounds__(256) void ft_nms_kernel(const float* __restrict__ s, int w, int h, int r, float thr,
                                                     int nbx, int nby, uint32_t* __restrict__ nms,
                                                     float* __restrict__ nms_score, uint32_t* __restrict__ stats,
                                                     const float2* __restrict__ txy, const uint8_t* __restrict__ tvalid,
                                                     int n_tracked, uint2* __restrict__ tpos) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int nb = nbx * nby;
    if (gid >= nb) {
        const int i = gid - nb;
        if (i < n_tracked) {
            uint2 p = make_uint2(kNone, kNone);
            if (!tvalid || tvalid[i]) {
                p.x = sat_u32(roundf(txy[i].x));
                p.y = sat_u32(roundf(txy[i].y));
                atomicMax(&stats[1], p.y + 1u > p.y ? p.y + 1u : p.y);
            }
            tpos[i] = p;
        }
        return;
    }
    const int byi = gid / nbx, bxi = gid - byi * nbx;
    const uint32_t step = (uint32_t)r + 1u;
    const uint32_t x = (uint32_t)bxi * step, y = (uint32_t)byi * step;
    const uint32_t W = (uint32_t)w, Hh = (uint32_t)h, R = (uint32_t)r;
    uint32_t bx = x, by = y;
    float best = s[(size_t)y * w + x];
    for (uint32_t cy = y; cy < min(Hh, y + R + 1); ++cy)
        for (uint32_t cx = x; cx < min(W, x + R + 1); ++cx) {
            const float ci = s[(size_t)cy * w + cx];
            if (ci < best) continue;
            if (ci > best || lex_less(cx, cy, bx, by)) {
                bx = cx;
                by = cy;
                best = ci;
            }
        }
    uint32_t out = kNone;
    if (best >= thr) {
        const uint32_t x0 = bx >= R ? bx - R : 0, x1 = x, x2 = min(W, x + R + 1), x3 = min(W, bx + R + 1);
        const uint32_t y0 = by >= R ? by - R : 0, y1 = y, y2 = min(Hh, y + R + 1), y3 = min(Hh, by + R + 1);
        bool failed = contains_greater(s, w, bx, by, best, y0, y1, x0, x3);
        failed |= contains_greater(s, w, bx, by, best, y1, y2, x0, x1);
        failed |= contains_greater(s, w, bx, by, best, y1, y2, x2, x3);
        failed |= contains_greater(s, w, bx, by, best, y2, y3, x0, x3);
        if (!failed) {
            out = bx | (by << 16);
            atomicMax(&stats[0], __float_as_uint(best) + 1u);  // scores are >= 0: bit order = value order
            atomicMax(&stats[1], by + 1u);
        }
    }
    nms[gid] = out;
    nms_score[gid] = best;
}

// imageproc suppress::local_maxima (feature_detection.rs:68) + the filter of :70-79, one
// workgroup per NMS block row.  A corner survives unless some candidate in rows
// [y - md, min(y + md + 1, height)) and columns [x - md, x + md] has a greater score, or an equal
// score at a smaller (y, x); height = the largest candidate y.  Tracked features (score
// max + 1) are candidates but never survivors.  Survivors are ranked in (y, x) order.
__global__ __launch_bounds__(1024) void ft_local_max_kernel(const uint32_t* __restrict__ nms,
                                                            const float* __restrict__ nms_score,
                                                            const uint32_t* __restrict__ stats, int w, int h, int r,
                                                            int nbx, int nby, int md, const uint2* __restrict__ tpos,
                                                            int n_tracked, uint32_t* __restrict__ staging,
                                                            int* __restrict__ row_count) {
    __shared__ uint2 tl[1024];
    __shared__ int scan[1024];
    const int by = blockIdx.x, bx = threadIdx.x;
    const uint32_t step = (uint32_t)r + 1u, MD = (uint32_t)md;
    const uint32_t c = bx < nbx ? nms[by * nbx + bx] : kNone;
    const bool has = c != kNone;
    const uint32_t cx = c & 0xFFFFu, cy = c >> 16;
    const float cs = has ? nms_score[by * nbx + bx] : 0.0f;
    const uint32_t height = stats[1] > 0u ? stats[1] - 1u : 0u;
    const uint32_t lo = MD > cy ? 0u : cy - MD;
    const uint32_t hi = cy + MD + 1u > height ? height : cy + MD + 1u;
    bool keep = has;
    if (keep && hi > lo) {
        const int b0 = (int)(lo / step), b1 = (int)((hi - 1u) / step);
        const int c0 = (int)((cx >= MD ? cx - MD : 0u) / step);
        const int c1 = min(nbx - 1, (int)((cx + MD) / step));
        for (int yb = b0; yb <= b1 && keep; ++yb)
            for (int xb = c0; xb <= c1; ++xb) {
                const uint32_t n = nms[yb * nbx + xb];
                if (n == kNone || (yb == by && xb == bx)) continue;
                const uint32_t nx = n & 0xFFFFu, ny = n >> 16;
                if (ny < lo || ny >= hi || nx + MD < cx || nx > cx + MD) continue;
                const float ns = nms_score[yb * nbx + xb];
                if (ns > cs || (ns == cs && (ny < cy || (ny == cy && nx < cx)))) {
                    keep = false;
                    break;
                }
            }
    }
    // tracked candidates: all scored max(corner scores) + 1 (feature_detection.rs:61-66)
    const float mx = stats[0] ? __uint_as_float(stats[0] - 1u) : -INFINITY;
    const float ts = mx + 1.0f;
    for (int t0 = 0; t0 < n_tracked; t0 += 1024) {
        const int nt = min(1024, n_tracked - t0);
        __syncthreads();
        if ((int)threadIdx.x < nt) tl[threadIdx.x] = tpos[t0 + threadIdx.x];
        __syncthreads();
        if (!keep || hi <= lo) continue;
        for (int k = 0; k < nt; ++k) {
            const uint2 t = tl[k];
            if (t.x == kNone) continue;
            if (t.y < lo || t.y >= hi) continue;
            if ((unsigned long long)t.x + MD < cx || (unsigned long long)t.x > (unsigned long long)cx + MD) continue;
            if (ts > cs || (ts == cs && (t.y < cy || (t.y == cy && t.x < cx)))) {
                keep = false;
                break;
            }
        }
    }
    // add_points :70-79: new corners inside [md, w - md) x [md, h - md)
    keep = keep && cx >= MD && cx < (uint32_t)w - MD && cy >= MD && cy < (uint32_t)h - MD;
    // rank in (y, x) order: sub-row s = y - by * step first, then block column
    const uint32_t sub = has ? cy - (uint32_t)by * step : 0u;
    int base = 0;
    for (uint32_t sr = 0; sr < step; ++sr) {
        const int f = keep && sub == sr ? 1 : 0;
        __syncthreads();
        scan[threadIdx.x] = f;
        __syncthreads();
        for (int off = 1; off < (int)blockDim.x; off <<= 1) {
            const int t = (int)threadIdx.x >= off ? scan[threadIdx.x - off] : 0;
            __syncthreads();
            scan[threadIdx.x] += t;
            __syncthreads();
        }
        if (f) staging[by * nbx + base + scan[threadIdx.x] - 1] = c;
        base += scan[blockDim.x - 1];
    }
    if (threadIdx.x == 0) row_count[by] = base;
}

// Block-wide exclusive scan (blockDim.x <= 1024)
__device__ int block_exclusive_scan(int v, int* sh, int* total) {
    const int tid = threadIdx.x;
    __syncthreads();
    sh[tid] = v;
    __syncthreads();
    for (int off = 1; off < (int)blockDim.x; off <<= 1) {
        const int t = tid >= off ? sh[tid - off] : 0;
        __syncthreads();
        sh[tid] += t;
        __syncthreads();
    }
    const int incl = sh[tid];
    *total = sh[blockDim.x - 1];
    __syncthreads();
    return incl - v;
}

// feature_tracker.rs:115-176: tracked features (previous order), then the new corners with
// consecutive ids (next_id, :71-75)
__global__ __launch_bounds__(1024) void ft_assemble_kernel(Assemble A) {
    __shared__ int sh[1024];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int per = (A.n_prev + nt - 1) / nt;
    const int b = tid * per, e = min(A.n_prev, b + per);
    int cnt = 0;
    for (int i = b; i < e; ++i) cnt += A.valid[i] ? 1 : 0;
    int n_tr;
    int pos = block_exclusive_scan(cnt, sh, &n_tr);
    for (int i = b; i < e; ++i) {
        if (!A.valid[i]) continue;
        if (pos < A.cap) {
            A.ids_cur[pos] = A.ids_prev[i];
            A.xy_cur[pos] = A.xy_tracked[i];
        }
        ++pos;
    }
    // block rows -> bases (nby <= 1024 * rows_per_thread)
    const int rp = (A.nby + nt - 1) / nt;
    const int r0 = tid * rp, r1 = min(A.nby, r0 + rp);
    int rc = 0;
    for (int r = r0; r < r1; ++r) rc += A.row_count[r];
    int n_new;
    int rb = block_exclusive_scan(rc, sh, &n_new);
    const unsigned long long id0 = *A.last_id;
    for (int r = r0; r < r1; ++r) {
        const int k = A.row_count[r];
        for (int j = 0; j < k; ++j) {
            const int o = n_tr + rb + j;
            if (o < A.cap) {
                const uint32_t c = A.staging[r * A.nbx + j];
                A.ids_cur[o] = id0 + (unsigned long long)(rb + j);
                A.xy_cur[o] = make_float2((float)(c & 0xFFFFu), (float)(c >> 16));
            }
        }
        rb += k;
    }
    __syncthreads();
    if (tid == 0) {
        const int total = n_tr + n_new;
        A.count_out[0] = min(total, A.cap);
        A.count_out[1] = n_tr;
        A.count_out[2] = total > A.cap ? 1 : 0;
        *A.last_id = id0 + (unsigned long long)n_new;
    }
}

}  // namespace

// image 0.25 fast_blur boxes_for_gauss (f32)
void boxes_for_gauss(float sigma, int n, int* out) {
    const float w_ideal = std::sqrt((12.0f * (sigma * sigma) / (float)n) + 1.0f);
    float w_l = std::floor(w_ideal);
    if (std::fmod(w_l, 2.0f) == 0.0f) w_l -= 1.0f;
    const float w_u = w_l + 2.0f;
    const float m_ideal = 0.25f * (float)n * (w_l + 3.0f) - 3.0f * (sigma * sigma) * (1.0f / (w_l + 1.0f));
    const int m = (int)std::round(m_ideal);
    for (int i = 0; i < n; ++i) out[i] = i < m ? (int)w_l : (int)w_u;
}

void enqueue_score(const DetectBufs& D, const float* fine, hipStream_t s) {
    const int n = D.w * D.h;
    hipLaunchKernelGGL(ft_grad_kernel, dim3((n + 255) / 256), dim3(256), 0, s, fine, D.w, D.h, D.planes);
    RSVIO_HIP(hipGetLastError());
    for (int k = 0; k < 3; ++k) {
        const int r = (D.boxes[k] - 1) / 2;
        hipLaunchKernelGGL(ft_boxblur_half, dim3((D.h + 63) / 64, 3), dim3(64), 0, s, D.planes, D.tmp, D.w, D.h, r,
                           (long)n);
        RSVIO_HIP(hipGetLastError());
        hipLaunchKernelGGL(ft_boxblur_half, dim3((D.w + 63) / 64, 3), dim3(64), 0, s, D.tmp, D.planes, D.h, D.w, r,
                           (long)n);
        RSVIO_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(ft_score_kernel, dim3((n + 255) / 256), dim3(256), 0, s, D.planes, n, D.score);
    RSVIO_HIP(hipGetLastError());
}

void enqueue_select(const DetectBufs& D, float threshold, int min_dist, const float2* tracked_xy,
                    const uint8_t* tracked_valid, int n_tracked, hipStream_t s) {
    if (n_tracked > D.tpos_cap) throw std::invalid_argument("too many tracked features");
    if (D.nbx > 1024) throw std::invalid_argument("image too wide for the local-maxima workgroup");
    RSVIO_HIP(hipMemsetAsync(D.stats, 0, 2 * sizeof(uint32_t), s));
    const int total = D.nbx * D.nby + n_tracked;
    hipLaunchKernelGGL(ft_nms_kernel, dim3((total + 255) / 256), dim3(256), 0, s, D.score, D.w, D.h, D.r, threshold,
                       D.nbx, D.nby, D.nms, D.nms_score, D.stats, tracked_xy, tracked_valid, n_tracked, D.tpos);
    RSVIO_HIP(hipGetLastError());
    const int threads = ((D.nbx + 63) / 64) * 64;
    hipLaunchKernelGGL(ft_local_max_kernel, dim3(D.nby), dim3(threads), 0, s, D.nms, D.nms_score, D.stats, D.w, D.h,
                       D.r, D.nbx, D.nby, min_dist, D.tpos, n_tracked, D.staging, D.row_count);
    RSVIO_HIP(hipGetLastError());
}

void enqueue_assemble(const Assemble& A, hipStream_t s) {
    hipLaunchKernelGGL(ft_assemble_kernel, dim3(1), dim3(1024), 0, s, A);
    RSVIO_HIP(hipGetLastError());
}

}  // namespace ft
}  // namespace rsvio
