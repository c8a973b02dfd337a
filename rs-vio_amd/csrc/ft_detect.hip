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
//   Kn  NMS:       one lane per (r+1) x (r+1) block (+ the tracked positions, rounded), corner list
//   Kt  tracked:   one wave per tracked feature marks the corners it suppresses
//   Kc  local max: one wave per corner, lanes over the window's NMS blocks
//   Kr  rank:      one workgroup per block row; survivors ranked in (y, x) order
//   Ka  assemble:  one workgroup: surviving tracks, then new corners with consecutive ids
#include <algorithm>
#include <atomic>
#include <cmath>
#include <type_traits>
#include <stdexcept>

#include "ft.hpp"

namespace rsvio {
namespace ft {

namespace {

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
// the reference's sequential f32 recurrence, so one lane owns one row for the whole pass.
// A workgroup (8 waves) owns 64 rows and walks them in chunks of kCW columns, three deep:
//   wave 0     runs the recurrence of chunk k from LDS tile T[k & 1] into V[k & 1]
//   waves 1-7  commit chunk k+1's window (already in registers) to T[(k+1) & 1], issue the global
//              loads of chunk k+2 into registers (a whole step to land), then divide / clamp /
//              store chunk k-1 from V[(k-1) & 1] (coalesced: 64 consecutive rows of one column)
// so neither the HBM latency nor the division sits on the recurrence's path; one barrier a step
// (which waits for LDS traffic only).  NSEG = 64-column segments of a tile row (kCW + 2r + 1).
constexpr int kCW = 64;       // columns per chunk
constexpr int kVS = kCW + 1;  // LDS row stride of the running-sum buffer (odd: conflict-free)
constexpr int kBBThreads = 512;
constexpr int kHW = kBBThreads / 64 - 1;           // helper waves
constexpr int kHRows = (64 + kHW - 1) / kHW;       // tile rows per helper wave

__host__ __device__ inline int bb_stride(int r) {
    const int s = kCW + 2 * r + 1;
    return (s & 1) ? s : s + 1;  // odd row stride: lanes (rows) on distinct banks
}
__host__ inline size_t bb_lds_bytes(int r) { return sizeof(float) * (2 * 64 * (size_t)bb_stride(r) + 2 * 64 * kVS); }

template <int NSEG>
__global__ __launch_bounds__(kBBThreads) void ft_boxblur_half(const float* __restrict__ in, float* __restrict__ out,
                                                              int width, int rows, int r, long plane) {
    extern __shared__ float sm[];   // T[2][64][S] | V[2][64][kVS]  (offsets, not pointers: keeps ds_* ops)
    const int S = bb_stride(r);
    const int tbuf = 64 * S, vbase = 128 * S, vbuf = 64 * kVS;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int row0 = blockIdx.x * 64;
    const float* __restrict__ src = in + blockIdx.y * plane;
    float* __restrict__ dst = out + blockIdx.y * plane;
    const int ncol = kCW + 2 * r + 1;
    const int nch = (width + kCW - 1) / kCW;
    const int last = width - 1;
    const float den = 2.0f * (float)r + 1.0f;
    const int o = 2 * r + 1;
    // helper state: tile rows hw + kHW * m, columns lane + 64 * q (clamped addresses: every load is
    // in bounds; only the LDS commit is masked)
    const int hw = wave - 1;
    float pre[kHRows][NSEG];
    const float* rowp[kHRows];
#pragma unroll
    for (int m = 0; m < kHRows; ++m) rowp[m] = src + (size_t)min(row0 + min(hw + kHW * m, 63), rows - 1) * width;
    auto issue = [&](int c0) {
#pragma unroll
        for (int q = 0; q < NSEG; ++q) {
            const int x = min(max(c0 - r + lane + 64 * q, 0), last);
#pragma unroll
            for (int m = 0; m < kHRows; ++m) pre[m][q] = rowp[m][x];
        }
    };
    auto commit = [&](int toff) {
#pragma unroll
        for (int m = 0; m < kHRows; ++m) {
            const int rr = hw + kHW * m;
#pragma unroll
            for (int q = 0; q < NSEG; ++q)
                if (rr < 64 && lane + 64 * q < ncol) sm[toff + rr * S + lane + 64 * q] = pre[m][q];
        }
    };
    if (wave > 0) {
        issue(0);
        commit(0);
        if (nch > 1) issue(kCW);
    }
    __syncthreads();
    float val = -0.0f;  // Rust's float Sum starts from -0.0
    if (wave == 0)
        for (int j = 0; j <= 2 * r; ++j) val = val + sm[lane * S + j];
    for (int k = 0; k <= nch; ++k) {
        if (wave == 0) {
            if (k < nch) {
                const int cw = min(kCW, width - k * kCW);
                const int tr = (k & 1) * tbuf + lane * S;
                const int vr = vbase + (k & 1) * vbuf + lane * kVS;
                if (cw == kCW) {
                    // window samples of 16 columns first (independent of the running sum), then the chain
#pragma unroll
                    for (int j0 = 0; j0 < kCW; j0 += 16) {
                        float A[16], B[16], Vv[16];
#pragma unroll
                        for (int j = 0; j < 16; ++j) {
                            A[j] = sm[tr + j0 + j];
                            B[j] = sm[tr + o + j0 + j];
                        }
#pragma unroll
                        for (int j = 0; j < 16; ++j) {
                            Vv[j] = val;
                            val = (val - A[j]) + B[j];
                        }
#pragma unroll
                        for (int j = 0; j < 16; ++j) sm[vr + j0 + j] = Vv[j];
                    }
                } else {
                    for (int j = 0; j < cw; ++j) {
                        sm[vr + j] = val;
                        val = (val - sm[tr + j]) + sm[tr + j + o];
                    }
                }
            }
        } else {
            if (k + 1 < nch) commit(((k + 1) & 1) * tbuf);
            if (k + 2 < nch) issue((k + 2) * kCW);
            if (k >= 1) {
                const int t = tid - 64;
                const int c0 = (k - 1) * kCW;
                const int cw = min(kCW, width - c0);
                const int vp = vbase + ((k - 1) & 1) * vbuf;
                for (int i = t; i < 64 * cw; i += kBBThreads - 64) {
                    const int col = i >> 6, rr = i & 63;
                    if (row0 + rr < rows) {
                        float v = sm[vp + rr * kVS + col] / den;
                        v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
                        dst[(size_t)(c0 + col) * rows + row0 + rr] = v;
                    }
                }
            }
        }
        __syncthreads();
    }
}

// Any radius: one lane per row straight from global memory (the same recurrence).
__global__ __launch_bounds__(256) void ft_boxblur_half_any(const float* __restrict__ in, float* __restrict__ out,
                                                          int width, int rows, int r, long plane) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= rows) return;
    const float* __restrict__ p = in + blockIdx.y * plane + (size_t)row * width;
    float* __restrict__ dst = out + blockIdx.y * plane;
    const int last = width - 1;
    const float den = 2.0f * (float)r + 1.0f;
    float val = -0.0f;
    for (int x = -r; x < r + 1; ++x) val = val + p[min(max(x, 0), last)];
    for (int col = 0; col < width; ++col) {
        float v = val / den;
        v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
        dst[(size_t)col * rows + row] = v;
        val = (val - p[min(max(col - r, 0), last)]) + p[min(col + r + 1, last)];
    }
}

// > 64 KB of dynamic LDS needs the function attribute, once per (kernel, device)
void allow_lds(const void* fn, int bytes, int slot) {
    static std::atomic<uint32_t> done[2];
    int dev = 0;
    RSVIO_HIP(hipGetDevice(&dev));
    const uint32_t bit = 1u << (dev & 31);
    if (done[slot].load(std::memory_order_acquire) & bit) return;
    RSVIO_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done[slot].fetch_or(bit, std::memory_order_acq_rel);
}

void launch_boxblur_half(const float* in, float* out, int width, int rows, int r, long plane, hipStream_t s) {
    const int nseg = (kCW + 2 * r + 1 + 63) / 64;
    const size_t lds = bb_lds_bytes(r);
    const dim3 grid((rows + 63) / 64, 3);
    if (nseg <= 2) {
        allow_lds(reinterpret_cast<const void*>(&ft_boxblur_half<2>), (int)bb_lds_bytes(31), 0);
        hipLaunchKernelGGL(ft_boxblur_half<2>, grid, dim3(kBBThreads), lds, s, in, out, width, rows, r, plane);
    } else if (nseg == 3) {
        allow_lds(reinterpret_cast<const void*>(&ft_boxblur_half<3>), (int)bb_lds_bytes(63), 1);
        hipLaunchKernelGGL(ft_boxblur_half<3>, grid, dim3(kBBThreads), lds, s, in, out, width, rows, r, plane);
    } else {
        hipLaunchKernelGGL(ft_boxblur_half_any, dim3((rows + 255) / 256, 3), dim3(256), 0, s, in, out, width, rows, r,
                           plane);
    }
    RSVIO_HIP(hipGetLastError());
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
// Corners are appended (any order) to clist for the per-corner local-maximum test.
__global__ __launch_bounds__(256) void ft_nms_kernel(const float* __restrict__ s, int w, int h, int r, float thr,
                                                     int nbx, int nby, uint32_t* __restrict__ nms,
                                                     float* __restrict__ nms_score, uint32_t* __restrict__ stats,
                                                     const float2* __restrict__ txy, const uint8_t* __restrict__ tvalid,
                                                     int n_tracked, uint2* __restrict__ tpos,
                                                     uint8_t* __restrict__ supp, uint8_t* __restrict__ keep,
                                                     uint32_t* __restrict__ clist) {
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
            clist[atomicAdd(&stats[2], 1u)] = (uint32_t)gid;
        }
    }
    nms[gid] = out;
    nms_score[gid] = best;
    supp[gid] = 0;
    keep[gid] = 0;
}

// imageproc suppress::local_maxima (feature_detection.rs:68): candidate c survives unless some
// candidate in rows [y - md, min(y + md + 1, height)) and columns [x - md, x + md] has a greater
// score, or an equal score at a smaller (y, x); height = the largest candidate y.
__device__ __forceinline__ bool beats(uint32_t ny, uint32_t nx, float ns, uint32_t cy, uint32_t cx, float cs,
                                      uint32_t lo, uint32_t hi, unsigned long long md) {
    return ny >= lo && ny < hi && (unsigned long long)nx + md >= cx && (unsigned long long)nx <= cx + md &&
           (ns > cs || (ns == cs && (ny < cy || (ny == cy && nx < cx))));
}

// The tracked features' side: all of them score max(corner scores) + 1 (feature_detection.rs:61-66).
// One wave per tracked feature t marks the corners c it beats; t can lie in c's window only if
// |cx - tx| <= md and |cy - ty| <= md, i.e. in a (2 md + 1)^2 box of NMS blocks (lanes in parallel).
__global__ __launch_bounds__(256) void ft_tracked_suppress_kernel(const uint2* __restrict__ tpos, int n_tracked,
                                                                  const uint32_t* __restrict__ nms,
                                                                  const float* __restrict__ nms_score,
                                                                  const uint32_t* __restrict__ stats, int r, int nbx,
                                                                  int nby, int md, uint8_t* __restrict__ supp) {
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    if (i >= n_tracked) return;
    const uint2 t = tpos[i];
    if (t.x == kNone) return;
    const unsigned long long step = (unsigned long long)r + 1ull, MD = (unsigned long long)md;
    const uint32_t height = stats[1] > 0u ? stats[1] - 1u : 0u;
    const float ts = (stats[0] ? __uint_as_float(stats[0] - 1u) : -INFINITY) + 1.0f;
    const unsigned long long tx = t.x, ty = t.y;
    const long long by0 = (long long)((ty > MD ? ty - MD : 0ull) / step);
    const long long by1 = min((long long)nby - 1, (long long)((ty + MD) / step));
    const long long bx0 = (long long)((tx > MD ? tx - MD : 0ull) / step);
    const long long bx1 = min((long long)nbx - 1, (long long)((tx + MD) / step));
    if (by1 < by0 || bx1 < bx0) return;
    const int nbw = (int)(bx1 - bx0 + 1), ncell = (int)(by1 - by0 + 1) * nbw;
    for (int k = lane; k < ncell; k += 64) {
        const int q = k / nbw;
        const long long g = (by0 + q) * nbx + bx0 + (k - q * nbw);
        const uint32_t c = nms[g];
        if (c == kNone) continue;
        const uint32_t cx = c & 0xFFFFu, cy = c >> 16;
        const uint32_t lo = (uint32_t)md > cy ? 0u : cy - (uint32_t)md;
        const uint32_t hi = cy + (uint32_t)md + 1u > height ? height : cy + (uint32_t)md + 1u;
        if (beats((uint32_t)ty, (uint32_t)tx, ts, cy, cx, nms_score[g], lo, hi, MD)) supp[g] = 1;
    }
}

// The corners' side of local_maxima + the filter of add_points :70-79, one wave per corner
// (persistent waves over clist): the lanes test the window's NMS blocks in parallel.
__global__ __launch_bounds__(256) void ft_corner_max_kernel(const uint32_t* __restrict__ clist,
                                                            const uint32_t* __restrict__ stats,
                                                            const uint32_t* __restrict__ nms,
                                                            const float* __restrict__ nms_score,
                                                            const uint8_t* __restrict__ supp, int w, int h, int r,
                                                            int nbx, int nby, int md, uint8_t* __restrict__ keep) {
    const int n = (int)stats[2];
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t step = (uint32_t)r + 1u, MD = (uint32_t)md;
    const uint32_t height = stats[1] > 0u ? stats[1] - 1u : 0u;
    for (int q = wave; q < n; q += nwaves) {
        const uint32_t g = clist[q];
        const uint32_t c = nms[g];
        const float cs = nms_score[g];
        const uint32_t cx = c & 0xFFFFu, cy = c >> 16;
        const uint32_t lo = MD > cy ? 0u : cy - MD;
        const uint32_t hi = cy + MD + 1u > height ? height : cy + MD + 1u;
        bool ok = !supp[g] && cx >= MD && cx < (uint32_t)w - MD && cy >= MD && cy < (uint32_t)h - MD;
        if (ok && hi > lo) {
            const int b0 = (int)(lo / step), b1 = min(nby - 1, (int)((hi - 1u) / step));
            const int c0 = (int)((cx >= MD ? cx - MD : 0u) / step), c1 = min(nbx - 1, (int)((cx + MD) / step));
            const int nbw = c1 - c0 + 1, ncell = (b1 - b0 + 1) * nbw;
            bool beaten = false;
            for (int k = lane; k < ncell; k += 64) {
                const int qq = k / nbw;
                const int gg = (b0 + qq) * nbx + c0 + (k - qq * nbw);
                const uint32_t e = nms[gg];
                if (e != kNone && (uint32_t)gg != g)
                    beaten |= beats(e >> 16, e & 0xFFFFu, nms_score[gg], cy, cx, cs, lo, hi, MD);
            }
            ok = __ballot(beaten) == 0ull;
        }
        if (lane == 0) keep[g] = ok ? 1 : 0;
    }
}

// Survivors of one NMS block row ranked in (y, x) order (sub-row y - by (r+1) first, then block
// column) -> staging[by][rank], row_count[by].
__global__ __launch_bounds__(1024) void ft_rank_kernel(const uint32_t* __restrict__ nms,
                                                       const uint8_t* __restrict__ keep, int r, int nbx,
                                                       uint32_t* __restrict__ staging, int* __restrict__ row_count) {
    __shared__ int scan[1024];
    const int by = blockIdx.x, bx = threadIdx.x;
    const uint32_t step = (uint32_t)r + 1u;
    const bool kp = bx < nbx && keep[by * nbx + bx];
    const uint32_t c = kp ? nms[by * nbx + bx] : kNone;
    const uint32_t sub = kp ? (c >> 16) - (uint32_t)by * step : 0u;
    int base = 0;
    for (uint32_t sr = 0; sr < step; ++sr) {
        const int f = kp && sub == sr ? 1 : 0;
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
        launch_boxblur_half(D.planes, D.tmp, D.w, D.h, r, (long)n, s);
        launch_boxblur_half(D.tmp, D.planes, D.h, D.w, r, (long)n, s);
    }
    hipLaunchKernelGGL(ft_score_kernel, dim3((n + 255) / 256), dim3(256), 0, s, D.planes, n, D.score);
    RSVIO_HIP(hipGetLastError());
}

void enqueue_select(const DetectBufs& D, float threshold, int min_dist, const float2* tracked_xy,
                    const uint8_t* tracked_valid, int n_tracked, hipStream_t s) {
    if (n_tracked > D.tpos_cap) throw std::invalid_argument("too many tracked features");
    if (D.nbx > 1024) throw std::invalid_argument("image too wide for the ranking workgroup");
    RSVIO_HIP(hipMemsetAsync(D.stats, 0, 4 * sizeof(uint32_t), s));
    const int total = D.nbx * D.nby + n_tracked;
    hipLaunchKernelGGL(ft_nms_kernel, dim3((total + 255) / 256), dim3(256), 0, s, D.score, D.w, D.h, D.r, threshold,
                       D.nbx, D.nby, D.nms, D.nms_score, D.stats, tracked_xy, tracked_valid, n_tracked, D.tpos,
                       D.supp, D.keep, D.clist);
    RSVIO_HIP(hipGetLastError());
    if (n_tracked > 0) {
        hipLaunchKernelGGL(ft_tracked_suppress_kernel, dim3((n_tracked + 3) / 4), dim3(256), 0, s, D.tpos, n_tracked,
                           D.nms, D.nms_score, D.stats, D.r, D.nbx, D.nby, min_dist, D.supp);
        RSVIO_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(ft_corner_max_kernel, dim3(512), dim3(256), 0, s, D.clist, D.stats, D.nms, D.nms_score, D.supp,
                       D.w, D.h, D.r, D.nbx, D.nby, min_dist, D.keep);
    RSVIO_HIP(hipGetLastError());
    const int threads = ((D.nbx + 63) / 64) * 64;
    hipLaunchKernelGGL(ft_rank_kernel, dim3(D.nby), dim3(threads), 0, s, D.nms, D.keep, D.r, D.nbx, D.staging,
                       D.row_count);
    RSVIO_HIP(hipGetLastError());
}

void enqueue_assemble(const Assemble& A, hipStream_t s) {
    hipLaunchKernelGGL(ft_assemble_kernel, dim3(1), dim3(1024), 0, s, A);
    RSVIO_HIP(hipGetLastError());
}

}  // namespace ft
}  // namespace rsvio
