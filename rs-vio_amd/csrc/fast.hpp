// fast.hpp -- detect_key_points on the grid (src/feature_tracker/image_utilities.rs:108-175):
// the grid geometry and the per-cell FAST-9 threshold ladder, shared by the tracker's frame (run
// inside the pyramid launch, pyramid.hip) and the rsvio_detect_keypoints parity entry point.
#pragma once
#include "common.hpp"

namespace rsvio {

constexpr int kEdge = 19;  // EDGE_THRESHOLD, image_utilities.rs:114

struct GridGeom {
    int w, h, g;
    int xs, ys, xe, ye;   // x_start, y_start, x_stop, y_stop (image_utilities.rs:121-125)
    int bin_rows, bin_cols;  // (h / g + 1) x (w / g + 1) counters
    int cells_x, cells_y;    // cells actually scanned
};

inline GridGeom make_grid(int w, int h, int g) {
    GridGeom G;
    G.w = w; G.h = h; G.g = g;
    G.xs = (w % g) / 2;
    G.xe = G.xs + g * (w / g - 1) + 1;
    G.ys = (h % g) / 2;
    G.ye = G.ys + g * (h / g - 1) + 1;
    G.bin_rows = h / g + 1;
    G.bin_cols = w / g + 1;
    G.cells_x = (G.xe - G.xs + g - 1) / g;
    G.cells_y = (G.ye - G.ys + g - 1) / g;
    return G;
}

// FAST-9 score of a candidate (largest t with a contiguous 9-arc all brighter than c + t or all
// darker than c - t); equals imageproc's binary-searched fast_corner_score whenever the pixel is
// a corner at the starting threshold.
__device__ __forceinline__ int fast9_score(const uint8_t* crop, int g, int x, int y) {
    const int8_t ox[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    const int8_t oy[16] = {-3, -3, -2, -1, 0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3};
    const int c = crop[y * g + x];
    int d[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = (int)crop[(y + oy[i]) * g + x + ox[i]] - c;
    int sb = -1000, sd = -1000;
#pragma unroll
    for (int a = 0; a < 16; ++a) {
        int mb = 1000, md = 1000;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            int v = d[(a + k) & 15];
            mb = min(mb, v);
            md = min(md, -v);
        }
        sb = max(sb, mb);
        sd = max(sd, md);
    }
    return max(sb, sd) - 1;
}

// detect_key_points per cell (image_utilities.rs:141-172): skip occupied cells; otherwise
// thresholds 40, 35, ..., 10 on the cell's grid x grid crop; keep the lowest-score corner
// (ties: crop scan order) that lies in [19, w-19] x [19, h-19].  Occupancy: the cell holds one
// of the n_pts existing points (pts_valid[i] != 0, or all when null) binned by
// image_utilities.rs:128-139 with feature_tracker.rs:228-237's rounding -- every workgroup
// tests the points itself, so no grid-wide binning pass precedes it.  new_aff (optional): the
// identity Affine2 at the cell's corner (feature_tracker.rs:143-152), indexed by cell.
// Cell s (scan order: x outer, y inner) by one 256-thread workgroup; crop: grid^2 bytes of LDS.
__device__ inline void fast_cell(const uint8_t* __restrict__ img, const GridGeom& G, int s,
                                 const float* __restrict__ pts_aff, const uint8_t* __restrict__ pts_valid, int n_pts,
                                 int4* __restrict__ cell_pt, float* __restrict__ new_aff, uint8_t* crop) {
    __shared__ int s_max, s_key;
    const int cx = s / G.cells_y, cy = s % G.cells_y;
    const int x0 = G.xs + cx * G.g, y0 = G.ys + cy * G.g;
    int occ = 0;
    for (int i = threadIdx.x; i < n_pts; i += blockDim.x) {
        if (pts_valid != nullptr && !pts_valid[i]) continue;
        const uint32_t x = sat_u32(roundf(pts_aff[6 * i + 4]));
        const uint32_t y = sat_u32(roundf(pts_aff[6 * i + 5]));
        if (x >= (uint32_t)G.xs && y >= (uint32_t)G.ys && x < (uint32_t)(G.xe + G.g) && y < (uint32_t)(G.ye + G.g) &&
            (int)((x - G.xs) / G.g) == cx && (int)((y - G.ys) / G.g) == cy)
            occ = 1;
    }
    if (__syncthreads_or(occ)) {
        if (threadIdx.x == 0) cell_pt[s] = make_int4(0, 0, 0, 0);
        return;
    }
    const int g = G.g;
    for (int i = threadIdx.x; i < g * g; i += blockDim.x) crop[i] = img[(size_t)(y0 + i / g) * G.w + x0 + i % g];
    if (threadIdx.x == 0) {
        s_max = -1;
        s_key = 0x7FFFFFFF;
    }
    __syncthreads();
    const int span = g - 6;  // crop-local candidates [3, g - 3)
    int my_best = -1;
    for (int i = threadIdx.x; i < span * span; i += blockDim.x) {
        const int x = 3 + i % span, y = 3 + i / span;
        const int X = x0 + x, Y = y0 + y;
        if (X < kEdge || X > G.w - kEdge || Y < kEdge || Y > G.h - kEdge) continue;
        int sc = fast9_score(crop, g, x, y);
        if (sc >= 10) my_best = max(my_best, sc);
    }
    if (my_best >= 0) atomicMax(&s_max, my_best);
    __syncthreads();
    const int smax = s_max;
    int tstar = -1;
    for (int t = 40; t >= 10; t -= 5)
        if (smax >= t) {
            tstar = t;
            break;
        }
    if (tstar < 0) {
        if (threadIdx.x == 0) cell_pt[s] = make_int4(0, 0, 0, 0);
        return;
    }
    int my_key = 0x7FFFFFFF;
    for (int i = threadIdx.x; i < span * span; i += blockDim.x) {
        const int x = 3 + i % span, y = 3 + i / span;
        const int X = x0 + x, Y = y0 + y;
        if (X < kEdge || X > G.w - kEdge || Y < kEdge || Y > G.h - kEdge) continue;
        int sc = fast9_score(crop, g, x, y);
        if (sc >= tstar) my_key = min(my_key, (sc << 16) | (y * g + x));
    }
    atomicMin(&s_key, my_key);
    __syncthreads();
    if (threadIdx.x == 0) {
        const int key = s_key;
        const int idx = key & 0xFFFF;
        const int px = x0 + idx % g, py = y0 + idx / g;
        cell_pt[s] = make_int4(px, py, key >> 16, 1);
        if (new_aff != nullptr) {
            float* a = new_aff + 6 * s;
            a[0] = 1.0f; a[1] = 0.0f; a[2] = 0.0f; a[3] = 1.0f;
            a[4] = (float)px;
            a[5] = (float)py;
        }
    }
}

}  // namespace rsvio
