// pyramid.hpp -- K1 image pyramid plan (see pyramid.hip).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "common.hpp"
#include "fast.hpp"

namespace rsvio {

constexpr int kMaxLevels = 8;

// Resampling taps (image::imageops Triangle) for every output row/column of every level.
struct TapTable {
    int* left = nullptr;
    int* count = nullptr;
    float* weights = nullptr;  // [entry][max_taps]
    int max_taps = 0;
    const int* ent_in_len = nullptr;
    const int* ent_out_len = nullptr;
    const int* ent_out_idx = nullptr;
};

struct PyrLaunch {
    uint32_t w, h;
    int levels;
    size_t pyr_bytes;
    int copy_blocks;
    int tile_start[kMaxLevels + 1];
    int tile_w[kMaxLevels];
    int tile_h[kMaxLevels];
    uint32_t direct;  // bit i: level i reads its vertical taps from HBM (strip exceeds LDS_CAP)
    int hx_ent[kMaxLevels];
    int vy_ent[kMaxLevels];
    TapTable tab;
};

constexpr int kMaxPyrIO = 8;
struct PyrIO {
    const uint8_t* src[kMaxPyrIO];
    uint8_t* dst[kMaxPyrIO];
    // packed mode (any number of images): image i at psrc + i * w * h, pyramid i at pdst + i * pyr_bytes
    const uint8_t* psrc;
    uint8_t* pdst;
    // optional: FAST-9 on every grid cell of image 0 (the tracker frame's detection, fast.hpp) as
    // fast_cells extra workgroups of the same launch -- it reads only the source image
    int fast_cells;
    GridGeom fg;
    int4* fast_pt;
    float* fast_aff;
};

struct PyramidPlan {
    int w = 0, h = 0, levels = 0;
    int n_entries = 0, max_taps = 0, total_blocks = 0;
    size_t lds_bytes = 0;  // dynamic LDS of pyramid_kernel: source strip (u8) + vertical pass (f32)
    PyrLaunch launch;
    DevBuf<int> i_in, i_out, i_idx, d_left, d_count;
    DevBuf<float> d_w;
    void init(int w, int h, int levels);
    size_t pyr_bytes() const { return level_offset(w, h, levels); }
    // n_img packed w*h images -> n_img packed pyramids
    void enqueue(const uint8_t* d_imgs, int n_img, uint8_t* d_pyrs, hipStream_t s) const;
    void enqueue(const PyrIO& io, int n_img, hipStream_t s) const;
};

}  // namespace rsvio
