// pyramid.hip -- K1: image pyramid (gfx950).
//
// Replaces build_image_pyramid (src/feature_tracker/feature_tracker.rs:209-220): level i is
// imageops::resize(full_res, W>>i, H>>i, Triangle) -- every level is resampled from the full
// resolution image, separable, vertical pass (f32) then horizontal pass (clamp, round to u8),
// image 0.25 semantics.  Bit-exact with the oracle: the tap weights and the sequential tap
// sums use the same f32 operations in the same order (-ffp-contract=off).
//
// One launch covers every level of every image: a workgroup owns a 64 x 8 output tile of
// one level; the vertical pass for the tile's rows over the tile's input-column span is
// staged in LDS (coalesced u8 reads along x), the horizontal pass reads it back.
#include "pyramid.hpp"

namespace rsvio {

namespace {

constexpr int TW = 64;               // widest output tile (level 1)
constexpr int TH = 8;                // tallest output tile (level 1)
constexpr int STRIP_COLS = 320;      // target input columns of a tile's source strip
constexpr size_t LDS_CAP = 64 << 10; // a level whose strip exceeds this reads its taps from HBM

__device__ __forceinline__ float triangle_kernel(float x) {
    float ax = fabsf(x);
    return ax < 1.0f ? 1.0f - ax : 0.0f;
}

// image 0.25 sample.rs: taps of one output index (same f32 ops as oracle make_taps)
__global__ void make_taps_kernel(TapTable tab, int n_entries) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_entries) return;
    int in_len = tab.ent_in_len[e];
    int out_len = tab.ent_out_len[e];
    int o = tab.ent_out_idx[e];
    float ratio = (float)in_len / (float)out_len;
    float sratio = ratio < 1.0f ? 1.0f : ratio;
    float support = 1.0f * sratio;
    float inputc = ((float)o + 0.5f) * ratio;
    long long left = (long long)floorf(inputc - support);
    if (left < 0) left = 0;
    if (left > (long long)in_len - 1) left = in_len - 1;
    long long right = (long long)ceilf(inputc + support);
    if (right < left + 1) right = left + 1;
    if (right > (long long)in_len) right = in_len;
    inputc = inputc - 0.5f;
    int cnt = (int)(right - left);
    float* w = tab.weights + (size_t)e * tab.max_taps;
    float sum = 0.0f;
    for (int k = 0; k < cnt; ++k) {
        float wv = triangle_kernel(((float)(left + k) - inputc) / sratio);
        w[k] = wv;
        sum += wv;
    }
    for (int k = 0; k < cnt; ++k) w[k] = w[k] / sum;
    tab.left[e] = (int)left;
    tab.count[e] = cnt;
}

__global__ __launch_bounds__(256) void pyramid_kernel(PyrLaunch L, PyrIO io) {
    extern __shared__ uint32_t smem[];
    const int img = blockIdx.y;
    {  // the FAST workgroups after the pyramid's (image 0 only)
        const int fb = (int)blockIdx.x - (L.copy_blocks + L.tile_start[L.levels]);
        if (fb >= 0) {
            if (img == 0 && fb < io.fast_cells) {
                const uint8_t* s0 = io.psrc ? io.psrc : io.src[0];
                fast_cell(s0, io.fg, fb, nullptr, nullptr, 0, io.fast_pt, io.fast_aff,
                          reinterpret_cast<uint8_t*>(smem));
            }
            return;
        }
    }
    const uint8_t* __restrict__ src = io.psrc ? io.psrc + (size_t)img * L.w * L.h : io.src[img];
    uint8_t* __restrict__ dst_base = io.psrc ? io.pdst + (size_t)img * L.pyr_bytes : io.dst[img];
    int b = blockIdx.x;
    const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst_base)) & 15) == 0;
    // level-0 copy blocks first (16 B per lane)
    if (b < L.copy_blocks) {
        const size_t tot = (size_t)L.w * L.h;
        if (!aligned) {
            for (size_t i = (size_t)b * blockDim.x + threadIdx.x; i < tot; i += (size_t)L.copy_blocks * blockDim.x)
                dst_base[i] = src[i];
            return;
        }
        const size_t n16 = tot / 16;
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst_base);
        for (size_t i = (size_t)b * blockDim.x + threadIdx.x; i < n16; i += (size_t)L.copy_blocks * blockDim.x)
            d4[i] = s4[i];
        size_t tail0 = n16 * 16;
        if (b == 0)
            for (size_t i = tail0 + threadIdx.x; i < tot; i += blockDim.x) dst_base[i] = src[i];
        return;
    }
    b -= L.copy_blocks;
    int lev = 1;
    while (lev < L.levels - 1 && b >= L.tile_start[lev + 1]) ++lev;
    b -= L.tile_start[lev];
    const int nw = (int)level_w(L.w, lev), nh = (int)level_h(L.h, lev);
    const int tw = L.tile_w[lev], th = L.tile_h[lev];
    const int tiles_x = (nw + tw - 1) / tw;
    const int tx = b % tiles_x, ty = b / tiles_x;
    const int ox0 = tx * tw, ox1 = min(ox0 + tw, nw);
    const int oy0 = ty * th, oy1 = min(oy0 + th, nh);
    const int rows = oy1 - oy0, cols_out = ox1 - ox0;
    const int hx = L.hx_ent[lev], vy = L.vy_ent[lev];
    const TapTable& T = L.tab;
    const int xl = T.left[hx + ox0];
    const int xr = T.left[hx + ox1 - 1] + T.count[hx + ox1 - 1];
    const int yl = T.left[vy + oy0];
    const int yr = T.left[vy + oy1 - 1] + T.count[vy + oy1 - 1];
    const int ncols = xr - xl, nrows = yr - yl;
    // 1. stage the source strip [yl, yr) x [xa, xr) in LDS: dword loads (every lane independent,
    //    one latency round) when rows are 4-byte aligned, else bytes.  Levels whose strip would
    //    not fit (ratio >= 64) read their taps from HBM instead (L.direct).
    const int xa = xl & ~3, xoff = xl - xa;
    const int pd = (xr - xa + 3) >> 2;  // dwords per strip row
    const bool direct = (L.direct >> lev) & 1;
    uint8_t* strip = reinterpret_cast<uint8_t*>(smem);
    if (!direct) {
        if (aligned && (L.w & 3) == 0) {
            // xr <= w and w % 4 == 0: the last dword of a row ends at or before the row's end
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
            const int wd = (int)(L.w >> 2);
            for (int idx = threadIdx.x; idx < nrows * pd; idx += blockDim.x) {
                const int r = idx / pd, d = idx - r * pd;
                smem[idx] = s32[(size_t)(yl + r) * wd + (xa >> 2) + d];
            }
        } else {
            for (int idx = threadIdx.x; idx < nrows * pd * 4; idx += blockDim.x) {
                const int r = idx / (pd * 4), c = idx - r * pd * 4;
                strip[idx] = (xa + c < (int)L.w) ? src[(size_t)(yl + r) * L.w + xa + c] : 0;
            }
        }
    }
    float* tmp = reinterpret_cast<float*>(smem + (direct ? 0 : nrows * pd));
    __syncthreads();
    // 2. vertical pass: tmp[r][c] = sum_k src[vleft + k][c] * vw[k], taps summed in order
    for (int idx = threadIdx.x; idx < rows * ncols; idx += blockDim.x) {
        const int r = idx / ncols, c = idx - r * ncols;
        const int e = vy + oy0 + r;
        const int vl = T.left[e], vc = T.count[e];
        const float* __restrict__ vw = T.weights + (size_t)e * T.max_taps;
        float acc = 0.0f;
        if (!direct) {
            const uint8_t* col = strip + (vl - yl) * pd * 4 + xoff + c;
            for (int k = 0; k < vc; ++k) acc += (float)col[k * pd * 4] * vw[k];
        } else {
            const uint8_t* __restrict__ col = src + (size_t)vl * L.w + xl + c;
            for (int k = 0; k < vc; k += 8) {
                float px[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) px[u] = (k + u < vc) ? (float)col[(size_t)(k + u) * L.w] : 0.0f;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (k + u < vc) acc += px[u] * vw[k + u];
            }
        }
        tmp[r * ncols + c] = acc;
    }
    __syncthreads();
    // 3. horizontal pass, clamp, round to u8
    uint8_t* __restrict__ dst = dst_base + level_offset(L.w, L.h, lev);
    for (int idx = threadIdx.x; idx < rows * cols_out; idx += blockDim.x) {
        const int r = idx / cols_out, c = idx - r * cols_out;
        const int e = hx + ox0 + c;
        const int hl = T.left[e] - xl, hc = T.count[e];
        const float* __restrict__ hw = T.weights + (size_t)e * T.max_taps;
        const float* __restrict__ row = tmp + r * ncols + hl;
        float acc = 0.0f;
        for (int k = 0; k < hc; ++k) acc += row[k] * hw[k];
        float cl = acc < 0.0f ? 0.0f : (acc > 255.0f ? 255.0f : acc);
        dst[(size_t)(oy0 + r) * nw + ox0 + c] = (uint8_t)roundf(cl);
    }
}

}  // namespace

void PyramidPlan::init(int w_, int h_, int levels_) {
    w = w_;
    h = h_;
    levels = levels_;
    if (levels < 1 || levels > kMaxLevels) throw std::invalid_argument("levels must be in [1, 8]");
    if (w < 16 || h < 16) throw std::invalid_argument("image too small");
    // entries: for each level >= 1: nw horizontal + nh vertical
    std::vector<int> in_len, out_len, out_idx;
    float max_ratio = 1.0f;
    memset(&launch, 0, sizeof(launch));
    for (int i = 1; i < levels; ++i) {
        int nw = (int)level_w(w, i), nh = (int)level_h(h, i);
        if (nw < 1 || nh < 1) throw std::invalid_argument("too many levels for image size");
        launch.hx_ent[i] = (int)in_len.size();
        for (int o = 0; o < nw; ++o) { in_len.push_back(w); out_len.push_back(nw); out_idx.push_back(o); }
        launch.vy_ent[i] = (int)in_len.size();
        for (int o = 0; o < nh; ++o) { in_len.push_back(h); out_len.push_back(nh); out_idx.push_back(o); }
        float rx = (float)w / nw, ry = (float)h / nh;
        max_ratio = std::max(max_ratio, std::max(rx, ry));
        // Equal work per tile across levels: deeper levels (more taps per output) get fewer
        // output rows and columns, so a level-5 tile is not 100x a level-1 tile.  A tile of tw
        // outputs spans at most tw * rx + 2 * rx + 3 input columns.
        launch.tile_h[i] = std::max(1, std::min(TH, (int)(16.0f / ry)));
        launch.tile_w[i] = std::max(1, std::min(TW, (int)std::floor((STRIP_COLS - 2.0f * rx - 4.0f) / rx)));
    }
    n_entries = (int)in_len.size();
    max_taps = (int)std::ceil(2.0f * max_ratio) + 4;
    int tiles = 0;
    for (int i = 1; i < levels; ++i) {
        launch.tile_start[i] = tiles;
        int nw = (int)level_w(w, i), nh = (int)level_h(h, i);
        tiles += ((nw + launch.tile_w[i] - 1) / launch.tile_w[i]) * ((nh + launch.tile_h[i] - 1) / launch.tile_h[i]);
    }
    launch.tile_start[levels] = tiles;
    launch.copy_blocks = std::max(1, (int)(((size_t)w * h / 16 + 255) / 256 / 4));
    total_blocks = launch.copy_blocks + tiles;
    launch.w = (uint32_t)w;
    launch.h = (uint32_t)h;
    launch.levels = levels;
    launch.pyr_bytes = level_offset(w, h, levels);
    if (n_entries > 0) {
        i_in.alloc(n_entries); i_out.alloc(n_entries); i_idx.alloc(n_entries);
        d_left.alloc(n_entries); d_count.alloc(n_entries);
        d_w.alloc((size_t)n_entries * max_taps);
        RSVIO_HIP(hipMemcpy(i_in.p, in_len.data(), sizeof(int) * n_entries, hipMemcpyHostToDevice));
        RSVIO_HIP(hipMemcpy(i_out.p, out_len.data(), sizeof(int) * n_entries, hipMemcpyHostToDevice));
        RSVIO_HIP(hipMemcpy(i_idx.p, out_idx.data(), sizeof(int) * n_entries, hipMemcpyHostToDevice));
        TapTable t;
        t.left = d_left.p; t.count = d_count.p; t.weights = d_w.p; t.max_taps = max_taps;
        t.ent_in_len = i_in.p; t.ent_out_len = i_out.p; t.ent_out_idx = i_idx.p;
        hipLaunchKernelGGL(make_taps_kernel, dim3((n_entries + 255) / 256), dim3(256), 0, 0, t, n_entries);
        RSVIO_HIP(hipGetLastError());
        RSVIO_HIP(hipDeviceSynchronize());
        launch.tab = t;
        // exact dynamic LDS: the largest (strip + vertical-pass) footprint over all tiles
        std::vector<int> left(n_entries), count(n_entries);
        RSVIO_HIP(hipMemcpy(left.data(), d_left.p, sizeof(int) * n_entries, hipMemcpyDeviceToHost));
        RSVIO_HIP(hipMemcpy(count.data(), d_count.p, sizeof(int) * n_entries, hipMemcpyDeviceToHost));
        for (int i = 1; i < levels; ++i) {
            const int nw = (int)level_w(w, i), nh = (int)level_h(h, i);
            const int tw = launch.tile_w[i], th = launch.tile_h[i];
            size_t strip = 0, vert = 0;
            for (int ox0 = 0; ox0 < nw; ox0 += tw) {
                const int ox1 = std::min(ox0 + tw, nw);
                const int xl = left[launch.hx_ent[i] + ox0];
                const int xr = left[launch.hx_ent[i] + ox1 - 1] + count[launch.hx_ent[i] + ox1 - 1];
                const size_t pd = (size_t)(xr - (xl & ~3) + 3) / 4;
                for (int oy0 = 0; oy0 < nh; oy0 += th) {
                    const int oy1 = std::min(oy0 + th, nh);
                    const int yl = left[launch.vy_ent[i] + oy0];
                    const int yr = left[launch.vy_ent[i] + oy1 - 1] + count[launch.vy_ent[i] + oy1 - 1];
                    strip = std::max(strip, 4 * pd * (size_t)(yr - yl));
                    vert = std::max(vert, 4 * (size_t)(oy1 - oy0) * (size_t)(xr - xl));
                }
            }
            if (vert > LDS_CAP) throw std::invalid_argument("image too wide for the pyramid tile");
            if (strip + vert > LDS_CAP) launch.direct |= 1u << i;
            lds_bytes = std::max(lds_bytes, ((launch.direct >> i) & 1) ? vert : strip + vert);
        }
    }
}

void PyramidPlan::enqueue(const PyrIO& io, int n_img, hipStream_t s) const {
    if (n_img <= 0) return;
    if (n_img > (io.psrc ? 65535 : kMaxPyrIO)) throw std::invalid_argument("too many images per pyramid launch");
    const size_t lds = io.fast_cells > 0 ? std::max(lds_bytes, (size_t)io.fg.g * io.fg.g) : lds_bytes;
    hipLaunchKernelGGL(pyramid_kernel, dim3(total_blocks + std::max(io.fast_cells, 0), n_img), dim3(256), lds, s,
                       launch, io);
    RSVIO_HIP(hipGetLastError());
}

void PyramidPlan::enqueue(const uint8_t* d_imgs, int n_img, uint8_t* d_pyrs, hipStream_t s) const {
    for (int i0 = 0; i0 < n_img; i0 += 65535) {
        PyrIO io{};
        io.psrc = d_imgs + (size_t)i0 * w * h;
        io.pdst = d_pyrs + (size_t)i0 * pyr_bytes();
        enqueue(io, std::min(65535, n_img - i0), s);
    }
}

}  // namespace rsvio
