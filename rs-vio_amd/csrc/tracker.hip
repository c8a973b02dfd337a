// tracker.hip -- device-resident StereoPatchTracker and the HP-T C ABI.
//
// Replaces StereoPatchTracker::{new, process_frame, get_track_points, remove_id}
// (src/feature_tracker/feature_tracker.rs:91-207), add_points (:222-251) and
// detect_key_points (src/feature_tracker/image_utilities.rs:108-175).
//
// Per stereo frame, all on one HIP stream, nothing leaves HBM except the final feature list:
//   K1 pyramid (both images, all levels, one launch)            pyramid.hip
//   K3 FAST-9 threshold ladder, one workgroup per grid cell, EVERY cell (integer, exact), as
//      extra workgroups of the K1 launch (it reads the left image itself)
//   K2 ONE launch: temporal track cam0 + cam1, and the stereo track cam0 -> cam1 of every
//      cell's corner (one job per cell, cells without a corner masked)   lk_track.hip
//   Ka compact the survivors, bin them, append the corners of the cells holding no surviving
//      cam0 track in cell scan order with consecutive ids, pack (+ unprojection) (1 workgroup)
// The reference detects only in the cells its surviving tracks leave empty and then tracks those
// corners; a cell's corner and its stereo track depend on nothing but the cell and the images,
// so detecting and tracking every cell up front and dropping the occupied ones afterwards gives
// the same points and tracks -- and lets the stereo jobs join the temporal launch (one LK
// latency per frame instead of two).
// Canonical order: track maps are kept sorted by id; new ids are assigned in detection scan
// order (the reference's HashMap iteration order is random, feature_tracker.rs:162-170).
#include <cmath>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "lk_track.hpp"
#include "pyramid.hpp"
#include "camera.hpp"
#include "fast.hpp"

namespace rsvio {

namespace {

thread_local std::string g_last_error;

// Block-wide exclusive scan of one int per thread (blockDim.x a multiple of 64, <= 1024): an
// inclusive scan within each wave (6 shuffle steps, no barrier), the wave totals scanned by
// wave 0 through LDS -- two barriers instead of two per doubling step.
__device__ int block_exclusive_scan(int v, int* sh, int* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
    }
    if (lane == 63) sh[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        int w = lane < nw ? sh[lane] : 0;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const int t = __shfl_up(w, off, 64);
            if (lane >= off) w += t;
        }
        if (lane < nw) sh[16 + lane] = w;  // inclusive prefix of wave totals
    }
    __syncthreads();
    *total = sh[16 + nw - 1];
    const int base = wave > 0 ? sh[16 + wave - 1] : 0;
    __syncthreads();  // sh is reused by the next scan
    return base + incl - v;
}

// detect_key_points per cell (fast.hpp): one 256-thread workgroup per cell, crop in dynamic LDS
__global__ __launch_bounds__(256) void fast_cells_kernel(const uint8_t* __restrict__ img, GridGeom G,
                                                         const float* __restrict__ pts_aff,
                                                         const uint8_t* __restrict__ pts_valid, int n_pts,
                                                         int4* __restrict__ cell_pt, float* __restrict__ new_aff) {
    extern __shared__ uint8_t crop[];
    fast_cell(img, G, (int)blockIdx.x, pts_aff, pts_valid, n_pts, cell_pt, new_aff, crop);
}

// New corners in scan order -> identity Affine2 at the corner (feature_tracker.rs:143-152)
__global__ __launch_bounds__(1024) void gather_new_kernel(const int4* __restrict__ cell_pt, int n_cells,
                                                          float* __restrict__ new_aff, int* __restrict__ new_count,
                                                          float* __restrict__ new_score) {
    __shared__ int sh[1024];
    const int per = (n_cells + blockDim.x - 1) / blockDim.x;
    const int b = threadIdx.x * per, e = min(n_cells, b + per);
    int local = 0;
    for (int i = b; i < e; ++i) local += cell_pt[i].w;
    int total;
    int pos = block_exclusive_scan(local, sh, &total);
    for (int i = b; i < e; ++i) {
        int4 c = cell_pt[i];
        if (!c.w) continue;
        float* a = new_aff + 6 * pos;
        a[0] = 1.0f; a[1] = 0.0f; a[2] = 0.0f; a[3] = 1.0f;
        a[4] = (float)c.x;
        a[5] = (float)c.y;
        if (new_score) new_score[pos] = (float)c.z;
        ++pos;
    }
    if (threadIdx.x == 0) *new_count = total;
}

struct CamPair {
    rsvio_camera cam[2];
    int on;
};

// The end of process_frame in one workgroup: (1) the surviving temporal tracks of each camera
// compacted in order from the tracker's output (at, valid) into the track map (feature_tracker.rs
// :131-141 -- failed tracks are dropped, the map keeps ascending ids); (2) the corners of the
// cells holding no cam0 survivor whose stereo track succeeded (cell_pt[i].w && new_valid[i])
// appended in cell scan order with consecutive ids (feature_tracker.rs:143-170, canonical order); (3) get_track_points packing, with the
// Frame::add_{left,right}_feature unprojection fused (frame.rs:118-119,131-132).  tracked = 0
// (first frame): the maps are taken as they are (counts = n0, n1).
__global__ __launch_bounds__(1024) void append_pack_kernel(
    GridGeom G, int* __restrict__ bins, int n0, int n1, int tracked, const float* __restrict__ at0, const float* __restrict__ at1,
    const uint8_t* __restrict__ tv0, const uint8_t* __restrict__ tv1, uint64_t* __restrict__ ids_tmp,
    const int4* __restrict__ cell_pt, int n_cells, const float* __restrict__ new_aff0,
    const float* __restrict__ new_aff1, const uint8_t* __restrict__ new_valid, float* __restrict__ map_aff0,
    float* __restrict__ map_aff1, uint64_t* __restrict__ ids0, uint64_t* __restrict__ ids1,
    int* __restrict__ counts, unsigned long long* __restrict__ last_id, int capacity,
    rsvio_feature* __restrict__ out0, rsvio_feature* __restrict__ out1, int* __restrict__ overflow,
    CamPair cams, float2* __restrict__ und0, float2* __restrict__ und1) {
    __shared__ int sh[1024];
    const int tid = threadIdx.x;
    int cnt[2] = {n0, n1};
    if (tracked) {
        for (int c = 0; c < 2; ++c) {
            const int n = c == 0 ? n0 : n1;
            const float* at = c == 0 ? at0 : at1;
            const uint8_t* vv = c == 0 ? tv0 : tv1;
            float* ma = c == 0 ? map_aff0 : map_aff1;
            uint64_t* ids = c == 0 ? ids0 : ids1;
            uint64_t* it = ids_tmp + (size_t)c * capacity;
            const int per = (n + blockDim.x - 1) / blockDim.x;
            const int b = tid * per, e = min(n, b + per);
            int local = 0;
            for (int i = b; i < e; ++i) {
                local += vv[i] ? 1 : 0;
                it[i] = ids[i];  // ids are compacted in place: through a copy
            }
            int total;
            int pos = block_exclusive_scan(local, sh, &total);  // its barriers order the copy
            for (int i = b; i < e; ++i) {
                if (!vv[i]) continue;
                for (int k = 0; k < 6; ++k) ma[6 * pos + k] = at[6 * i + k];
                ids[pos] = it[i];
                ++pos;
            }
            cnt[c] = total;
        }
    }
    // bin the cam0 survivors into the grid counters (image_utilities.rs:128-139 with
    // feature_tracker.rs:228-237's rounding); a cell with a count keeps no new corner
    for (int i = tid; i < G.bin_rows * G.bin_cols; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    for (int i = tid; i < cnt[0]; i += blockDim.x) {
        const uint32_t x = sat_u32(roundf(map_aff0[6 * i + 4]));
        const uint32_t y = sat_u32(roundf(map_aff0[6 * i + 5]));
        if (x >= (uint32_t)G.xs && y >= (uint32_t)G.ys && x < (uint32_t)(G.xe + G.g) && y < (uint32_t)(G.ye + G.g))
            atomicAdd(&bins[((y - G.ys) / G.g) * G.bin_cols + (x - G.xs) / G.g], 1);
    }
    __syncthreads();
    auto is_new = [&](int i) {  // cell i (scan order: x outer, y inner) contributes a new point
        const int cx = i / G.cells_y, cy = i % G.cells_y;
        return cell_pt[i].w != 0 && new_valid[i] != 0 && bins[cy * G.bin_cols + cx] == 0;
    };
    const int per = (n_cells + blockDim.x - 1) / blockDim.x;
    const int b = tid * per, e = min(n_cells, b + per);
    int local = 0;
    for (int i = b; i < e; ++i) local += is_new(i) ? 1 : 0;
    int total;
    int pos = block_exclusive_scan(local, sh, &total);
    const int c0 = cnt[0], c1 = cnt[1];
    const unsigned long long base = *last_id;
    // Both cameras append the same new points (feature_tracker.rs:162-170), so admit only as many as
    // the fuller camera has room for: no slot beyond what was written is ever counted, and ids stay
    // consecutive.  A frame with more new points than room raises the overflow flag (reported by
    // fetch() as RSVIO_ERR_CAPACITY); the flag is rewritten every frame.
    const int admit = min(total, max(0, min(capacity - c0, capacity - c1)));
    for (int i = b; i < e; ++i) {
        if (!is_new(i)) continue;
        if (pos < admit) {
            const int d0 = c0 + pos, d1 = c1 + pos;
            for (int k = 0; k < 6; ++k) {
                map_aff0[6 * d0 + k] = new_aff0[6 * i + k];
                map_aff1[6 * d1 + k] = new_aff1[6 * i + k];
            }
            ids0[d0] = base + pos;
            ids1[d1] = base + pos;
        }
        ++pos;
    }
    __syncthreads();
    const int m0 = c0 + admit, m1 = c1 + admit;
    if (tid == 0) {
        counts[0] = m0;
        counts[1] = m1;
        *last_id = base + (unsigned long long)admit;
        *overflow = total > admit ? 1 : 0;
    }
    // get_track_points packing, both cameras spread over the block
    for (int j = tid; j < m0 + m1; j += blockDim.x) {
        const int c = j < m0 ? 0 : 1;
        const int i = c == 0 ? j : j - m0;
        const float* a = (c == 0 ? map_aff0 : map_aff1) + 6 * i;
        rsvio_feature f;
        f.id = (c == 0 ? ids0 : ids1)[i]; f.x = a[4]; f.y = a[5];
        f.r[0] = a[0]; f.r[1] = a[1]; f.r[2] = a[2]; f.r[3] = a[3];
        (c == 0 ? out0 : out1)[i] = f;
        if (cams.on) {
            const Undist u = unproject_one(cams.cam[c], f.x, f.y);
            (c == 0 ? und0 : und1)[i] = make_float2(u.x, u.y);
        }
    }
}

// StereoPatchTracker::remove_id (feature_tracker.rs:201-206)
__global__ __launch_bounds__(1024) void remove_ids_kernel(const uint64_t* __restrict__ rm, int n_rm,
                                                          float* __restrict__ map_aff0, float* __restrict__ map_aff1,
                                                          uint64_t* __restrict__ ids0, uint64_t* __restrict__ ids1,
                                                          float* __restrict__ tmp_aff, uint64_t* __restrict__ tmp_ids,
                                                          int* __restrict__ counts, rsvio_feature* out0,
                                                          rsvio_feature* out1, float2* und0, float2* und1,
                                                          float2* __restrict__ tmp_und) {
    __shared__ int sh[1024];
    for (int c = 0; c < 2; ++c) {
        float* ma = c == 0 ? map_aff0 : map_aff1;
        uint64_t* ids = c == 0 ? ids0 : ids1;
        rsvio_feature* out = c == 0 ? out0 : out1;
        float2* und = c == 0 ? und0 : und1;  // the fused unprojection's output, compacted alike
        const int n = counts[c];
        const int per = (n + blockDim.x - 1) / blockDim.x;
        const int b = threadIdx.x * per, e = min(n, b + per);
        int local = 0;
        for (int i = b; i < e; ++i) {
            bool drop = false;
            for (int k = 0; k < n_rm; ++k) drop |= (rm[k] == ids[i]);
            local += drop ? 0 : 1;
            tmp_ids[i] = drop ? ~0ull : ids[i];
            for (int k = 0; k < 6; ++k) tmp_aff[6 * i + k] = ma[6 * i + k];
            if (und) tmp_und[i] = und[i];
        }
        int total;
        int pos = block_exclusive_scan(local, sh, &total);
        for (int i = b; i < e; ++i) {
            if (tmp_ids[i] == ~0ull) continue;
            for (int k = 0; k < 6; ++k) ma[6 * pos + k] = tmp_aff[6 * i + k];
            ids[pos] = tmp_ids[i];
            if (und) und[pos] = tmp_und[i];
            ++pos;
        }
        __syncthreads();
        if (threadIdx.x == 0) counts[c] = total;
        for (int i = threadIdx.x; i < total; i += blockDim.x) {
            const float* a = ma + 6 * i;
            rsvio_feature f;
            f.id = ids[i]; f.x = a[4]; f.y = a[5]; f.r[0] = a[0]; f.r[1] = a[1]; f.r[2] = a[2]; f.r[3] = a[3];
            out[i] = f;
        }
        __syncthreads();
    }
}

}  // namespace

void set_last_error(const std::string& msg) { g_last_error = msg; }

// ------------------------------------------------------------------------------------------
struct Tracker {
    rsvio_tracker_params P;
    GridGeom G;
    PyramidPlan plan;
    hipStream_t stream = nullptr;
    size_t pyr_bytes = 0;
    int cap = 0;
    int n_cells = 0;
    int cur = 0;            // pyramid ping-pong index
    bool has_prev = false;
    int host_count[2] = {0, 0};
    DevBuf<uint8_t> d_img, d_pyr;   // 2 images; 2 slots x 2 cams pyramids
    DevBuf<float> map_aff, tmp_aff, new_aff, new_aff1;
    DevBuf<uint64_t> ids, ids_tmp, rm_ids;
    DevBuf<uint8_t> valid, new_valid;
    DevBuf<int> counts, bins, overflow;
    DevBuf<int4> cell_pt;
    DevBuf<unsigned long long> last_id;
    // packed output lists, TWO frame slots (2 x 2 cams x cap): frame t writes slot t & 1, so a
    // consumer of the last collected frame (track_motion_tracker, remove_ids, undistorted) reads
    // a slot that the next frame -- submitted before that consumer runs, in the Estimator's
    // one-frame look-ahead -- does not write
    DevBuf<rsvio_feature> out;
    HostBuf<int> h_counts;
    CamPair cams{};                 // T12 unprojection fused into append_pack_kernel when on
    DevBuf<float2> undist;          // 2 slots x 2 x cap
    DevBuf<float2> tmp_und;         // cap (remove_ids compaction scratch)
    HostBuf<float2> h_undist;       // pinned read-back of the undistorted coordinates, one per output
                                    // slot (2 slots x 2 cams x cap): a submit's copies land in its own
                                    // slot, undistorted() reads the collected one
    HostBuf<rsvio_feature> h_out;   // pinned staging of both packed feature lists (2 x cap)
    size_t last_n[2] = {0, 0};
    int wslot = 0;                  // the output slot the next submitted frame writes
    int rslot = 0;                  // the output slot of the last collected frame
    int coll_n[2] = {0, 0};         // its device list lengths (<= cap)
    bool inflight = false;          // a frame was submitted and not yet collected
    size_t bnd[2] = {0, 0};         // the list bounds the submit's copies covered
    hipEvent_t ev_done = nullptr;   // after the submitted frame's read-back copies

    uint8_t* pyr(int slot, int cam) { return d_pyr.p + (size_t)(2 * slot + cam) * pyr_bytes; }

    void init(const rsvio_tracker_params& p) {
        P = p;
        if (P.width < 32 || P.height < 32 || P.levels < 1 || P.levels > kMaxLevels || P.grid_size < 8 ||
            P.grid_size > 128 || P.max_iterations < 0)
            throw std::invalid_argument("invalid tracker parameters");
        if (P.grid_size > P.width || P.grid_size > P.height) throw std::invalid_argument("grid larger than image");
        cap = P.max_features > 0 ? P.max_features : 4096;
        RSVIO_HIP(hipSetDevice(P.device));
        RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        plan.init(P.width, P.height, P.levels);
        pyr_bytes = plan.pyr_bytes();
        G = make_grid(P.width, P.height, P.grid_size);
        n_cells = G.cells_x * G.cells_y;
        const size_t img = (size_t)P.width * P.height;
        d_img.alloc(2 * img);
        d_pyr.alloc(4 * pyr_bytes);
        map_aff.alloc((size_t)2 * cap * 6);
        tmp_aff.alloc((size_t)2 * cap * 6);
        ids.alloc((size_t)2 * cap);
        ids_tmp.alloc((size_t)2 * cap);
        valid.alloc((size_t)2 * cap);
        new_aff.alloc((size_t)n_cells * 6);
        new_aff1.alloc((size_t)n_cells * 6);
        new_valid.alloc(n_cells);
        counts.alloc(2);
        bins.alloc((size_t)G.bin_rows * G.bin_cols);
        overflow.alloc(1);
        cell_pt.alloc(n_cells);
        last_id.alloc(1);
        out.alloc((size_t)4 * cap);
        h_counts.alloc(4);
        RSVIO_HIP(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
        h_out.alloc((size_t)2 * cap);
        RSVIO_HIP(hipMemsetAsync(counts.p, 0, sizeof(int) * 2, stream));
        RSVIO_HIP(hipMemsetAsync(last_id.p, 0, sizeof(unsigned long long), stream));
        RSVIO_HIP(hipMemsetAsync(overflow.p, 0, sizeof(int), stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
    }
    ~Tracker() {
        if (stream) (void)hipStreamSynchronize(stream);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (stream) (void)hipStreamDestroy(stream);
    }

    float* maff(int c) { return map_aff.p + (size_t)c * cap * 6; }
    float* taff(int c) { return tmp_aff.p + (size_t)c * cap * 6; }
    uint64_t* mid(int c) { return ids.p + (size_t)c * cap; }
    rsvio_feature* outp(int slot, int c) { return out.p + (size_t)(2 * slot + c) * cap; }
    float2* undp(int slot, int c) { return cams.on ? undist.p + (size_t)(2 * slot + c) * cap : nullptr; }
    float2* hund(int slot, int c) { return h_undist.p + (size_t)(2 * slot + c) * cap; }

    // Enqueue one frame; images already in device memory.
    void enqueue_frame(const uint8_t* d_left, const uint8_t* d_right) {
        const int nxt = has_prev ? 1 - cur : cur;
        // K1 + K3: both pyramids and FAST-9 in every cell of the left image (its corner as a
        // cell-indexed identity affine) in one launch
        PyrIO io{};
        io.src[0] = d_left; io.dst[0] = pyr(nxt, 0);
        io.src[1] = d_right; io.dst[1] = pyr(nxt, 1);
        io.fast_cells = n_cells; io.fg = G; io.fast_pt = cell_pt.p; io.fast_aff = new_aff.p;
        plan.enqueue(io, 2, stream);
        {  // one LK launch: [cam0 temporal, cam1 temporal,] stereo of every cell's corner
            TrackLaunch L{};
            L.w = P.width; L.h = P.height; L.levels = P.levels; L.max_iter = P.max_iterations;
            L.thresh = P.convergence_threshold;
            int b = 0;
            L.start[0] = 0;
            if (has_prev) {
                for (int c = 0; c < 2; ++c, ++b) {
                    L.pyr0[b] = pyr(cur, c); L.pyr1[b] = pyr(nxt, c);
                    L.ain[b] = maff(c); L.aout[b] = taff(c); L.valid[b] = valid.p + (size_t)c * cap;
                    L.start[b + 1] = L.start[b] + host_count[c];
                }
            }
            L.pyr0[b] = pyr(nxt, 0); L.pyr1[b] = pyr(nxt, 1);
            L.ain[b] = new_aff.p; L.aout[b] = new_aff1.p; L.valid[b] = new_valid.p;
            L.mask[b] = cell_pt.p;  // cells without a corner exit at once
            L.start[b + 1] = L.start[b] + n_cells;
            L.nb = b + 1;
            enqueue_track(L, stream);
        }
        hipLaunchKernelGGL(append_pack_kernel, dim3(1), dim3(1024), 0, stream, G, bins.p, host_count[0],
                           host_count[1], has_prev ? 1 : 0, taff(0), taff(1), valid.p, valid.p + cap, ids_tmp.p,
                           cell_pt.p, n_cells, new_aff.p, new_aff1.p, new_valid.p, maff(0), maff(1), mid(0), mid(1),
                           counts.p, last_id.p, cap, outp(wslot, 0), outp(wslot, 1), overflow.p, cams,
                           undp(wslot, 0), undp(wslot, 1));
        RSVIO_HIP(hipGetLastError());
        cur = nxt;
        has_prev = true;
    }

    // Counts, overflow flag and both feature lists (+ undistorted coordinates) in ONE round trip:
    // the lists are copied up to a host-known bound into pinned staging -- a camera's list is its
    // previous survivors plus at most one new point per grid cell (feature_tracker.rs:143-170) --
    // and a second copy covers any excess (never expected).
    void copy_lists(int slot, size_t l0, size_t l1, size_t r0, size_t r1) {
        if (l1 > l0) RSVIO_HIP(hipMemcpyAsync(h_out.p + l0, outp(slot, 0) + l0, (l1 - l0) * sizeof(rsvio_feature),
                                              hipMemcpyDeviceToHost, stream));
        if (r1 > r0) RSVIO_HIP(hipMemcpyAsync(h_out.p + cap + r0, outp(slot, 1) + r0, (r1 - r0) * sizeof(rsvio_feature),
                                              hipMemcpyDeviceToHost, stream));
        if (cams.on) {
            if (l1 > l0) RSVIO_HIP(hipMemcpyAsync(hund(slot, 0) + l0, undp(slot, 0) + l0, (l1 - l0) * sizeof(float2),
                                                  hipMemcpyDeviceToHost, stream));
            if (r1 > r0) RSVIO_HIP(hipMemcpyAsync(hund(slot, 1) + r0, undp(slot, 1) + r0,
                                                  (r1 - r0) * sizeof(float2), hipMemcpyDeviceToHost, stream));
        }
    }

    // submit: the frame's kernels, then the read-back of counts, overflow flag and both lists
    // (+ undistorted coordinates) up to a host-known bound, all on the stream; returns at once.
    void submit(const uint8_t* d_left, const uint8_t* d_right) {
        enqueue_frame(d_left, d_right);
        bnd[0] = std::min((size_t)cap, (size_t)host_count[0] + (size_t)n_cells);
        bnd[1] = std::min((size_t)cap, (size_t)host_count[1] + (size_t)n_cells);
        RSVIO_HIP(hipMemcpyAsync(h_counts.p, counts.p, sizeof(int) * 2, hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipMemcpyAsync(h_counts.p + 2, overflow.p, sizeof(int), hipMemcpyDeviceToHost, stream));
        copy_lists(wslot, 0, bnd[0], 0, bnd[1]);
        RSVIO_HIP(hipEventRecord(ev_done, stream));
        inflight = true;
    }

    void require_collected(const char* what) {
        if (inflight) throw CallOrderError(std::string(what) + ": a frame is in flight (collect it first)");
    }

    // collect: wait for the submitted frame's read-back, then the host lists
    int fetch(rsvio_feature* out_l, size_t cap_l, size_t* n_l, rsvio_feature* out_r, size_t cap_r, size_t* n_r) {
        if (!inflight) throw CallOrderError("no frame in flight (submit one first)");
        inflight = false;
        const int slot = wslot;
        wslot ^= 1;
        rslot = slot;
        RSVIO_HIP(hipEventSynchronize(ev_done));
        const size_t bl = bnd[0], br = bnd[1];
        host_count[0] = h_counts.p[0];
        host_count[1] = h_counts.p[1];
        const size_t ml = std::min((size_t)host_count[0], (size_t)cap), mr = std::min((size_t)host_count[1], (size_t)cap);
        coll_n[0] = (int)ml;
        coll_n[1] = (int)mr;
        if (ml > bl || mr > br) {
            copy_lists(slot, bl, std::max(ml, bl), br, std::max(mr, br));
            RSVIO_HIP(hipStreamSynchronize(stream));
        }
        const size_t nl = std::min(ml, cap_l), nr = std::min(mr, cap_r);
        if (nl) std::memcpy(out_l, h_out.p, nl * sizeof(rsvio_feature));
        if (nr) std::memcpy(out_r, h_out.p + cap, nr * sizeof(rsvio_feature));
        last_n[0] = cams.on ? nl : 0;
        last_n[1] = cams.on ? nr : 0;
        *n_l = nl;
        *n_r = nr;
        if (h_counts.p[2]) {
            set_last_error("StereoPatchTracker: new points exceed max_features; the excess was dropped");
            return RSVIO_ERR_CAPACITY;
        }
        if (nl < ml || nr < mr) {
            set_last_error("StereoPatchTracker: feature list exceeds the output capacity (truncated)");
            return RSVIO_ERR_CAPACITY;
        }
        return RSVIO_OK;
    }
};

// Parity-level context: taps + scratch for the stateless entry points
struct TrackCtx {
    PyramidPlan plan;
    int device = 0;
};

}  // namespace rsvio

struct rsvio_tracker {
    rsvio::Tracker t;
};
struct rsvio_track_ctx {
    rsvio::TrackCtx c;
};

namespace rsvio {
TrackerView tracker_view(rsvio_tracker* h) {
    Tracker& T = h->t;
    TrackerView v{};
    v.stream = T.stream;
    // the last COLLECTED frame's slot and lengths: a frame submitted since writes the other slot
    v.out[0] = T.outp(T.rslot, 0);
    v.out[1] = T.outp(T.rslot, 1);
    v.undist[0] = T.undp(T.rslot, 0);
    v.undist[1] = T.undp(T.rslot, 1);
    v.n[0] = T.coll_n[0];
    v.n[1] = T.coll_n[1];
    v.device = T.P.device;
    return v;
}
}  // namespace rsvio

using rsvio::guarded;

extern "C" {

const char* rsvio_last_error(void) { return rsvio::g_last_error.c_str(); }

int rsvio_device_info(int device, char* name_out, size_t cap, int* n_cus) {
    return guarded([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
            rsvio::set_last_error("no HIP device visible");
            return (int)RSVIO_ERR_NO_DEVICE;
        }
        hipDeviceProp_t prop;
        RSVIO_HIP(hipGetDeviceProperties(&prop, device));
        if (name_out && cap) snprintf(name_out, cap, "%s", prop.gcnArchName);
        if (n_cus) *n_cus = prop.multiProcessorCount;
        if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
            rsvio::set_last_error(std::string("device is ") + prop.gcnArchName + ", library built for gfx950");
            return (int)RSVIO_ERR_NO_DEVICE;
        }
        return (int)RSVIO_OK;
    });
}

namespace {
// rsvio_upload_async's copy: 16-B system-scope loads of the page-locked source (host_load2x16:
// each a PCIe read of host memory, nothing served stale from a cache), two per thread in flight
// before the stores; the tail bytes (< 16) by the first thread
__global__ __launch_bounds__(256) void upload_words_kernel(const uint4* src, uint4* __restrict__ dst, long long n_words,
                                                           const unsigned char* src_tail,
                                                           unsigned char* __restrict__ dst_tail, int n_tail) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x, st = (long long)gridDim.x * 256;
    const long long i0 = t, i1 = t + st;
    if (n_words > 0) {
        uint4 a, b;
        rsvio::host_load2x16(src + min(i0, n_words - 1), src + min(i1, n_words - 1), a, b);
        if (i0 < n_words) dst[i0] = a;
        if (i1 < n_words) dst[i1] = b;
    }
    if (t == 0)
        for (int i = 0; i < n_tail; ++i)
            dst_tail[i] = __hip_atomic_load(src_tail + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

int rsvio_upload_async(void* d_dst, const void* h_src, size_t bytes, void* stream) {
    if ((!d_dst || !h_src) && bytes) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        if (!bytes) return (int)RSVIO_OK;
        const hipStream_t s = static_cast<hipStream_t>(stream);
        void* dp = nullptr;
        const bool pinned = hipHostGetDevicePointer(&dp, const_cast<void*>(h_src), 0) == hipSuccess && dp;
        if (!pinned || ((reinterpret_cast<uintptr_t>(dp) | reinterpret_cast<uintptr_t>(d_dst)) & 15)) {
            (void)hipGetLastError();  // (not page-locked, or not 16-B aligned: the runtime's copy)
            RSVIO_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, s));
            return (int)RSVIO_OK;
        }
        const long long nw = (long long)(bytes / 16);
        const int tail = (int)(bytes % 16);
        const unsigned grid = (unsigned)std::max<long long>(1, (nw + 511) / 512);
        auto* src16 = static_cast<const uint4*>(dp);
        auto* dst16 = static_cast<uint4*>(d_dst);
        hipLaunchKernelGGL(upload_words_kernel, dim3(grid), dim3(256), 0, s, src16, dst16, nw,
                           reinterpret_cast<const unsigned char*>(src16 + nw),
                           reinterpret_cast<unsigned char*>(dst16 + nw), tail);
        RSVIO_HIP(hipGetLastError());
        return (int)RSVIO_OK;
    });
}

int rsvio_stream_create(int32_t device, const uint32_t* cu_mask, uint32_t mask_words, void** out) {
    if (!out || (cu_mask && mask_words == 0)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        RSVIO_HIP(hipSetDevice(device));
        hipStream_t s = nullptr;
        if (cu_mask)
            RSVIO_HIP(hipExtStreamCreateWithCUMask(&s, mask_words, cu_mask));
        else
            RSVIO_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        *out = s;
        return (int)RSVIO_OK;
    });
}

int rsvio_stream_destroy(void* stream) {
    if (!stream) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        RSVIO_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
        return (int)RSVIO_OK;
    });
}

int rsvio_tracker_create(const rsvio_tracker_params* params, rsvio_tracker** out) {
    if (!params || !out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto* h = new rsvio_tracker();
        try {
            h->t.init(*params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
        return (int)RSVIO_OK;
    });
}

void rsvio_tracker_destroy(rsvio_tracker* t) { delete t; }

void* rsvio_tracker_stream(rsvio_tracker* t) { return t ? (void*)t->t.stream : nullptr; }

int rsvio_tracker_process_frame(rsvio_tracker* t, const uint8_t* left, const uint8_t* right, size_t stride,
                                rsvio_feature* out_l, size_t cap_l, size_t* n_l, rsvio_feature* out_r,
                                size_t cap_r, size_t* n_r) {
    if (!t || !left || !right || !n_l || !n_r) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& T = t->t;
        const size_t w = (size_t)T.P.width, h = (size_t)T.P.height;
        if (stride == 0) stride = w;
        if (stride < w) throw std::invalid_argument("stride < width");
        T.require_collected("rsvio_tracker_process_frame");
        RSVIO_HIP(hipMemcpy2DAsync(T.d_img.p, w, left, stride, w, h, hipMemcpyHostToDevice, T.stream));
        RSVIO_HIP(hipMemcpy2DAsync(T.d_img.p + w * h, w, right, stride, w, h, hipMemcpyHostToDevice, T.stream));
        T.submit(T.d_img.p, T.d_img.p + w * h);
        return T.fetch(out_l, cap_l, n_l, out_r, cap_r, n_r);
    });
}

int rsvio_tracker_process_frame_device(rsvio_tracker* t, const uint8_t* d_left, const uint8_t* d_right,
                                       rsvio_feature* out_l, size_t cap_l, size_t* n_l, rsvio_feature* out_r,
                                       size_t cap_r, size_t* n_r) {
    if (!t || !d_left || !d_right || !n_l || !n_r) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        t->t.require_collected("rsvio_tracker_process_frame_device");
        t->t.submit(d_left, d_right);
        return t->t.fetch(out_l, cap_l, n_l, out_r, cap_r, n_r);
    });
}

int rsvio_tracker_submit_device(rsvio_tracker* t, const uint8_t* d_left, const uint8_t* d_right) {
    if (!t || !d_left || !d_right) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        t->t.require_collected("rsvio_tracker_submit_device");
        t->t.submit(d_left, d_right);
        return (int)RSVIO_OK;
    });
}

int rsvio_tracker_submit(rsvio_tracker* t, const uint8_t* left, const uint8_t* right, size_t stride) {
    if (!t || !left || !right) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& T = t->t;
        const size_t w = (size_t)T.P.width, h = (size_t)T.P.height;
        if (stride == 0) stride = w;
        if (stride < w) throw std::invalid_argument("stride < width");
        T.require_collected("rsvio_tracker_submit");
        RSVIO_HIP(hipMemcpy2DAsync(T.d_img.p, w, left, stride, w, h, hipMemcpyHostToDevice, T.stream));
        RSVIO_HIP(hipMemcpy2DAsync(T.d_img.p + w * h, w, right, stride, w, h, hipMemcpyHostToDevice, T.stream));
        T.submit(T.d_img.p, T.d_img.p + w * h);
        return (int)RSVIO_OK;
    });
}

int rsvio_tracker_collect(rsvio_tracker* t, rsvio_feature* out_l, size_t cap_l, size_t* n_l, rsvio_feature* out_r,
                          size_t cap_r, size_t* n_r) {
    if (!t || !n_l || !n_r || (cap_l && !out_l) || (cap_r && !out_r)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] { return t->t.fetch(out_l, cap_l, n_l, out_r, cap_r, n_r); });
}

int rsvio_tracker_set_cameras(rsvio_tracker* t, const rsvio_camera* left, const rsvio_camera* right) {
    if (!t || (!left) != (!right)) return RSVIO_ERR_INVALID_ARG;
    if (left && (!rsvio::camera_ok(left) || !rsvio::camera_ok(right))) {
        rsvio::set_last_error("rsvio_tracker_set_cameras: invalid camera");
        return RSVIO_ERR_INVALID_ARG;
    }
    return guarded([&] {
        auto& T = t->t;
        T.require_collected("rsvio_tracker_set_cameras");
        RSVIO_HIP(hipStreamSynchronize(T.stream));
        if (!left) {
            T.cams.on = 0;
            T.last_n[0] = T.last_n[1] = 0;
            return (int)RSVIO_OK;
        }
        if (!T.undist.p) {
            T.undist.alloc((size_t)4 * T.cap);
            T.h_undist.alloc((size_t)4 * T.cap);
            T.tmp_und.alloc((size_t)T.cap);
        }
        T.cams.cam[0] = *left;
        T.cams.cam[1] = *right;
        T.cams.on = 1;
        return (int)RSVIO_OK;
    });
}

int rsvio_tracker_undistorted(rsvio_tracker* t, float* out_l, size_t cap_l, float* out_r, size_t cap_r) {
    if (!t || (cap_l && !out_l) || (cap_r && !out_r)) return RSVIO_ERR_INVALID_ARG;
    auto& T = t->t;
    if (!T.cams.on) {
        rsvio::set_last_error("rsvio_tracker_undistorted: no cameras attached");
        return RSVIO_ERR_INVALID_ARG;
    }
    if (cap_l < T.last_n[0] || cap_r < T.last_n[1]) return RSVIO_ERR_CAPACITY;
    // the collected frame's slot: a frame submitted since copies into the other one
    std::memcpy(out_l, T.hund(T.rslot, 0), T.last_n[0] * sizeof(float2));
    std::memcpy(out_r, T.hund(T.rslot, 1), T.last_n[1] * sizeof(float2));
    return RSVIO_OK;
}

int rsvio_tracker_remove_ids(rsvio_tracker* t, const uint64_t* ids, size_t n) {
    if (!t || (!ids && n)) return RSVIO_ERR_INVALID_ARG;
    if (n == 0) return RSVIO_OK;
    return guarded([&] {
        auto& T = t->t;
        T.require_collected("rsvio_tracker_remove_ids");
        if (T.rm_ids.n < n) T.rm_ids.alloc(n);
        RSVIO_HIP(hipMemcpyAsync(T.rm_ids.p, ids, n * sizeof(uint64_t), hipMemcpyHostToDevice, T.stream));
        hipLaunchKernelGGL(rsvio::remove_ids_kernel, dim3(1), dim3(1024), 0, T.stream, T.rm_ids.p, (int)n, T.maff(0),
                           T.maff(1), T.mid(0), T.mid(1), T.tmp_aff.p, T.ids_tmp.p, T.counts.p, T.outp(T.rslot, 0),
                           T.outp(T.rslot, 1), T.undp(T.rslot, 0), T.undp(T.rslot, 1), T.tmp_und.p);
        RSVIO_HIP(hipGetLastError());
        RSVIO_HIP(hipMemcpyAsync(T.h_counts.p, T.counts.p, sizeof(int) * 2, hipMemcpyDeviceToHost, T.stream));
        RSVIO_HIP(hipStreamSynchronize(T.stream));
        T.host_count[0] = T.h_counts.p[0];
        T.host_count[1] = T.h_counts.p[1];
        T.coll_n[0] = std::min(T.host_count[0], T.cap);
        T.coll_n[1] = std::min(T.host_count[1], T.cap);
        if (T.cams.on) {  // undistorted() stays aligned with the compacted feature lists
            const size_t nl = std::min(T.last_n[0], (size_t)T.host_count[0]);
            const size_t nr = std::min(T.last_n[1], (size_t)T.host_count[1]);
            if (nl) RSVIO_HIP(hipMemcpyAsync(T.hund(T.rslot, 0), T.undp(T.rslot, 0), nl * sizeof(float2), hipMemcpyDeviceToHost, T.stream));
            if (nr) RSVIO_HIP(hipMemcpyAsync(T.hund(T.rslot, 1), T.undp(T.rslot, 1), nr * sizeof(float2),
                                             hipMemcpyDeviceToHost, T.stream));
            RSVIO_HIP(hipStreamSynchronize(T.stream));
            T.last_n[0] = nl;
            T.last_n[1] = nr;
        }
        return (int)RSVIO_OK;
    });
}

size_t rsvio_pyramid_bytes(int32_t w, int32_t h, int32_t levels) {
    if (w <= 0 || h <= 0 || levels <= 0) return 0;
    return rsvio::level_offset((uint32_t)w, (uint32_t)h, levels);
}

int rsvio_track_ctx_create(int32_t w, int32_t h, int32_t levels, int32_t device, rsvio_track_ctx** out) {
    if (!out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        RSVIO_HIP(hipSetDevice(device));
        auto* c = new rsvio_track_ctx();
        try {
            c->c.device = device;
            c->c.plan.init(w, h, levels);
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
        return (int)RSVIO_OK;
    });
}

void rsvio_track_ctx_destroy(rsvio_track_ctx* c) { delete c; }

int rsvio_build_pyramids_d(rsvio_track_ctx* c, const uint8_t* d_imgs, int32_t n_img, uint8_t* d_pyrs, void* stream) {
    if (!c || !d_imgs || !d_pyrs || n_img < 0) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        c->c.plan.enqueue(d_imgs, n_img, d_pyrs, (hipStream_t)stream);
        return (int)RSVIO_OK;
    });
}

int rsvio_track_points_d(rsvio_track_ctx* c, const rsvio_track_batch* batches, int32_t n_batches,
                         int32_t max_iterations, float thresh, void* stream) {
    if (!c || !batches || n_batches < 0 || n_batches > rsvio::kMaxTrackBatches) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        rsvio::TrackLaunch L{};
        L.w = c->c.plan.w; L.h = c->c.plan.h; L.levels = c->c.plan.levels;
        L.max_iter = max_iterations; L.thresh = thresh; L.nb = n_batches;
        L.start[0] = 0;
        for (int b = 0; b < n_batches; ++b) {
            if (batches[b].n < 0) throw std::invalid_argument("negative batch size");
            L.start[b + 1] = L.start[b] + batches[b].n;
            L.pyr0[b] = batches[b].d_pyr0; L.pyr1[b] = batches[b].d_pyr1;
            L.ain[b] = batches[b].d_aff_in; L.aout[b] = batches[b].d_aff_out; L.valid[b] = batches[b].d_valid;
            L.dcount[b] = nullptr;
        }
        rsvio::enqueue_track(L, (hipStream_t)stream);
        return (int)RSVIO_OK;
    });
}

int rsvio_track_points_table_d(rsvio_track_ctx* c, const rsvio_track_batch* d_table, const int32_t* d_start,
                               int32_t n_batches, int32_t total, int32_t max_iterations, float thresh,
                               void* stream) {
    if (!c || n_batches < 0 || total < 0 || (n_batches > 0 && (!d_table || !d_start))) return RSVIO_ERR_INVALID_ARG;
    if (n_batches == 0 || total == 0) return RSVIO_OK;
    return guarded([&] {
        rsvio::TrackLaunch L{};
        L.w = c->c.plan.w; L.h = c->c.plan.h; L.levels = c->c.plan.levels;
        L.max_iter = max_iterations; L.thresh = thresh; L.nb = n_batches;
        L.start[0] = total;  // table mode: the grid size
        L.table = d_table;
        L.tstart = d_start;
        rsvio::enqueue_track(L, (hipStream_t)stream);
        return (int)RSVIO_OK;
    });
}

int rsvio_build_pyramid(const uint8_t* img, int32_t w, int32_t h, int32_t levels, uint8_t* out) {
    if (!img || !out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        rsvio::PyramidPlan plan;
        plan.init(w, h, levels);
        rsvio::DevBuf<uint8_t> di((size_t)w * h), dp(plan.pyr_bytes());
        RSVIO_HIP(hipMemcpy(di.p, img, (size_t)w * h, hipMemcpyHostToDevice));
        plan.enqueue(di.p, 1, dp.p, nullptr);
        RSVIO_HIP(hipMemcpy(out, dp.p, plan.pyr_bytes(), hipMemcpyDeviceToHost));
        return (int)RSVIO_OK;
    });
}

int rsvio_track_points(const uint8_t* pyr0, const uint8_t* pyr1, int32_t w, int32_t h, int32_t levels,
                       const float* aff_in, int32_t n, int32_t max_iterations, float thresh, float* aff_out,
                       uint8_t* valid_out) {
    if (!pyr0 || !pyr1 || n < 0 || (n > 0 && (!aff_in || !aff_out || !valid_out))) return RSVIO_ERR_INVALID_ARG;
    if (levels < 1 || levels > rsvio::kMaxLevels || w < 1 || h < 1) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        const size_t pb = rsvio::level_offset(w, h, levels);
        rsvio::DevBuf<uint8_t> d0(pb), d1(pb), dv(std::max(n, 1));
        rsvio::DevBuf<float> ai((size_t)std::max(n, 1) * 6), ao((size_t)std::max(n, 1) * 6);
        RSVIO_HIP(hipMemcpy(d0.p, pyr0, pb, hipMemcpyHostToDevice));
        RSVIO_HIP(hipMemcpy(d1.p, pyr1, pb, hipMemcpyHostToDevice));
        if (n) RSVIO_HIP(hipMemcpy(ai.p, aff_in, sizeof(float) * 6 * n, hipMemcpyHostToDevice));
        rsvio::TrackLaunch L{};
        L.w = w; L.h = h; L.levels = levels; L.max_iter = max_iterations; L.thresh = thresh; L.nb = 1;
        L.start[0] = 0; L.start[1] = n;
        L.pyr0[0] = d0.p; L.pyr1[0] = d1.p; L.ain[0] = ai.p; L.aout[0] = ao.p; L.valid[0] = dv.p;
        L.dcount[0] = nullptr;
        rsvio::enqueue_track(L, nullptr);
        if (n) {
            RSVIO_HIP(hipMemcpy(aff_out, ao.p, sizeof(float) * 6 * n, hipMemcpyDeviceToHost));
            RSVIO_HIP(hipMemcpy(valid_out, dv.p, n, hipMemcpyDeviceToHost));
        }
        return (int)RSVIO_OK;
    });
}

int rsvio_detect_keypoints(const uint8_t* img, int32_t w, int32_t h, int32_t grid, const float* existing_xy,
                           int32_t n_existing, uint32_t* out_xy, float* out_score, int32_t cap, int32_t* n_out) {
    if (!img || !out_xy || !n_out || n_existing < 0 || (n_existing && !existing_xy) || grid < 8 || grid > 128 ||
        grid > w || grid > h)
        return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        rsvio::GridGeom G = rsvio::make_grid(w, h, grid);
        const int n_cells = G.cells_x * G.cells_y;
        const int ne = std::max(n_existing, 1);
        rsvio::DevBuf<uint8_t> di((size_t)w * h);
        rsvio::DevBuf<float> ea((size_t)ne * 6), na((size_t)n_cells * 6), ns(n_cells);
        rsvio::DevBuf<int> nc(1);
        rsvio::DevBuf<int4> cp(n_cells);
        RSVIO_HIP(hipMemcpy(di.p, img, (size_t)w * h, hipMemcpyHostToDevice));
        std::vector<float> aff((size_t)ne * 6, 0.0f);
        for (int i = 0; i < n_existing; ++i) {
            aff[6 * i + 4] = existing_xy[2 * i];
            aff[6 * i + 5] = existing_xy[2 * i + 1];
        }
        RSVIO_HIP(hipMemcpy(ea.p, aff.data(), sizeof(float) * aff.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(rsvio::fast_cells_kernel, dim3(n_cells), dim3(256), (size_t)grid * grid, nullptr, di.p, G,
                           ea.p, nullptr, n_existing, cp.p, nullptr);
        RSVIO_HIP(hipGetLastError());
        hipLaunchKernelGGL(rsvio::gather_new_kernel, dim3(1), dim3(1024), 0, nullptr, cp.p, n_cells, na.p, nc.p, ns.p);
        RSVIO_HIP(hipGetLastError());
        int m = 0;
        RSVIO_HIP(hipMemcpy(&m, nc.p, sizeof(int), hipMemcpyDeviceToHost));
        std::vector<float> a((size_t)std::max(m, 1) * 6), sc(std::max(m, 1));
        if (m) {
            RSVIO_HIP(hipMemcpy(a.data(), na.p, sizeof(float) * 6 * m, hipMemcpyDeviceToHost));
            RSVIO_HIP(hipMemcpy(sc.data(), ns.p, sizeof(float) * m, hipMemcpyDeviceToHost));
        }
        const int k = std::min(m, cap);
        for (int i = 0; i < k; ++i) {
            out_xy[2 * i] = (uint32_t)a[6 * i + 4];
            out_xy[2 * i + 1] = (uint32_t)a[6 * i + 5];
            if (out_score) out_score[i] = sc[i];
        }
        *n_out = k;
        return m > cap ? (int)RSVIO_ERR_CAPACITY : (int)RSVIO_OK;
    });
}

}  // extern "C"
