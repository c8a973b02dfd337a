// ft.hpp -- the feature_tracker/ crate variant: launch
// descriptors shared by ft_track.hip (pyramid + LK), ft_detect.hip (Shi-Tomasi detection) and
// ft_tracker.hip (the FeatureTracker handle and its C ABI).
//
// Images are f32 luma in [0, 1] (DynamicImage::to_luma32f, players/tartanair_player.rs:53).
// A pyramid is packed: level l (round(w / ratio^l) x round(h / ratio^l), image_operations.rs:69-70)
// starts at float offset off[l].
#pragma once
#include <vector>

#include "common.hpp"

namespace rsvio {
namespace ft {

constexpr int kMaxLevels = 8;
constexpr uint32_t kNone = 0xFFFFFFFFu;

struct PyrGeom {
    int n;
    int w[kMaxLevels], h[kMaxLevels];
    long off[kMaxLevels];
    long total;
};
PyrGeom make_geom(int w, int h, int nlevels, double ratio);

// ---- resampling (image 0.25 sample.rs) ----
// One 1-D pass: for output index o, taps left[o] .. left[o] + cnt[o] - 1 with weights
// w[woff[o] ..], already normalised (the reference's f32 arithmetic, built on the host).
struct TapsDev {
    const int* left;
    const int* cnt;
    const int* woff;
    const float* w;
};
// Host-built tap tables for a whole pyramid (blur + every resize), uploaded once per handle.
struct PyrPlan {
    PyrGeom g;
    bool blur = false;
    int span[kMaxLevels] = {0};                      // max source columns of a 64-wide output tile
    bool copy[kMaxLevels] = {false};                 // same-size resize = copy
    DevBuf<int> meta;                                // left | cnt | woff of every pass
    DevBuf<float> wts;
    int n_meta = 0;
    // pass p = 2 * level + {0: vertical, 1: horizontal}; level 0 = the pre-blur
    int moff[2 * kMaxLevels] = {};
    void init(int w, int h, int nlevels, double ratio, bool blur_on, float sigma);
    TapsDev taps(int pass) const;
};
// Build the packed pyramid of `img` (w x h f32) into `pyr` on `s`.
void enqueue_pyramid(const PyrPlan& P, const float* img, float* pyr, hipStream_t s);

// ---- LK (feature_tracking.rs:16-192, patch.rs:57-255) ----
enum { kSSD = 0, kLSSD = 1 };
struct LkLaunch {
    const float* pyr0;    // previous frame
    const float* pyr1;    // current frame
    PyrGeom g;
    const float2* xy;     // n feature centres (previous frame)
    int n;
    int max_iter;
    float lambda;
    int cost;
    float2* xy_out;       // forward-tracked centre (transform0 * centre)
    uint8_t* valid;
    float4* iso_out;      // optional: forward transform {cos, sin, tx, ty}
};
void enqueue_lk(const LkLaunch& L, hipStream_t s);

// ---- detection (feature_detection.rs:47-285) ----
struct DetectBufs {
    int w, h;
    int r;                 // suppress_non_maximum radius (1, feature_detection.rs:59)
    int nbx, nby;          // NMS blocks: ceil(w / (r + 1)) x ceil(h / (r + 1))
    float* planes;         // 3 x w x h: dxx, dyy, dxy, blurred in place
    float* tmp;            // 3 x w x h transposed half-pass scratch
    float* score;          // w x h
    uint32_t* nms;         // nbx x nby packed corner (x | y << 16) or kNone
    float* nms_score;      // nbx x nby
    uint32_t* stats;       // [0] max(bits(score)) + 1 over corners (0: none), [1] max candidate y + 1,
                           // [2] corner count
    uint32_t* clist;       // corner block indices (any order)
    uint8_t* keep;         // nbx x nby: corner survives local_maxima and the border filter
    uint2* tpos;           // tracked positions (round, saturating) or {kNone, kNone}
    uint8_t* supp;         // nbx x nby: corner suppressed by a tracked feature
    int tpos_cap;
    uint32_t* staging;     // nby x nbx survivors (x | y << 16), (y, x) order within a block row
    int* row_count;        // nby
    int boxes[3];          // fast_blur box widths (boxes_for_gauss(detection_blur, 3))
};
void boxes_for_gauss(float sigma, int n, int* out);
// score map of the fine level (grad, 3 x fast_blur, Shi-Tomasi score)
void enqueue_score(const DetectBufs& D, const float* fine, hipStream_t s);
// NMS + local maxima against the tracked features (valid[i] (null: all) && round(xy[i]))
// -> staging / row_count
void enqueue_select(const DetectBufs& D, float threshold, int min_dist, const float2* tracked_xy,
                    const uint8_t* tracked_valid, int n_tracked, hipStream_t s);

// Frame assembly: surviving tracks (previous order) then new corners ((y, x) order) with
// consecutive ids, into the device list of the current frame.
struct Assemble {
    int n_prev;
    const uint64_t* ids_prev;
    const float2* xy_tracked;     // n_prev forward-tracked centres
    const uint8_t* valid;         // n_prev
    const uint32_t* staging;
    const int* row_count;
    int nby, nbx;
    uint64_t* ids_cur;
    float2* xy_cur;
    int cap;
    unsigned long long* last_id;  // device counter (next id)
    int* count_out;               // device: {n_cur (<= cap), n_tracked, overflow}
};
void enqueue_assemble(const Assemble& A, hipStream_t s);

}  // namespace ft
}  // namespace rsvio
