// ft_tracker.hip -- device-resident FeatureTracker of the feature_tracker/ crate and its C ABI.
//
// Replaces FeatureTracker::{new, process_frame, get_pyramid} (feature_tracker/src/
// feature_tracker.rs:51-194).  Per frame, on one HIP stream, nothing leaves HBM except the
// frame's feature list:
//   pyramid (blur + one resize launch per level)                  ft_track.hip
//   LK forward + backward of the previous frame's features        ft_track.hip
//   Shi-Tomasi score, NMS, local maxima vs the tracked features   ft_detect.hip
//   assembly: tracked (previous order) then new corners, new ids  ft_detect.hip
// The feature list and the pyramid ping-pong between two slots (the reference moves them into
// previous_frame_pyramid, :184).
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "ft.hpp"

namespace rsvio {
namespace ft {

namespace {

struct Scratch {
    DevBuf<float> planes, tmp, score, nms_score;
    DevBuf<uint32_t> nms, stats, staging;
    DevBuf<uint2> tpos;
    DevBuf<uint8_t> supp, keep;
    DevBuf<uint32_t> clist;
    DevBuf<int> row_count;
    DetectBufs D{};

    void init(int w, int h, float detection_blur, int tracked_cap) {
        const size_t n = (size_t)w * h;
        D.w = w;
        D.h = h;
        D.r = 1;  // feature_detection.rs:59
        D.nbx = (w + D.r) / (D.r + 1);
        D.nby = (h + D.r) / (D.r + 1);
        if (D.nbx > 1024) throw std::invalid_argument("image wider than 2048 pixels");
        planes.alloc(3 * n);
        tmp.alloc(3 * n);
        score.alloc(n);
        nms.alloc((size_t)D.nbx * D.nby);
        nms_score.alloc((size_t)D.nbx * D.nby);
        stats.alloc(4);
        staging.alloc((size_t)D.nbx * D.nby);
        tpos.alloc(std::max(1, tracked_cap));
        supp.alloc((size_t)D.nbx * D.nby);
        keep.alloc((size_t)D.nbx * D.nby);
        clist.alloc((size_t)D.nbx * D.nby);
        row_count.alloc(D.nby);
        D.planes = planes.p;
        D.tmp = tmp.p;
        D.score = score.p;
        D.nms = nms.p;
        D.nms_score = nms_score.p;
        D.stats = stats.p;
        D.tpos = tpos.p;
        D.supp = supp.p;
        D.keep = keep.p;
        D.clist = clist.p;
        D.tpos_cap = std::max(1, tracked_cap);
        D.staging = staging.p;
        D.row_count = row_count.p;
        boxes_for_gauss(detection_blur, 3, D.boxes);
    }
};

}  // namespace

struct Tracker {
    rsvio_ft_config C{};
    PyrPlan plan;
    Scratch S;
    hipStream_t stream = nullptr;
    int cap = 0;
    int cur = 0;
    bool has_prev = false;
    int n_prev = 0;
    DevBuf<float> d_img, d_pyr;         // image; 2 pyramid slots
    DevBuf<uint64_t> ids;               // 2 x cap
    DevBuf<float2> xy, xy_tr;           // 2 x cap; cap
    DevBuf<uint8_t> valid;              // cap
    DevBuf<int> counts;                 // {n, n_tracked, overflow}
    DevBuf<unsigned long long> last_id;
    HostBuf<int> h_counts;
    HostBuf<uint64_t> h_ids;
    HostBuf<float2> h_xy;

    float* pyr(int slot) { return d_pyr.p + (size_t)slot * plan.g.total; }

    void init(const rsvio_ft_config& c) {
        C = c;
        if (C.width < 16 || C.height < 16 || C.nlevels < 1 || C.nlevels > kMaxLevels || C.optical_flow_max_iter < 0 ||
            !(C.ratio > 0.0) || (C.matching_cost != kSSD && C.matching_cost != kLSSD) ||
            C.detection_min_dist * 2 >= (uint32_t)std::min(C.width, C.height) || C.max_features < 0)
            throw std::invalid_argument("invalid FeatureTrackingConfig");
        cap = C.max_features > 0 ? C.max_features : 8192;
        RSVIO_HIP(hipSetDevice(C.device));
        RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        plan.init(C.width, C.height, C.nlevels, C.ratio, C.preprocessing_blur != 0, C.preprocessing_blur_sigma);
        S.init(C.width, C.height, C.detection_blur, cap);
        d_img.alloc((size_t)C.width * C.height);
        d_pyr.alloc(2 * (size_t)plan.g.total);
        ids.alloc(2 * (size_t)cap);
        xy.alloc(2 * (size_t)cap);
        xy_tr.alloc(cap);
        valid.alloc(cap);
        counts.alloc(3);
        last_id.alloc(1);
        h_counts.alloc(3);
        h_ids.alloc(cap);
        h_xy.alloc(cap);
        RSVIO_HIP(hipMemsetAsync(last_id.p, 0, sizeof(unsigned long long), stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
    }
    ~Tracker() {
        if (stream) (void)hipStreamDestroy(stream);
    }

    void enqueue_frame(const float* d_image) {
        const int nxt = has_prev ? 1 - cur : cur;
        enqueue_pyramid(plan, d_image, pyr(nxt), stream);
        const int n_tr = has_prev ? n_prev : 0;
        if (n_tr > 0) {
            LkLaunch L{};
            L.pyr0 = pyr(cur);
            L.pyr1 = pyr(nxt);
            L.g = plan.g;
            L.xy = xy.p + (size_t)cur * cap;
            L.n = n_tr;
            L.max_iter = C.optical_flow_max_iter;
            L.lambda = C.optical_flow_lm_lambda;
            L.cost = C.matching_cost;
            L.xy_out = xy_tr.p;
            L.valid = valid.p;
            L.iso_out = nullptr;
            enqueue_lk(L, stream);
        }
        enqueue_score(S.D, pyr(nxt), stream);
        enqueue_select(S.D, C.detection_threshold, (int)C.detection_min_dist, xy_tr.p, valid.p, n_tr, stream);
        Assemble A{};
        A.n_prev = n_tr;
        A.ids_prev = ids.p + (size_t)cur * cap;
        A.xy_tracked = xy_tr.p;
        A.valid = valid.p;
        A.staging = S.D.staging;
        A.row_count = S.D.row_count;
        A.nby = S.D.nby;
        A.nbx = S.D.nbx;
        A.ids_cur = ids.p + (size_t)nxt * cap;
        A.xy_cur = xy.p + (size_t)nxt * cap;
        A.cap = cap;
        A.last_id = last_id.p;
        A.count_out = counts.p;
        enqueue_assemble(A, stream);
        cur = nxt;
        has_prev = true;
    }

    // Read the frame's features back (2 round trips: the count, then the list).
    int fetch(rsvio_ft_feature* out, size_t cap_out, size_t* n_out) {
        RSVIO_HIP(hipMemcpyAsync(h_counts.p, counts.p, 3 * sizeof(int), hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
        n_prev = h_counts.p[0];
        const size_t n = std::min((size_t)n_prev, cap_out);
        if (n) {
            RSVIO_HIP(hipMemcpyAsync(h_ids.p, ids.p + (size_t)cur * cap, n * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                     stream));
            RSVIO_HIP(hipMemcpyAsync(h_xy.p, xy.p + (size_t)cur * cap, n * sizeof(float2), hipMemcpyDeviceToHost,
                                     stream));
            RSVIO_HIP(hipStreamSynchronize(stream));
            for (size_t i = 0; i < n; ++i) {
                out[i].feature_id = h_ids.p[i];
                out[i].x = h_xy.p[i].x;
                out[i].y = h_xy.p[i].y;
            }
        }
        *n_out = n;
        if (h_counts.p[2] || n < (size_t)n_prev) {
            set_last_error("FeatureTracker: frame has more features than the output capacity");
            return RSVIO_ERR_CAPACITY;
        }
        return RSVIO_OK;
    }
};

}  // namespace ft
}  // namespace rsvio

struct rsvio_ft {
    rsvio::ft::Tracker t;
};

using rsvio::guarded;
namespace F = rsvio::ft;

namespace {

template <class T>
struct Dev {
    rsvio::DevBuf<T> b;
    Dev(const T* host, size_t n) : b(n) {
        if (n && host) RSVIO_HIP(hipMemcpy(b.p, host, n * sizeof(T), hipMemcpyHostToDevice));
    }
    explicit Dev(size_t n) : b(n) {}
    void get(T* host, size_t n) const {
        if (n) RSVIO_HIP(hipMemcpy(host, b.p, n * sizeof(T), hipMemcpyDeviceToHost));
    }
};

int check_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        rsvio::set_last_error("no HIP device visible");
        return RSVIO_ERR_NO_DEVICE;
    }
    return RSVIO_OK;
}

}  // namespace

extern "C" {

int rsvio_ft_create(const rsvio_ft_config* cfg, rsvio_ft** out) {
    if (!cfg || !out) return RSVIO_ERR_INVALID_ARG;
    if (check_device() != RSVIO_OK) return RSVIO_ERR_NO_DEVICE;
    return guarded([&] {
        auto* h = new rsvio_ft();
        try {
            h->t.init(*cfg);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
        return (int)RSVIO_OK;
    });
}

void rsvio_ft_destroy(rsvio_ft* t) { delete t; }

void* rsvio_ft_stream(rsvio_ft* t) { return t ? (void*)t->t.stream : nullptr; }

int rsvio_ft_process_frame(rsvio_ft* t, const float* img, size_t stride, rsvio_ft_feature* out, size_t cap,
                           size_t* n) {
    if (!t || !img || !n || (cap && !out)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& T = t->t;
        const size_t w = (size_t)T.C.width, h = (size_t)T.C.height;
        if (stride == 0) stride = w;
        if (stride < w) throw std::invalid_argument("stride < width");
        RSVIO_HIP(hipMemcpy2DAsync(T.d_img.p, w * sizeof(float), img, stride * sizeof(float), w * sizeof(float), h,
                                   hipMemcpyHostToDevice, T.stream));
        T.enqueue_frame(T.d_img.p);
        return T.fetch(out, cap, n);
    });
}

int rsvio_ft_process_frame_device(rsvio_ft* t, const float* d_img, rsvio_ft_feature* out, size_t cap, size_t* n) {
    if (!t || !d_img || !n || (cap && !out)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        t->t.enqueue_frame(d_img);
        return t->t.fetch(out, cap, n);
    });
}

int rsvio_ft_get_pyramid(rsvio_ft* t, float* out, size_t cap_floats) {
    if (!t || !out) return RSVIO_ERR_INVALID_ARG;
    auto& T = t->t;
    if (!T.has_prev) {
        rsvio::set_last_error("rsvio_ft_get_pyramid: no frame processed yet");
        return RSVIO_ERR_INVALID_ARG;
    }
    if (cap_floats < (size_t)T.plan.g.total) return RSVIO_ERR_CAPACITY;
    return guarded([&] {
        RSVIO_HIP(hipMemcpyAsync(out, T.pyr(T.cur), sizeof(float) * T.plan.g.total, hipMemcpyDeviceToHost, T.stream));
        RSVIO_HIP(hipStreamSynchronize(T.stream));
        return (int)RSVIO_OK;
    });
}

size_t rsvio_ft_pyramid_floats(int32_t w, int32_t h, int32_t nlevels, double ratio) {
    try {
        return (size_t)F::make_geom(w, h, nlevels, ratio).total;
    } catch (...) {
        return 0;
    }
}

int rsvio_ft_build_pyramid(const float* img, int32_t w, int32_t h, int32_t nlevels, double ratio, int32_t blur,
                           float sigma, float* out) {
    if (!img || !out || w <= 0 || h <= 0) return RSVIO_ERR_INVALID_ARG;
    if (check_device() != RSVIO_OK) return RSVIO_ERR_NO_DEVICE;
    return guarded([&] {
        F::PyrPlan P;
        P.init(w, h, nlevels, ratio, blur != 0, sigma);
        Dev<float> di(img, (size_t)w * h), dp((size_t)P.g.total);
        F::enqueue_pyramid(P, di.b.p, dp.b.p, nullptr);
        RSVIO_HIP(hipDeviceSynchronize());
        dp.get(out, (size_t)P.g.total);
        return (int)RSVIO_OK;
    });
}

int rsvio_ft_track_points(const float* pyr0, const float* pyr1, int32_t w, int32_t h, int32_t nlevels, double ratio,
                          const float* xy, int32_t n, int32_t max_iter, float lm_lambda, int32_t matching_cost,
                          float* iso_out, uint8_t* valid_out) {
    if (!pyr0 || !pyr1 || n < 0 || (n > 0 && (!xy || !iso_out || !valid_out)) || max_iter < 0 ||
        (matching_cost != F::kSSD && matching_cost != F::kLSSD))
        return RSVIO_ERR_INVALID_ARG;
    if (check_device() != RSVIO_OK) return RSVIO_ERR_NO_DEVICE;
    if (n == 0) return RSVIO_OK;
    return guarded([&] {
        const F::PyrGeom g = F::make_geom(w, h, nlevels, ratio);
        Dev<float> d0(pyr0, (size_t)g.total), d1(pyr1, (size_t)g.total);
        Dev<float2> dxy(reinterpret_cast<const float2*>(xy), n), dout(n);
        Dev<uint8_t> dv(n);
        Dev<float4> diso(n);
        F::LkLaunch L{};
        L.pyr0 = d0.b.p;
        L.pyr1 = d1.b.p;
        L.g = g;
        L.xy = dxy.b.p;
        L.n = n;
        L.max_iter = max_iter;
        L.lambda = lm_lambda;
        L.cost = matching_cost;
        L.xy_out = dout.b.p;
        L.valid = dv.b.p;
        L.iso_out = diso.b.p;
        F::enqueue_lk(L, nullptr);
        RSVIO_HIP(hipDeviceSynchronize());
        diso.get(reinterpret_cast<float4*>(iso_out), n);
        dv.get(valid_out, n);
        return (int)RSVIO_OK;
    });
}

int rsvio_ft_shi_tomasi_score(const float* img, int32_t w, int32_t h, float detection_blur, float* score) {
    if (!img || !score || w < 4 || h < 4 || w > 2048) return RSVIO_ERR_INVALID_ARG;
    if (check_device() != RSVIO_OK) return RSVIO_ERR_NO_DEVICE;
    return guarded([&] {
        F::Scratch S;
        S.init(w, h, detection_blur, 1);
        Dev<float> di(img, (size_t)w * h);
        F::enqueue_score(S.D, di.b.p, nullptr);
        RSVIO_HIP(hipDeviceSynchronize());
        RSVIO_HIP(hipMemcpy(score, S.D.score, sizeof(float) * w * h, hipMemcpyDeviceToHost));
        return (int)RSVIO_OK;
    });
}

int rsvio_ft_add_points(const float* fine, int32_t w, int32_t h, const float* tracked_xy, int32_t n_tracked,
                        float threshold, int32_t min_dist, float detection_blur, uint32_t* out_xy, int32_t cap,
                        int32_t* n_out) {
    if (!fine || !n_out || w < 4 || h < 4 || w > 2048 || n_tracked < 0 || (n_tracked && !tracked_xy) || cap < 0 ||
        (cap && !out_xy) || min_dist < 0 || 2 * min_dist >= std::min(w, h))
        return RSVIO_ERR_INVALID_ARG;
    if (check_device() != RSVIO_OK) return RSVIO_ERR_NO_DEVICE;
    return guarded([&] {
        F::Scratch S;
        S.init(w, h, detection_blur, n_tracked);
        Dev<float> di(fine, (size_t)w * h);
        Dev<float2> dt(reinterpret_cast<const float2*>(tracked_xy), (size_t)n_tracked);
        F::enqueue_score(S.D, di.b.p, nullptr);
        F::enqueue_select(S.D, threshold, min_dist, dt.b.p, nullptr, n_tracked, nullptr);
        RSVIO_HIP(hipDeviceSynchronize());
        std::vector<int> rc(S.D.nby);
        std::vector<uint32_t> st((size_t)S.D.nbx * S.D.nby);
        RSVIO_HIP(hipMemcpy(rc.data(), S.D.row_count, sizeof(int) * rc.size(), hipMemcpyDeviceToHost));
        RSVIO_HIP(hipMemcpy(st.data(), S.D.staging, sizeof(uint32_t) * st.size(), hipMemcpyDeviceToHost));
        int k = 0;
        for (int r = 0; r < S.D.nby; ++r)
            for (int j = 0; j < rc[r]; ++j, ++k)
                if (k < cap) {
                    const uint32_t c = st[(size_t)r * S.D.nbx + j];
                    out_xy[2 * k] = c & 0xFFFFu;
                    out_xy[2 * k + 1] = c >> 16;
                }
        *n_out = k;
        return k <= cap ? (int)RSVIO_OK : (int)RSVIO_ERR_CAPACITY;
    });
}

}  // extern "C"
