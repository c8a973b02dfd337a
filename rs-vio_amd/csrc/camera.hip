// camera.hip -- batched unprojection (T12, src/estimator/frame.rs:107-134) behind
// rsvio_unproject / rsvio_unproject_d.  The per-point math is rsvio::unproject_one
// (camera.hpp), which the tracker also fuses into its output packing.
//
// One lane per point; f64 VALU work (radtan: a handful of Newton steps of ~50 flops and two
// IEEE divisions) over 8 B in / 9 B out per point.  At config-5 sizes (80,000 observations)
// this is one short launch; the roofline is the f64 VALU rate.
#include "camera.hpp"
#include "common.hpp"

namespace rsvio {

__global__ __launch_bounds__(256) void unproject_kernel(rsvio_camera cam, const float2* __restrict__ px,
                                                        int n, float2* __restrict__ out,
                                                        uint8_t* __restrict__ valid) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 q = px[i];
    const Undist r = unproject_one(cam, q.x, q.y);
    out[i] = make_float2(r.x, r.y);
    if (valid) valid[i] = r.ok ? 1 : 0;
}

bool camera_ok(const rsvio_camera* c) {
    if (!c) return false;
    if (c->model != RSVIO_CAM_OPENCV5 && c->model != RSVIO_CAM_EUCM) return false;
    if (c->convention != RSVIO_UNPROJ_PLANE && c->convention != RSVIO_UNPROJ_RAY) return false;
    return c->params[0] != 0.0 && c->params[1] != 0.0;
}

void enqueue_unproject(const rsvio_camera& cam, const float* d_px, size_t n, float* d_out, uint8_t* d_valid,
                       hipStream_t stream) {
    if (n == 0) return;
    if (n > (size_t)INT32_MAX) throw std::invalid_argument("too many points");
    const int blocks = (int)((n + 255) / 256);
    hipLaunchKernelGGL(unproject_kernel, dim3(blocks), dim3(256), 0, stream, cam,
                       reinterpret_cast<const float2*>(d_px), (int)n, reinterpret_cast<float2*>(d_out), d_valid);
    RSVIO_HIP(hipGetLastError());
}

}  // namespace rsvio

extern "C" {

int rsvio_unproject(const rsvio_camera* cam, const float* px, size_t n, float* out_xy, uint8_t* valid_out) {
    if (!rsvio::camera_ok(cam) || (n && (!px || !out_xy))) {
        rsvio::set_last_error("rsvio_unproject: invalid camera or buffers");
        return RSVIO_ERR_INVALID_ARG;
    }
    return rsvio::guarded([&] {
        if (n == 0) return (int)RSVIO_OK;
        rsvio::DevBuf<float> dp(2 * n), dout(2 * n);
        rsvio::DevBuf<uint8_t> dv(n);
        RSVIO_HIP(hipMemcpy(dp.p, px, sizeof(float) * 2 * n, hipMemcpyHostToDevice));
        rsvio::enqueue_unproject(*cam, dp.p, n, dout.p, dv.p, nullptr);
        RSVIO_HIP(hipMemcpy(out_xy, dout.p, sizeof(float) * 2 * n, hipMemcpyDeviceToHost));
        if (valid_out) RSVIO_HIP(hipMemcpy(valid_out, dv.p, n, hipMemcpyDeviceToHost));
        return (int)RSVIO_OK;
    });
}

int rsvio_unproject_d(const rsvio_camera* cam, const float* d_px, size_t n, float* d_out_xy,
                      uint8_t* d_valid_out, void* stream) {
    if (!rsvio::camera_ok(cam) || (n && (!d_px || !d_out_xy))) {
        rsvio::set_last_error("rsvio_unproject_d: invalid camera or buffers");
        return RSVIO_ERR_INVALID_ARG;
    }
    return rsvio::guarded([&] {
        rsvio::enqueue_unproject(*cam, d_px, n, d_out_xy, d_valid_out, static_cast<hipStream_t>(stream));
        return (int)RSVIO_OK;
    });
}

}  // extern "C"
