// common.hpp -- shared helpers for the rsvio_gpu C-ABI library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "rsvio_gpu.h"

namespace rsvio {

void set_last_error(const std::string& msg);

struct HipError {
    hipError_t err;
    std::string where;
};

#define RSVIO_HIP(expr)                                                                    \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            throw ::rsvio::HipError{_e, std::string(#expr) + " @ " + __FILE__ + ":" +      \
                                            std::to_string(__LINE__)};                     \
    } while (0)

// A caller error: a bad argument or an entry point called in the wrong order (e.g. while a solve
// is in flight).  std::invalid_argument and this map to RSVIO_ERR_INVALID_ARG; other
// std::logic_errors (length_error, out_of_range from the STL) are internal failures.
struct CallOrderError : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};

// Run a C-ABI body, translating exceptions into status codes (never unwinds across the ABI).
template <class F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const HipError& e) {
        set_last_error(std::string("HIP error ") + hipGetErrorString(e.err) + " in " + e.where);
        return RSVIO_ERR_HIP;
    } catch (const std::bad_alloc&) {
        set_last_error("host allocation failed");
        return RSVIO_ERR_NOMEM;
    } catch (const std::invalid_argument& e) {  // bad arguments or call order (CallOrderError)
        set_last_error(e.what());
        return RSVIO_ERR_INVALID_ARG;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return RSVIO_ERR_INTERNAL;
    }
}

// Diagnostic phase stamps (make stamps -> lib/librsvio_gpu_stamps.so, tools/*_probe.py only):
// thread 0 of block b writes the shader clock into slot k of row b after draining its
// outstanding memory operations.  Compiled out of the product library.
#ifdef RSVIO_STAMPS
#define RSVIO_DBG_DECL static __device__ unsigned long long g_dbg[4096 * 32];
#define STAMP(k)                                                              \
    do {                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 4096) {                          \
            __builtin_amdgcn_s_waitcnt(0);                                    \
            g_dbg[blockIdx.x * 32 + (k)] = (unsigned long long)clock64();     \
        }                                                                     \
    } while (0)
#define RSVIO_DBG_READER(name)                                                             \
    extern "C" int name(unsigned long long* out, int n) {                                  \
        if (n > 4096 * 32) n = 4096 * 32;                                                  \
        return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), sizeof(unsigned long long) * n); \
    }
// wall-clock stamps (s_memrealtime, 100 MHz, one clock for every CU): slot k of row blockIdx,
// taken at issue (no drain), so kernel entry / exit spreads and boundary gaps can be read
#define RSVIO_RT_DECL static __device__ unsigned long long g_rt[4096 * 16];
#define RTSTAMP(k)                                                                              \
    do {                                                                                        \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                                              \
            g_rt[blockIdx.x * 16 + (k)] = (unsigned long long)__builtin_amdgcn_s_memrealtime();  \
    } while (0)
#define RSVIO_RT_READER(name)                                                              \
    extern "C" int name(unsigned long long* out, int n) {                                  \
        if (n > 4096 * 16) n = 4096 * 16;                                                  \
        return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt), sizeof(unsigned long long) * n); \
    }
#else
#define RSVIO_RT_DECL
#define RTSTAMP(k) \
    do {           \
    } while (0)
#define RSVIO_RT_READER(name)
#define RSVIO_DBG_DECL
#define STAMP(k) \
    do {         \
    } while (0)
#define RSVIO_DBG_READER(name)
#endif

// The tracker's device-resident output of the last COLLECTED frame (tracker.hip), for consumers
// on the device (pnp.hip): features (AoS rsvio_feature), fused undistorted coordinates, lengths.
// Complete when the view is taken (the collect waited for it); a frame submitted since writes the
// other output slot.
struct TrackerView {
    hipStream_t stream;
    const rsvio_feature* out[2];
    const float2* undist[2];   // null unless cameras are attached
    int n[2];                  // list lengths (n_l, n_r)
    int device;
};
TrackerView tracker_view(rsvio_tracker* t);

// Rust's saturating `as u32` (NaN and v <= 0 -> 0, v >= 2^32 -> u32::MAX) as selects, not
// branches: the range tests and the conversion are all evaluated, no exec-mask round trips
__device__ __forceinline__ uint32_t sat_u32(float v) {
    const uint32_t t = (uint32_t)fminf(fmaxf(v, 0.0f), 4294967040.0f);
    return v >= 4294967296.0f ? 0xFFFFFFFFu : (v > 0.0f ? t : 0u);
}

// Pyramid level geometry: level i = (w / 2^i) x (h / 2^i), packed back to back
// (feature_tracker.rs:215-216).
// Two 16-B loads of page-locked host memory at system scope (sc0 sc1: each request goes over PCIe
// to host memory, nothing served from a GPU cache), both in flight, complete on return -- the
// staging kernels' reads (ba_stage_in, rsvio_upload_async).  a and b must be 16-B aligned.
__device__ __forceinline__ void host_load2x16(const void* a, const void* b, uint4& va, uint4& vb) {
    __asm__ volatile(
        "global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
        "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(va), "=&v"(vb)
        : "v"(a), "v"(b)
        : "memory");
}

__host__ __device__ inline uint32_t level_w(uint32_t w, int i) { return w / (1u << i); }
__host__ __device__ inline uint32_t level_h(uint32_t h, int i) { return h / (1u << i); }
__host__ __device__ inline size_t level_offset(uint32_t w, uint32_t h, int level) {
    size_t off = 0;
    for (int i = 0; i < level; ++i) off += (size_t)level_w(w, i) * level_h(h, i);
    return off;
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    void alloc(size_t count) {
        release();
        if (count) RSVIO_HIP(hipMalloc(&p, count * sizeof(T)));
        n = count;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { release(); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

// Pinned host staging buffer
template <class T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    void alloc(size_t count, unsigned flags = hipHostMallocDefault) {
        release();
        if (count) RSVIO_HIP(hipHostMalloc(&p, count * sizeof(T), flags));
        n = count;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    ~HostBuf() { release(); }
};

}  // namespace rsvio
