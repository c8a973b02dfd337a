// trig.hip -- parity entry points for the trackers' f32 sin/cos (trig.hpp, glibc sinf/cosf
// restated): a direct evaluation over a buffer and a per-chunk digest over any range of f32 bit
// patterns, so a test can compare the device's values with the host's libm over all 2^32 inputs
// without moving 32 GB (tests/test_trig_gpu.py against orc_libm_sincosf_digest).
#include "common.hpp"
#include "trig.hpp"

namespace rsvio {

// splitmix64 finaliser of (sin bits, cos bits) salted by the input's bit pattern; NaNs are
// canonical (their payload and sign are not part of the contract).
__device__ __forceinline__ uint64_t trig_digest_term(uint32_t u, float s, float c) {
    const uint32_t sb = (s != s) ? 0x7fc00000u : __float_as_uint(s);
    const uint32_t cb = (c != c) ? 0x7fc00000u : __float_as_uint(c);
    uint64_t z = (((uint64_t)sb << 32) | cb) + (uint64_t)u * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// One 256-thread block per 2^16 inputs (256 per thread); the block's sum is added to its chunk.
__global__ __launch_bounds__(256) void trig_digest_kernel(uint64_t first, uint64_t count, uint32_t chunk_log2,
                                                          unsigned long long* __restrict__ digests) {
    const uint64_t base = (uint64_t)blockIdx.x << 16;
    uint64_t acc = 0;
    for (int k = 0; k < 256; ++k) {
        const uint64_t off = base + (uint64_t)k * 256 + threadIdx.x;
        if (off < count) {
            const uint32_t u = (uint32_t)(first + off);
            float s, c;
            libm_trig::sincosf(__uint_as_float(u), &s, &c);
            acc += trig_digest_term(u, s, c);
        }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    __shared__ uint64_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t sum = part[0] + part[1] + part[2] + part[3];
        atomicAdd(&digests[base >> chunk_log2], (unsigned long long)sum);
    }
}

__global__ __launch_bounds__(256) void sincosf_kernel(const float* __restrict__ x, int n, float* __restrict__ s,
                                                      float* __restrict__ c) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) libm_trig::sincosf(x[i], &s[i], &c[i]);
}

}  // namespace rsvio

extern "C" {

int rsvio_sincosf(const float* x, size_t n, float* sin_out, float* cos_out) {
    if (n && (!x || !sin_out || !cos_out)) {
        rsvio::set_last_error("rsvio_sincosf: null buffer");
        return RSVIO_ERR_INVALID_ARG;
    }
    if (n > (size_t)INT32_MAX) {
        rsvio::set_last_error("rsvio_sincosf: too many values");
        return RSVIO_ERR_INVALID_ARG;
    }
    return rsvio::guarded([&] {
        if (n == 0) return (int)RSVIO_OK;
        rsvio::DevBuf<float> dx(n), ds(n), dc(n);
        RSVIO_HIP(hipMemcpy(dx.p, x, sizeof(float) * n, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(rsvio::sincosf_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, dx.p,
                           (int)n, ds.p, dc.p);
        RSVIO_HIP(hipGetLastError());
        RSVIO_HIP(hipMemcpy(sin_out, ds.p, sizeof(float) * n, hipMemcpyDeviceToHost));
        RSVIO_HIP(hipMemcpy(cos_out, dc.p, sizeof(float) * n, hipMemcpyDeviceToHost));
        return (int)RSVIO_OK;
    });
}

int rsvio_sincosf_digest(uint64_t first, uint64_t count, uint32_t chunk_log2, uint64_t* digests_out) {
    if (chunk_log2 < 16 || chunk_log2 > 32 || count == 0 || count > (1ull << 32) ||
        first + count > (1ull << 32) || (first & ((1ull << chunk_log2) - 1)) || !digests_out) {
        rsvio::set_last_error("rsvio_sincosf_digest: range must be chunk-aligned within 2^32, chunk 2^16..2^32");
        return RSVIO_ERR_INVALID_ARG;
    }
    return rsvio::guarded([&] {
        const uint64_t n_chunks = (count + (1ull << chunk_log2) - 1) >> chunk_log2;
        rsvio::DevBuf<unsigned long long> d(n_chunks);
        RSVIO_HIP(hipMemset(d.p, 0, sizeof(unsigned long long) * n_chunks));
        const uint64_t blocks = (count + 65535) >> 16;
        hipLaunchKernelGGL(rsvio::trig_digest_kernel, dim3((unsigned)blocks), dim3(256), 0, nullptr, first, count,
                           chunk_log2, d.p);
        RSVIO_HIP(hipGetLastError());
        RSVIO_HIP(hipMemcpy(digests_out, d.p, sizeof(uint64_t) * n_chunks, hipMemcpyDeviceToHost));
        return (int)RSVIO_OK;
    });
}

}  // extern "C"
