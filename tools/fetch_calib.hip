// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE for the access widths our kernels use
// (MI355X_MICROARCH.md, HBM section: FETCH_SIZE reads 1/2 of the bytes of wide 16-B-per-lane
// streaming reads on gfx950; other widths are uncalibrated).  Each kernel reads a fresh 64 MiB
// buffer (past every XCD's L2) once, with a known number of distinct 128-B lines:
//   wide16   16 B per lane, coalesced               -> 64 MiB of lines
//   byte1    1 B per lane, coalesced                -> 64 MiB of lines
//   u16_l128 one 2-B load per 128-B line            -> 64 MiB of lines
//   u16_l64  one 2-B load per 64-B half-line        -> 64 MiB of lines (two loads per line)
//   u8_gath  52 lanes x 4 bytes of an 11 x 11 patch at a random 16 B-aligned spot per wave
//            (the LK gather shape)                  -> lines counted on the host
// Run:  rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_calib   (prints the expected bytes)
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            return 1;                                                                \
        }                                                                            \
    } while (0)

constexpr size_t kBytes = size_t(64) << 20;

__global__ void wide16(const uint4* __restrict__ p, size_t n, unsigned* __restrict__ sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads; never true for the fill below
}

__global__ void byte1(const uint8_t* __restrict__ p, size_t n, unsigned* __restrict__ sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

__global__ void u16_stride(const uint8_t* __restrict__ p, size_t n_loads, size_t stride, unsigned* __restrict__ sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_loads; i += (size_t)gridDim.x * blockDim.x)
        acc += *reinterpret_cast<const uint16_t*>(p + i * stride);
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

// one wave per patch: lanes < 52 read 4 bytes (2 rows x 2 columns, like a bilinear sample)
// around a pattern point inside an 11 x 11 window of a 752-wide image
// `never` is a kernel argument (not a constant the compiler can bound the sum against), so the
// loads are kept: a constant test that the 4-byte sum provably never meets lets them be deleted
__global__ void u8_gath(const uint8_t* __restrict__ img, const int* __restrict__ base, unsigned* __restrict__ sink,
                        unsigned never) {
    const int lane = threadIdx.x;
    const int b = base[blockIdx.x];
    unsigned acc = 0;
    if (lane < 52) {
        const int dx = lane % 8, dy = lane / 8;  // 8 x 7 spread over the window
        const uint8_t* q = img + b + dy * 752 + dx;
        acc = q[0] + q[1] + q[752] + q[753];
    }
    if (acc == never) sink[0] = acc;
}

int main() {
    uint8_t* bufs[5];
    for (auto& b : bufs) {
        CK(hipMalloc(&b, kBytes));
        CK(hipMemset(b, 1, kBytes));
    }
    unsigned* sink;
    CK(hipMalloc(&sink, 4));
    // flush: stream 512 MiB through another buffer so no calibration buffer sits in the caches
    uint8_t* flush;
    CK(hipMalloc(&flush, size_t(512) << 20));
    CK(hipMemset(flush, 2, size_t(512) << 20));
    CK(hipDeviceSynchronize());
    const dim3 g(2048), b(256);
    hipLaunchKernelGGL(wide16, g, b, 0, 0, reinterpret_cast<const uint4*>(bufs[0]), kBytes / 16, sink);
    CK(hipMemset(flush, 3, size_t(512) << 20));
    hipLaunchKernelGGL(byte1, g, b, 0, 0, bufs[1], kBytes, sink);
    CK(hipMemset(flush, 4, size_t(512) << 20));
    hipLaunchKernelGGL(u16_stride, g, b, 0, 0, bufs[2], kBytes / 128, (size_t)128, sink);
    CK(hipMemset(flush, 5, size_t(512) << 20));
    hipLaunchKernelGGL(u16_stride, g, b, 0, 0, bufs[3], kBytes / 64, (size_t)64, sink);
    CK(hipMemset(flush, 6, size_t(512) << 20));
    // gathers: 100k patches at random spots of 480-row images laid over the buffer
    const int n_patch = 100000;
    std::vector<int> base(n_patch);
    std::set<size_t> lines;
    srand(7);
    for (int i = 0; i < n_patch; ++i) {
        const size_t img0 = (size_t)(rand() % 180) * 752 * 480;
        const int x = 8 + rand() % 700, y = 8 + rand() % 460;
        base[i] = (int)(img0 + (size_t)y * 752 + x);
        for (int lane = 0; lane < 52; ++lane) {
            const size_t a = base[i] + (lane / 8) * 752 + (lane % 8);
            lines.insert(a / 128);
            lines.insert((a + 1) / 128);
            lines.insert((a + 752) / 128);
            lines.insert((a + 753) / 128);
        }
    }
    int* d_base;
    CK(hipMalloc(&d_base, n_patch * sizeof(int)));
    CK(hipMemcpy(d_base, base.data(), n_patch * sizeof(int), hipMemcpyHostToDevice));
    CK(hipMemset(flush, 7, size_t(512) << 20));
    hipLaunchKernelGGL(u8_gath, dim3(n_patch), dim3(64), 0, 0, bufs[4], d_base, sink, 0xFFFFFFFFu);
    CK(hipDeviceSynchronize());
    printf("expected line bytes: wide16 %zu byte1 %zu u16_l128 %zu u16_l64 %zu u8_gath %zu (distinct 128-B lines x 128)\n",
           kBytes, kBytes, kBytes, kBytes, lines.size() * 128);
    return 0;
}
