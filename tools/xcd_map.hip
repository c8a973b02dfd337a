// GPU box: which XCD (and CU) the workgroups of a CU-masked stream run on, for the bench's tracker
// / BA partitions (bench.py cu_partition: "block" = CUs 0..63 of the mask, "stride" = every 4th).
// Reads the hardware XCC_ID and HW_ID registers per workgroup (s_getreg; vector stores only) and
// prints, per mask, the XCDs used with their workgroup counts and the XCD of workgroups 0..15.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/xcd_map tools/xcd_map.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

__global__ void where(unsigned* out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
        out[2 * blockIdx.x] = xcc & 0xF;
        out[2 * blockIdx.x + 1] = hw;
    }
    // keep the workgroup resident for a while so the dispatcher spreads the grid
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 200) {
    }
}

static void run(const char* name, const std::vector<uint32_t>& mask, int n_wg) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    unsigned* d;
    CK(hipMalloc(&d, sizeof(unsigned) * 2 * n_wg));
    CK(hipMemsetAsync(d, 0xFF, sizeof(unsigned) * 2 * n_wg, s));
    hipLaunchKernelGGL(where, dim3(n_wg), dim3(64), 0, s, d);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(s));
    std::vector<unsigned> h(2 * n_wg);
    CK(hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * n_wg, hipMemcpyDeviceToHost));
    int per_xcc[16] = {0};
    std::vector<int> cus[16];
    for (int i = 0; i < n_wg; ++i) {
        const unsigned x = h[2 * i];
        if (x < 16) {
            ++per_xcc[x];
            const unsigned hw = h[2 * i + 1];
            const int cu = (int)((hw >> 8) & 0xF), sh = (int)((hw >> 12) & 1), se = (int)((hw >> 13) & 7);
            const int key = se * 32 + sh * 16 + cu;
            bool seen = false;
            for (int c : cus[x]) seen = seen || c == key;
            if (!seen) cus[x].push_back(key);
        }
    }
    std::printf("%-8s", name);
    for (int x = 0; x < 16; ++x)
        if (per_xcc[x]) std::printf("  xcd%d: %d wg on %zu CUs", x, per_xcc[x], cus[x].size());
    std::printf("\n         first workgroups' XCDs:");
    for (int i = 0; i < 16; ++i) std::printf(" %u", h[2 * i]);
    std::printf("\n");
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
}

int main() {
    int n_cu = 0;
    CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
    const int words = (n_cu + 31) / 32;
    std::printf("CUs %d\n", n_cu);
    auto mk = [&](auto pred) {
        std::vector<uint32_t> m(words, 0u);
        for (int i = 0; i < n_cu; ++i)
            if (pred(i)) m[i / 32] |= 1u << (i % 32);
        return m;
    };
    const int n_wg = 4096;
    run("all", mk([](int) { return true; }), n_wg);
    run("block", mk([](int i) { return i < 64; }), n_wg);
    run("stride", mk([](int i) { return i % 4 == 0; }), n_wg);
    run("ba_blk", mk([](int i) { return i >= 64; }), n_wg);
    run("ba_str", mk([](int i) { return i % 4 != 0; }), n_wg);
    run("mod8_01", mk([](int i) { return i % 8 < 2; }), n_wg);
    return 0;
}
