// lat_probe.hip -- dependent-issue latency of the f64 operations on K5's pivot chain (gfx950),
// one wave, shader-clock cycles per operation of a 256-long dependent chain.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o tools/lat_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 256;

__device__ __forceinline__ double rl64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// straight-line code vs the same work in a rolled loop: 4096 FMAs on 8 independent chains
// (~32 KB of code unrolled) -- what a cold instruction cache costs a long unrolled kernel
__global__ void straight(const double* c, double* out, long long* cyc) {
    const int lane = threadIdx.x;
    double z[8];
    const double a = c[0], b = c[1];
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = c[2] + lane + k;
    const long long t0 = clock64();
#pragma unroll
    for (int i = 0; i < 512; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = fma(z[k], a, b + (double)(i & 3));
#pragma unroll
    for (int k = 0; k < 8; ++k) __asm__ volatile("" ::"v"(z[k]));
    const long long t1 = clock64();
    double acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += z[k];
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}
__global__ void rolled(const double* c, double* out, long long* cyc) {
    const int lane = threadIdx.x;
    double z[8];
    const double a = c[0], b = c[1];
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = c[2] + lane + k;
    const long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < 128; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 8; ++k) z[k] = fma(z[k], a, b + (double)j);
#pragma unroll
    for (int k = 0; k < 8; ++k) __asm__ volatile("" ::"v"(z[k]));
    const long long t1 = clock64();
    double acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += z[k];
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}

__global__ void chains(double x0, double* out, long long* cyc) {
    const int lane = threadIdx.x;
    double x = x0 + lane * 1e-3;
    long long t0, t1;
    // 1. dependent v_fma_f64
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) x = fma(x, 0.9999999, 1e-9);
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[0] = t1 - t0;
    // 2. dependent v_rcp_f64
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) x = __builtin_amdgcn_rcp(x);
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[1] = t1 - t0;
    // 3. dependent readlane pair -> f64 add (the pivot broadcast)
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) x = x + rl64(x, i & 63);
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[2] = t1 - t0;
    // 4. dependent v_mul_f64
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) x = x * 1.0000001;
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[3] = t1 - t0;
    // 5. dependent f32 fma (reference)
    float y = (float)x;
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) y = fmaf(y, 0.9999f, 1e-6f);
    __asm__ volatile("" ::"v"(y));
    t1 = clock64();
    cyc[4] = t1 - t0;
    // 6. independent f64 fma issue (8 chains interleaved)
    double z[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = x + k;
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN / 8; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = fma(z[k], 0.9999999, 1e-9);
#pragma unroll
    for (int k = 0; k < 8; ++k) __asm__ volatile("" ::"v"(z[k]));
    t1 = clock64();
    cyc[5] = t1 - t0;
    // 7. dependent ds_write -> ds_read round trip through LDS
    __shared__ double sh[64];
    t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < kN / 8; ++i) {
        sh[lane] = x;
        __builtin_amdgcn_wave_barrier();
        x = sh[(lane + 1) & 63] + 1.0;
    }
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[6] = (t1 - t0) * 8;
    double acc = x + y;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += z[k];
    out[lane] = acc;
}


// f32 operations on LK's per-iteration chain (lk_track.hip), compiled with the library's flags
__global__ void chains32(float x0, const unsigned char* img, float* out, long long* cyc) {
    const int lane = threadIdx.x;
    float x = x0 + lane * 1e-3f;
    long long t0, t1;
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) x = x + 1.0001f;
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[0] = t1 - t0;
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN / 4; ++i) x = 3.0f / x;
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[1] = (t1 - t0) * 4;
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN / 4; ++i) x = sqrtf(x + 2.0f);
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[2] = (t1 - t0) * 4;
    __shared__ float sh[64 * 4];
    t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < kN / 8; ++i) {
        sh[lane] = x;
        __builtin_amdgcn_wave_barrier();
        const float4 q = reinterpret_cast<const float4*>(sh)[(lane + 1) & 15];
        __builtin_amdgcn_wave_barrier();
        x = q.x + 1.0f;
    }
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[3] = (t1 - t0) * 8;
    // dependent u8 gather chain in a 64 KB image (L2/L1 resident after the first pass)
    unsigned idx = lane * 977u;
    for (int i = 0; i < 64; ++i) idx = (idx * 131u + img[idx & 65535u]) & 65535u;
    t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < kN / 8; ++i) idx = (idx * 131u + img[idx & 65535u]) & 65535u;
    t1 = clock64();
    cyc[4] = (t1 - t0) * 8;
    // dependent readlane -> v_add_f32 (SGPR operand)
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) x = x + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), i & 63));
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[5] = t1 - t0;
    // dependent f32 add with the other operand from a readlane issued ahead (independent)
    float yv = x * 0.5f;
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) x = x + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yv), i & 63));
    __asm__ volatile("" ::"v"(x));
    t1 = clock64();
    cyc[6] = t1 - t0;
    // dependent f64 add
    double d = x;
    t0 = clock64();
#pragma unroll
    for (int i = 0; i < kN; ++i) d = d + 1.0000001;
    __asm__ volatile("" ::"v"(d));
    t1 = clock64();
    cyc[7] = t1 - t0;
    out[lane] = x + (float)idx + (float)d;
}

int main() {
    double* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, 8 * sizeof(long long));
    long long h[8];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(chains, dim3(1), dim3(64), 0, 0, 1.5, out, cyc);
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    }
    double hc[3] = {0.9999999, 1e-9, 1.5};
    double* dc;
    hipMalloc(&dc, sizeof hc);
    hipMemcpy(dc, hc, sizeof hc, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        long long a = 0, b = 0;
        hipLaunchKernelGGL(straight, dim3(1), dim3(64), 0, 0, dc, out, cyc);
        hipMemcpy(&a, cyc, sizeof a, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(rolled, dim3(1), dim3(64), 0, 0, dc, out, cyc);
        hipMemcpy(&b, cyc, sizeof b, hipMemcpyDeviceToHost);
        printf("4096 f64 FMAs: straight-line %lld cycles, rolled loop %lld cycles\n", a, b);
    }
    const char* names[7] = {"fma_f64 dep", "rcp_f64 dep", "readlane2+add_f64 dep", "mul_f64 dep", "fma_f32 dep",
                            "fma_f64 indep (issue)", "ds_write->ds_read dep"};
    for (int i = 0; i < 7; ++i) printf("%-24s %6.1f cycles/op\n", names[i], (double)h[i] / kN);
    unsigned char* img;
    hipMalloc(&img, 65536);
    hipMemset(img, 7, 65536);
    float* o32;
    hipMalloc(&o32, 64 * sizeof(float));
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(chains32, dim3(1), dim3(64), 0, 0, 1.5f, img, o32, cyc);
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    }
    const char* n32[8] = {"add_f32 dep", "div_f32 (IEEE) dep", "sqrt_f32 (IEEE) dep", "ds_write->ds_read_b128 dep",
                          "u8 global gather dep (L1/L2)", "readlane->add_f32 dep", "add_f32 dep, readlane operand",
                          "add_f64 dep"};
    for (int i = 0; i < 8; ++i) printf("%-30s %6.1f cycles/op\n", n32[i], (double)h[i] / kN);
    return 0;
}
