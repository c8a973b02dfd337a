// mfma_probe.hip -- one-wave latency / throughput of the operations K5's factorisation is made of
// (gfx950, shader-clock cycles): v_mfma_f64_16x16x4f64 dependent and 4 independent chains, a
// dependent f64 FMA, rcp_f64 (v_rcp_f64 + folded Newton), a dependent LDS load chain, and a
// 4-wave workgroup barrier round.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int kN = 64;

__global__ void probe(const double* in, double* out, long long* cyc) {
    __shared__ double lds[4096];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 4096; i += blockDim.x) lds[i] = (double)((i * 7 + 1) & 4095);
    __syncthreads();
    const double a = in[lane], b = in[64 + lane];
    if (wave == 0) {
        // 1. dependent MFMA chain
        dbl4 c = {in[0], in[1], in[2], in[3]};
        __builtin_amdgcn_sched_barrier(0);
        long long t0 = clock64();
#pragma unroll
        for (int i = 0; i < kN; ++i) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
        __asm__ volatile("s_nop 0" ::"v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_sched_barrier(0);
        long long t1 = clock64();
        // 2. four independent chains
        dbl4 d0 = c, d1 = c + 1.0, d2 = c + 2.0, d3 = c + 3.0;
        __builtin_amdgcn_sched_barrier(0);
        long long t2 = clock64();
#pragma unroll
        for (int i = 0; i < kN / 4; ++i) {
            d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d1, 0, 0, 0);
            d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d2, 0, 0, 0);
            d3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d3, 0, 0, 0);
        }
        __asm__ volatile("s_nop 0" ::"v"(d0[0]), "v"(d1[0]), "v"(d2[0]), "v"(d3[0]));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_sched_barrier(0);
        long long t3 = clock64();
        // 3. dependent f64 FMA
        double x = a;
        __builtin_amdgcn_sched_barrier(0);
        long long t4 = clock64();
#pragma unroll
        for (int i = 0; i < 256; ++i) x = fma(x, b, 0.5);
        __asm__ volatile("s_nop 0" ::"v"(x));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_sched_barrier(0);
        long long t5 = clock64();
        // 4. dependent rcp_f64 (+ folded Newton, as se3.hpp)
        double y = a + 2.0;
        __builtin_amdgcn_sched_barrier(0);
        long long t6 = clock64();
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            const double r = __builtin_amdgcn_rcp(y);
            const double e = fma(-y, r, 1.0);
            y = fma(r, fma(e, e, e), r) + 1.5;
        }
        __asm__ volatile("s_nop 0" ::"v"(y));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_sched_barrier(0);
        long long t7 = clock64();
        // 5. dependent LDS load chain (address from the loaded value)
        int idx = lane;
        __builtin_amdgcn_sched_barrier(0);
        long long t8 = clock64();
#pragma unroll
        for (int i = 0; i < 64; ++i) idx = (int)lds[idx] & 4095;
        __asm__ volatile("s_nop 0" ::"v"(idx));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_sched_barrier(0);
        long long t9 = clock64();
        // 6. 64 broadcast ds_read_b64 issued back to back, then one wait
        double s = 0.0;
        __builtin_amdgcn_sched_barrier(0);
        long long t10 = clock64();
        double v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = lds[(idx & 7) + 37 * i];
#pragma unroll
        for (int i = 0; i < 32; ++i) s += v[i];
        __asm__ volatile("s_nop 0" ::"v"(s));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_sched_barrier(0);
        long long t11 = clock64();
        out[lane] = c[0] + d0[0] + d1[1] + d2[2] + d3[3] + x + y + idx + s;
        if (lane == 0) {
            cyc[0] = t1 - t0;
            cyc[1] = t3 - t2;
            cyc[2] = t5 - t4;
            cyc[3] = t7 - t6;
            cyc[4] = t9 - t8;
            cyc[5] = t11 - t10;
        }
    }
    // 7. barrier rounds with all 4 waves
    __syncthreads();
    long long tb0 = clock64();
    for (int i = 0; i < 64; ++i) __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
        long long tb1 = clock64();
    if (tid == 0) cyc[6] = tb1 - tb0;
}

int main() {
    double *in, *out;
    long long* cyc;
    hipMalloc(&in, 256 * sizeof(double));
    hipMalloc(&out, 256 * sizeof(double));
    hipMalloc(&cyc, 16 * sizeof(long long));
    double h[256];
    for (int i = 0; i < 256; ++i) h[i] = 1.0 + 1e-3 * i;
    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    long long c[16];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, in, out, cyc);
        hipDeviceSynchronize();
        hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
    }
    printf("mfma_f64_16x16x4 dependent      %7.1f cycles/op\n", (double)c[0] / kN);
    printf("mfma_f64_16x16x4 4 indep chains %7.1f cycles/op\n", (double)c[1] / kN);
    printf("fma_f64 dependent               %7.1f cycles/op\n", (double)c[2] / 256);
    printf("rcp_f64 + Newton + add dep.     %7.1f cycles/op\n", (double)c[3] / 64);
    printf("ds_read_b64 dependent chain     %7.1f cycles/op\n", (double)c[4] / 64);
    printf("32 ds_read_b64 + sum            %7.1f cycles total\n", (double)c[5]);
    printf("__syncthreads (4 waves)         %7.1f cycles/op\n", (double)c[6] / 64);
    return 0;
}
