// chain_probe.hip -- cycles per 52-term sequential f32 sum (LK's lane_chains) on gfx950, one wave:
// LDS-staged transposed chains (lane_chains<N>) vs readlane-operand chains, N = 1 and 3.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/chain_probe.hip -o tools/chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NP = 52, kLd = 68, kReps = 64;

template <int N>
__device__ __forceinline__ void lds_chains(const float (&v)[N], float (&out)[N], float* sh, int lane) {
#pragma unroll
    for (int i = 0; i < N; ++i) sh[i * kLd + lane] = v[i];
    __builtin_amdgcn_wave_barrier();
    const float4* row = reinterpret_cast<const float4*>(sh + (lane < N ? lane : 0) * kLd);
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) {
        const float4 x = row[q];
        acc = q == 0 ? x.x : acc + x.x;
        acc = acc + x.y;
        acc = acc + x.z;
        acc = acc + x.w;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), i));
}

template <int N>
__device__ __forceinline__ void rl_chains(const float (&v)[N], float (&out)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        float acc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[i]), 0));
#pragma unroll
        for (int k = 1; k < NP; ++k) acc = acc + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[i]), k));
        out[i] = acc;
    }
}

__global__ void probe(const float* in, float* o, long long* cyc) {
    __shared__ __attribute__((aligned(16))) float sh[3 * kLd];
    const int lane = threadIdx.x;
    float a = in[lane], b = in[lane + 64], c = in[lane + 128];
    long long t0, t1;
#define RUN(slot, N, ...)                                                \
    t0 = clock64();                                                       \
    _Pragma("unroll 1") for (int r = 0; r < kReps; ++r) {                 \
        const float v[N > 1 ? 3 : 1] = {a};                               \
        float s[N > 1 ? 3 : 1];                                           \
        (void)v;                                                          \
        __VA_ARGS__;                                                          \
        a = a * 0.5f + s[0];                                              \
    }                                                                     \
    t1 = clock64();                                                       \
    cyc[slot] = (t1 - t0) / kReps;
    RUN(0, 1, { const float w[1] = {a}; lds_chains<1>(w, s, sh, lane); });
    RUN(1, 3, { const float w[3] = {a, b * a, c * a}; lds_chains<3>(w, s, sh, lane); a = a + s[1] * s[2]; });
    RUN(2, 1, { const float w[1] = {a}; rl_chains<1>(w, s); });
    RUN(3, 3, { const float w[3] = {a, b * a, c * a}; rl_chains<3>(w, s); a = a + s[1] * s[2]; });
    o[lane] = a;
}

int main() {
    float* in;
    float* o;
    long long* cyc;
    hipMalloc(&in, 192 * sizeof(float));
    hipMalloc(&o, 64 * sizeof(float));
    hipMalloc(&cyc, 8 * sizeof(long long));
    float h[192];
    for (int i = 0; i < 192; ++i) h[i] = 1e-3f * (float)(i % 17);
    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    long long c[8] = {0};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, in, o, cyc);
        hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
    }
    printf("lds_chains<1> %lld cycles, lds_chains<3> %lld, readlane chain x1 %lld, readlane chains x3 %lld\n", c[0],
           c[1], c[2], c[3]);
    return 0;
}
