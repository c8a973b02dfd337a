// wave.hpp -- cross-lane f64 moves and deterministic wave reductions for gfx950 (wave64).
#pragma once
#include <hip/hip_runtime.h>

#include "se3.hpp"

namespace rsvio {

// 64-bit cross-lane moves built from 32-bit lane ops
__device__ __forceinline__ void swap32_f64(double& x, double& y) {  // v_permlane32_swap
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double(hi[0], lo[0]);
    y = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ void swap16_f64(double& x, double& y) {  // v_permlane16_swap
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(y), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(y), false, false);
    x = __hiloint2double(hi[0], lo[0]);
    y = __hiloint2double(hi[1], lo[1]);
}

// Deterministic reduce-scatter of N = 16 M per-lane values over the wave.  Afterwards lane l
// holds the wave totals of values M (l >> 2) + j, j < M, in v[0..M) (the 4 lanes of a quad hold
// identical bits).  Fixed pairings (run-to-run identical): lanes l / l+32 (permlane32 swap),
// rows 0/1 and 2/3 (permlane16 swap), l / l^8 inside a row (row_ror 8), the half-row mirror,
// then butterflies over quad xor 2 and xor 1.  ~4 instructions per value at the first level and
// geometrically fewer after, instead of ~12 per value for separate wave sums.
template <int M>
__device__ __forceinline__ void wave_reduce_scatter(double (&v)[16 * M], int lane) {
#pragma unroll
    for (int i = 0; i < 8 * M; ++i) {
        swap32_f64(v[i], v[8 * M + i]);
        v[i] = v[i] + v[8 * M + i];  // lanes 0-31: value i, lanes 32-63: value 8M + i
    }
#pragma unroll
    for (int i = 0; i < 4 * M; ++i) {
        swap16_f64(v[i], v[4 * M + i]);
        v[i] = v[i] + v[4 * M + i];
    }
    const bool b3 = lane & 8, b2 = lane & 4;
#pragma unroll
    for (int i = 0; i < 2 * M; ++i) {
        const double keep = b3 ? v[2 * M + i] : v[i], send = b3 ? v[i] : v[2 * M + i];
        v[i] = keep + dpp64<0x128>(send);  // row_ror:8 -> lane l^8
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const double keep = b2 ? v[M + i] : v[i], send = b2 ? v[i] : v[M + i];
        v[i] = keep + dpp64<0x141>(send);  // row_half_mirror: l <-> 7-l in each half-row
    }
#pragma unroll
    for (int i = 0; i < M; ++i) v[i] = v[i] + dpp64<0x4E>(v[i]);  // quad_perm [2,3,0,1]
#pragma unroll
    for (int i = 0; i < M; ++i) v[i] = v[i] + dpp64<0xB1>(v[i]);  // quad_perm [1,0,3,2]
}

}  // namespace rsvio
