// aac_wave.h -- wave64 reductions shared by the row kernels (one wave per row, lane = feature).
#pragma once
#include <hip/hip_runtime.h>

namespace aacw {

// wave-wide sum by DPP (rocPRIM's gfx9 pattern): xor 1, xor 2, row_ror 4, row_ror 8 leave each
// row's sum in every lane of the row, row_bcast 15 / 31 fold the rows into lane 63, which is
// broadcast with readlane.  No LDS round trips (ds_swizzle / bpermute) in the chain.
#define DPP_STEP(x, ctrl)                                                                                  \
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), ctrl, 0xf, 0xf, \
                                                               false))
__device__ __forceinline__ float wsum(float x) {
    DPP_STEP(x, 0xb1);   // quad_perm [1,0,3,2]
    DPP_STEP(x, 0x4e);   // quad_perm [2,3,0,1]
    DPP_STEP(x, 0x124);  // row_ror:4
    DPP_STEP(x, 0x128);  // row_ror:8
    DPP_STEP(x, 0x142);  // row_bcast:15
    DPP_STEP(x, 0x143);  // row_bcast:31
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}

// N independent wave sums with each DPP step applied to all N values before the next: the same
// per-value order as wsum (bit-identical results), with the step latencies overlapped
template <int N>
__device__ __forceinline__ void wsum_n(float (&v)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) DPP_STEP(v[k], 0xb1);
#pragma unroll
    for (int k = 0; k < N; ++k) DPP_STEP(v[k], 0x4e);
#pragma unroll
    for (int k = 0; k < N; ++k) DPP_STEP(v[k], 0x124);
#pragma unroll
    for (int k = 0; k < N; ++k) DPP_STEP(v[k], 0x128);
#pragma unroll
    for (int k = 0; k < N; ++k) DPP_STEP(v[k], 0x142);
#pragma unroll
    for (int k = 0; k < N; ++k) DPP_STEP(v[k], 0x143);
#pragma unroll
    for (int k = 0; k < N; ++k)
        v[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v[k]), 63));
}
#undef DPP_STEP

}  // namespace aacw
