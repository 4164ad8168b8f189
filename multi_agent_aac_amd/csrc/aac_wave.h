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

// ordered list of the envs whose flag is set: rlist = [count, e...] (ascending).  Called by ONE
// workgroup of 1024 threads (a ballot + wave prefix per 1024 envs), so that an auto-reset launch
// can pack its workgroups with resetting envs instead of walking contiguous env ranges.
__device__ inline void compact_flags(const uint8_t *__restrict__ mask, int E, int32_t *rlist) {
    __shared__ int wsum[16];
    __shared__ int base_s;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < E; c0 += 1024) {
        const int e = c0 + threadIdx.x;
        const bool a = e < E && mask[e] != 0;
        const unsigned long long b = __ballot(a);
        const int pre = __popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(b);
        __syncthreads();
        int off = base_s;
        for (int k = 0; k < w; ++k) off += wsum[k];
        if (a) rlist[1 + off + pre] = e;
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int k = 0; k < 16; ++k) tot += wsum[k];
            base_s += tot;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) rlist[0] = base_s;
}

}  // namespace aacw
