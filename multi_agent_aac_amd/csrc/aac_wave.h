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

// sum over the lane's 16-lane DPP row (the first four steps of wsum): every lane of the row holds it
__device__ __forceinline__ float rsum16(float x) {
    DPP_STEP(x, 0xb1);
    DPP_STEP(x, 0x4e);
    DPP_STEP(x, 0x124);
    DPP_STEP(x, 0x128);
    return x;
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
// workgroup of 1024 threads; each thread owns 8 consecutive envs of a 8192-env tile (one pass at
// E <= 8192): local count, wave prefix by shuffles, wave totals through LDS.  An auto-reset launch
// then packs its workgroups with resetting envs instead of walking contiguous env ranges.
__device__ inline void compact_flags(const uint8_t *__restrict__ mask, int E, int32_t *rlist) {
    constexpr int PER = 8, TILE = 1024 * PER;
    __shared__ int wsum[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int base = 0;
    for (int t0 = 0; t0 < E; t0 += TILE) {
        const int e0 = t0 + threadIdx.x * PER;
        unsigned bits = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) bits |= (e0 + k < E && mask[e0 + k] != 0) ? (1u << k) : 0u;
        const int c = __popc(bits);
        int incl = c;     // inclusive prefix over the wave
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d, 64);
            if (lane >= d) incl += v;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        int off = base + incl - c, tot = 0;
        for (int k = 0; k < 16; ++k) {
            const int s = wsum[k];
            if (k < w) off += s;
            tot += s;
        }
        for (int k = 0; k < PER; ++k)
            if (bits & (1u << k)) rlist[1 + off++] = e0 + k;
        base += tot;
        __syncthreads();     // wsum is rewritten by the next tile
    }
    if (threadIdx.x == 0) rlist[0] = base;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations, not for its
// global loads in flight (__syncthreads waits for both), so loads issued before it keep going
// across the barrier.  Use where the barrier protects LDS data only.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

}  // namespace aacw
