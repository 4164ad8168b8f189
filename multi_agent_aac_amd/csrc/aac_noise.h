// aac_noise.h -- the exploration-noise pieces shared by the act-path kernels (aac_learn.hip:
// noise_kernel, actor_out_noise_kernel; aac_gru.hip: gru_actor_fwd_kernel): the per-launch RNG epoch
// and the per-row Box-Muller noise of choose_action (ATT/maddpg:476-500, WGRU/maddpg:336-428).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace aacn {

// SplitMix64 finaliser (the same function as aac_geom.h / aac_learn.hip's mix64)
__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// A launch-wide counter advanced by the launch itself (no one-thread follow-up kernel): word =
// epoch (low 32 bits) | arrivals (high 32 bits, 0 between launches).  Thread 0 of every workgroup
// takes the epoch with one atomic add to the arrivals; the last workgroup to arrive has seen every
// other one take it and stores epoch + 1 with arrivals 0.  Returns the epoch to the whole group.
__device__ inline uint64_t take_epoch(uint64_t *word) {
    __shared__ uint64_t ep;
    if (threadIdx.x == 0) {
        const uint64_t old = atomicAdd(reinterpret_cast<unsigned long long *>(word), 1ull << 32);
        ep = old & 0xffffffffull;
        if ((old >> 32) == (uint64_t)(gridDim.x * gridDim.y * gridDim.z) - 1)
            // low 32 bits only: the arrival field must restart at 0 even when the epoch wraps
            atomicExch(reinterpret_cast<unsigned long long *>(word), (unsigned long long)((ep + 1) & 0xffffffffull));
    }
    __syncthreads();
    return ep;
}

// The same counter with the arrival moved to the end of the launch, off the start of its chain:
// every thread reads the epoch with one load (the word holds epoch | 0 between launches), and
// end_epoch -- reached by every workgroup after its last use of the epoch -- counts the arrival;
// the last workgroup stores epoch + 1.  Every workgroup has read the epoch before it arrives, so
// none reads the advanced word.  The counter's sequence is take_epoch's.
__device__ inline uint64_t read_epoch(const uint64_t *word) {
    return __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffull;
}

__device__ inline void end_epoch(uint64_t *word, uint64_t ep) {
    __syncthreads();      // (its fence completes this workgroup's reads of the word)
    if (threadIdx.x == 0) {
        const uint64_t old = atomicAdd(reinterpret_cast<unsigned long long *>(word), 1ull << 32);
        if ((old >> 32) == (uint64_t)(gridDim.x * gridDim.y * gridDim.z) - 1)
            atomicExch(reinterpret_cast<unsigned long long *>(word), (unsigned long long)((ep + 1) & 0xffffffffull));
    }
}

// the exploration noise of agent row `row` (env row / N): var from the env's episode (linear
// schedule to eps_end, then noise_end), Box-Muller pair from the hash of (seed, epoch, row)
__device__ __forceinline__ void row_noise(int64_t row, int N, const int32_t *episode, int eps_end, float noise_start,
                                          float noise_end, uint64_t seed, uint64_t ctr, float &n0, float &n1) {
    const int e = (int)(row / N);
    const int ep = episode ? episode[e] : 1;
    double var;
    if (ep <= eps_end) {
        const double slope = ((double)noise_end - (double)noise_start) / (double)(eps_end - 1);
        var = (double)noise_start + slope * (double)(ep - 1);
    } else {
        var = (double)noise_end;
    }
    const uint64_t h1 = mix64(mix64(mix64(seed) ^ ctr) ^ (uint64_t)(2 * row));
    const uint64_t h2 = mix64(h1 ^ 0xD1B54A32D192ED03ull);
    const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);   // (0, 1]
    const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
    const double rr = sqrt(-2.0 * log(u1));
    const double z0 = rr * cos(6.283185307179586 * u2), z1 = rr * sin(6.283185307179586 * u2);
    n0 = (float)(z0 * var);
    n1 = (float)(z1 * var);
}

}  // namespace aacn
