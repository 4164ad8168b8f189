// aac_mpe.hip -- batched MPE simple_spread (include/aac_mpe.h).
//
// One thread per environment, the N <= 8 agents and L <= 8 landmarks of its world in registers
// (loops unrolled to the compile-time maxima, guarded by the runtime N / L).  fp64 throughout, in
// the element order of the reference's numpy (no fma contraction: -ffp-contract=off):
//   F_i  = float(u_i * 5)                                         (environment.py:193-197)
//   for a < b: d = p_a - p_b, |d| = sqrt(d0^2 + d1^2),
//              pen = logaddexp(0, -(|d| - 0.3) / 1e-3) * 1e-3,  f = 1e2 d / |d| * pen
//              F_a = f + F_a,  F_b = -f + F_b                     (core.py:141-153, 172-195)
//   v = v * 0.75;  v += (F / 1) * 0.1;  p += v * 0.1               (core.py:156-166)
//   (with one agent no contact term promotes F to float64, so that product is float32 as numpy's)
//   rew_i = 0 - sum_l min_a |p_a - l| - #{a : |p_a - p_i| < 0.3}   (simple_spread.py:73-82)
// Memory-bound: 80 B of state per agent read and written, obs 4 (4 + 2L + 4(N-1)) B written.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/aac_mpe.h"

namespace {

thread_local std::string m_err;

int mfail(const std::string &m) {
    m_err = m;
    return -1;
}

constexpr int NM = AAC_MPE_MAX_AGENTS, LM = AAC_MPE_MAX_LANDMARKS;
constexpr double SIZE2 = 0.15 + 0.15, K = 1e-3, CF = 1e2, DT = 0.1, DAMP = 0.25;

// numpy's logaddexp(0, x) (npy_logaddexp): equal -> 0 + ln2; else max + log1p(exp(-|diff|))
__device__ __forceinline__ double logaddexp0(double x) {
    if (x == 0.0) return 0.6931471805599453;
    const double tmp = 0.0 - x;
    if (tmp > 0) return 0.0 + log1p(exp(-tmp));
    return x + log1p(exp(tmp));
}

__device__ __forceinline__ double dnorm(double x, double y) { return sqrt(x * x + y * y); }

__device__ __forceinline__ void observe_env(const double (&px)[NM], const double (&py)[NM], const double (&vx)[NM],
                            const double (&vy)[NM], const double (&lx)[LM], const double (&ly)[LM], int N, int L,
                            float *obs, double *rew) {
    const int W = 4 + 2 * L + 4 * (N - 1);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        if (i >= N) continue;
        float *o = obs + (size_t)i * W;
        o[0] = (float)vx[i];
        o[1] = (float)vy[i];
        o[2] = (float)px[i];
        o[3] = (float)py[i];
        int c = 4;
#pragma unroll
        for (int j = 0; j < LM; ++j) {
            if (j >= L) continue;
            o[c++] = (float)(lx[j] - px[i]);
            o[c++] = (float)(ly[j] - py[i]);
        }
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            if (j >= N || j == i) continue;
            o[c++] = (float)(px[j] - px[i]);
            o[c++] = (float)(py[j] - py[i]);
        }
        for (int j = 0; j < 2 * (N - 1); ++j) o[c++] = 0.0f;      // silent agents' comm
        double r = 0.0;
#pragma unroll
        for (int l = 0; l < LM; ++l) {
            if (l >= L) continue;
            double mn = INFINITY;
#pragma unroll
            for (int a = 0; a < NM; ++a) {
                if (a >= N) continue;
                const double d = dnorm(px[a] - lx[l], py[a] - ly[l]);
                mn = d < mn ? d : mn;                 // python min(): first minimum
            }
            r = r - mn;
        }
#pragma unroll
        for (int a = 0; a < NM; ++a) {
            if (a >= N) continue;
            if (dnorm(px[a] - px[i], py[a] - py[i]) < SIZE2) r = r - 1.0;   // self included
        }
        rew[i] = r;
    }
}

__device__ __forceinline__ void load_env(const double *pos, const double *vel, const double *lmk, int e, int N, int L,
                                         double (&px)[NM], double (&py)[NM], double (&vx)[NM], double (&vy)[NM],
                                         double (&lx)[LM], double (&ly)[LM]) {
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        if (i >= N) continue;
        const size_t o = ((size_t)e * N + i) * 2;
        px[i] = pos[o];
        py[i] = pos[o + 1];
        vx[i] = vel[o];
        vy[i] = vel[o + 1];
    }
#pragma unroll
    for (int j = 0; j < LM; ++j) {
        if (j >= L) continue;
        const size_t o = ((size_t)e * L + j) * 2;
        lx[j] = lmk[o];
        ly[j] = lmk[o + 1];
    }
}

__global__ void __launch_bounds__(128) mpe_step_kernel(double *pos, double *vel, const double *lmk, const float *act, int E, int N, int L,
                                float *obs, double *rew) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    double px[NM], py[NM], vx[NM], vy[NM], lx[LM], ly[LM], fx[NM], fy[NM];
    load_env(pos, vel, lmk, e, N, L, px, py, vx, vy, lx, ly);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        if (i >= N) continue;
        const size_t o = ((size_t)e * N + i) * 2;
        fx[i] = (double)(act[o] * 5.0f);
        fy[i] = (double)(act[o + 1] * 5.0f);
    }
#pragma unroll
    for (int a = 0; a < NM; ++a) {
#pragma unroll
        for (int b = a + 1; b < NM; ++b) {
            if (b >= N) continue;
            const double dx = px[a] - px[b], dy = py[a] - py[b];
            const double dist = dnorm(dx, dy);
            const double pen = logaddexp0(-(dist - SIZE2) / K) * K;
            const double gx = CF * dx / dist * pen, gy = CF * dy / dist * pen;
            fx[a] = gx + fx[a];
            fy[a] = gy + fy[a];
            fx[b] = -gx + fx[b];
            fy[b] = -gy + fy[b];
        }
    }
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        if (i >= N) continue;
        vx[i] = vx[i] * (1.0 - DAMP);
        vy[i] = vy[i] * (1.0 - DAMP);
        if (N > 1) {
            vx[i] += (fx[i] / 1.0) * DT;
            vy[i] += (fy[i] / 1.0) * DT;
        } else {   // no contact term ever promoted the float32 force: numpy's (F / 1.0) * dt is float32
            vx[i] += (double)(((float)fx[i] / 1.0f) * 0.1f);
            vy[i] += (double)(((float)fy[i] / 1.0f) * 0.1f);
        }
        px[i] += vx[i] * DT;
        py[i] += vy[i] * DT;
        const size_t o = ((size_t)e * N + i) * 2;
        pos[o] = px[i];
        pos[o + 1] = py[i];
        vel[o] = vx[i];
        vel[o + 1] = vy[i];
    }
    const int W = 4 + 2 * L + 4 * (N - 1);
    observe_env(px, py, vx, vy, lx, ly, N, L, obs + (size_t)e * N * W, rew + (size_t)e * N);
}

__global__ void __launch_bounds__(128) mpe_observe_kernel(const double *pos, const double *vel, const double *lmk, int E, int N, int L,
                                   float *obs, double *rew) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    double px[NM], py[NM], vx[NM], vy[NM], lx[LM], ly[LM];
    load_env(pos, vel, lmk, e, N, L, px, py, vx, vy, lx, ly);
    const int W = 4 + 2 * L + 4 * (N - 1);
    observe_env(px, py, vx, vy, lx, ly, N, L, obs + (size_t)e * N * W, rew + (size_t)e * N);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void mpe_reset_kernel(double *pos, double *vel, double *lmk, int E, int N, int L, const uint8_t *mask,
                                 uint64_t seed, const uint64_t *counter) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E || (mask && !mask[e])) return;
    const uint64_t base = mix64(mix64(seed) ^ *counter) ^ ((uint64_t)e << 16);
    auto uni = [&](int k) {     // uniform [-1, 1) with 53 random bits
        return -1.0 + 2.0 * ((double)(mix64(base + (uint64_t)k) >> 11) * (1.0 / 9007199254740992.0));
    };
    for (int i = 0; i < N; ++i) {
        const size_t o = ((size_t)e * N + i) * 2;
        pos[o] = uni(2 * i);
        pos[o + 1] = uni(2 * i + 1);
        vel[o] = 0.0;
        vel[o + 1] = 0.0;
    }
    for (int j = 0; j < L; ++j) {
        const size_t o = ((size_t)e * L + j) * 2;
        lmk[o] = uni(2 * N + 2 * j);
        lmk[o + 1] = uni(2 * N + 2 * j + 1);
    }
}

__global__ void mpe_counter_kernel(uint64_t *c) { *c += 1; }

int check(int E, int N, int L) {
    if (E <= 0) return mfail("mpe: E > 0");
    if (N < 1 || N > NM) return mfail("mpe: 1 <= N <= AAC_MPE_MAX_AGENTS");
    if (L < 0 || L > LM) return mfail("mpe: 0 <= L <= AAC_MPE_MAX_LANDMARKS");
    return 0;
}

}  // namespace

extern "C" {

const char *aac_mpe_last_error(void) { return m_err.c_str(); }

int aac_mpe_step(double *pos, double *vel, const double *lmk, const float *act, int32_t E, int32_t N, int32_t L,
                 float *obs, double *rew, void *stream) {
    if (check(E, N, L)) return -1;
    hipLaunchKernelGGL(mpe_step_kernel, dim3((E + 127) / 128), dim3(128), 0, (hipStream_t)stream, pos, vel, lmk, act, E,
                       N, L, obs, rew);
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? 0 : mfail(std::string("mpe_step: ") + hipGetErrorString(err));
}

int aac_mpe_observe(const double *pos, const double *vel, const double *lmk, int32_t E, int32_t N, int32_t L,
                    float *obs, double *rew, void *stream) {
    if (check(E, N, L)) return -1;
    hipLaunchKernelGGL(mpe_observe_kernel, dim3((E + 127) / 128), dim3(128), 0, (hipStream_t)stream, pos, vel, lmk, E,
                       N, L, obs, rew);
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? 0 : mfail(std::string("mpe_observe: ") + hipGetErrorString(err));
}

int aac_mpe_reset(double *pos, double *vel, double *lmk, int32_t E, int32_t N, int32_t L, const uint8_t *env_mask,
                  uint64_t seed, uint64_t *counter, void *stream) {
    if (check(E, N, L)) return -1;
    if (!counter) return mfail("mpe_reset: counter");
    hipLaunchKernelGGL(mpe_reset_kernel, dim3((E + 127) / 128), dim3(128), 0, (hipStream_t)stream, pos, vel, lmk, E, N,
                       L, env_mask, seed, counter);
    hipLaunchKernelGGL(mpe_counter_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counter);
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? 0 : mfail(std::string("mpe_reset: ") + hipGetErrorString(err));
}

}  // extern "C"
