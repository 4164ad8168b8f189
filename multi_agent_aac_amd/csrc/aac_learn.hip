// aac_learn.hip -- gfx950 kernels for the MADDPG learner side (see include/aac_learn.h).
//
// attention : one 64-lane wave per row, lane = embedding dim (the reference's 64-wide
//             attention, ATT/nets:186-189), K <= 32 neighbours held in registers, dot products
//             by wave butterfly reductions; the mask (nei.mean(-1) != 0) is computed in-kernel.
// replay    : fixed-width fp32 rows; push = one workgroup per transition, sample = one 1024-thread
//             workgroup drawing B distinct indices with an LDS hash table (deterministic,
//             permutation-symmetric => uniform over B-subsets, like random.sample), gather =
//             one workgroup per sampled row writing field-contiguous batch tensors.
// adam/polyak: elementwise over one flat fp32 buffer (all parameters of a network).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/aac_learn.h"
#include "aac_wave.h"
#include "aac_noise.h"

using aacn::row_noise;
using aacn::take_epoch;

namespace {

constexpr int MAXK = 32;
constexpr int LEARN_BLOCK = 256;

thread_local std::string l_err;

int lfail(const std::string &m) {
    l_err = m;
    return -1;
}

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ inline float wave_sum(float x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// ------------------------------------------------------------------------------ attention
template <int KM>
__global__ void __launch_bounds__(LEARN_BLOCK) attn_fwd_kernel(const float *__restrict__ q,
                                                              const float *__restrict__ k,
                                                              const float *__restrict__ v, int kvs,
                                                              const float *__restrict__ nei, float *out, int outs,
                                                              float *alpha, int R, int K) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * (LEARN_BLOCK / 64) + (threadIdx.x >> 6);
    if (r >= R) return;
    const float qd = q[(size_t)r * 64 + lane];
    float s[KM];
    float mx = -INFINITY;
    unsigned valid = 0;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (j >= K) continue;
        const float kd = k[((size_t)r * K + j) * kvs + lane];
        const float sc = wave_sum(qd * kd) / 8.0f;   // score / sqrt(64)
        bool m = true;
        if (nei) {
            const float *nb = nei + ((size_t)r * K + j) * 6;
            float acc = nb[0];
            for (int c = 1; c < 6; ++c) acc += nb[c];
            m = acc != 0.0f;
        }
        s[j] = sc;
        if (m) {
            valid |= 1u << j;
            mx = sc > mx ? sc : mx;
        }
    }
    float den = 0.0f;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (j >= K) continue;
        float e = (valid >> j & 1) ? expf(s[j] - mx) : 0.0f;
        s[j] = e;
        den += e;
    }
    float o = 0.0f;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (j >= K) continue;
        const float a = (valid >> j & 1) ? s[j] / den : 0.0f;
        o += a * v[((size_t)r * K + j) * kvs + lane];
        if (lane == j) alpha[(size_t)r * K + j] = a;
    }
    out[(size_t)r * outs + lane] = o;
}

template <int KM>
__global__ void __launch_bounds__(LEARN_BLOCK) attn_bwd_kernel(const float *__restrict__ q,
                                                              const float *__restrict__ k,
                                                              const float *__restrict__ v, int kvs,
                                                              const float *__restrict__ alpha,
                                                              const float *__restrict__ dout, int douts, float *dq,
                                                              float *dk, float *dv, int R, int K) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * (LEARN_BLOCK / 64) + (threadIdx.x >> 6);
    if (r >= R) return;
    const float g = dout[(size_t)r * douts + lane];
    const float qd = q[(size_t)r * 64 + lane];
    float a[KM], da[KM];
    float S = 0.0f;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (j >= K) continue;
        a[j] = alpha[(size_t)r * K + j];
        da[j] = wave_sum(v[((size_t)r * K + j) * kvs + lane] * g);
        S += a[j] * da[j];
    }
    float dqd = 0.0f;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (j >= K) continue;
        const size_t off = ((size_t)r * K + j) * kvs + lane;
        const float ds = a[j] * (da[j] - S) / 8.0f;
        dv[off] = a[j] * g;
        dk[off] = ds * qd;
        dqd += ds * k[off];
    }
    dq[(size_t)r * 64 + lane] = dqd;
}

// --------------------------------------------------------------------------------- replay
struct Fields {
    const void *src[AAC_MAX_FIELDS];
    float *dst[AAC_MAX_FIELDS];
    int width[AAC_MAX_FIELDS];
    int offset[AAC_MAX_FIELDS + 1];
    int dtype[AAC_MAX_FIELDS];
    int n;
};


__global__ void __launch_bounds__(LEARN_BLOCK) push_kernel(float *ring, int rw, int64_t cap, const int64_t *meta,
                                                          Fields F) {
    const int e = blockIdx.x;
    const int64_t row = (meta[0] + e) % cap;
    float *dst = ring + row * rw;
    for (int c = threadIdx.x; c < F.offset[F.n]; c += LEARN_BLOCK) {      // data columns (rw may be padded)
        int f = 0;
        while (c >= F.offset[f + 1]) ++f;
        const int w = F.width[f], cc = c - F.offset[f];
        float val;
        if (F.dtype[f] == 1) val = (float)(reinterpret_cast<const uint8_t *>(F.src[f])[(size_t)e * w + cc]);
        else val = reinterpret_cast<const float *>(F.src[f])[(size_t)e * w + cc];
        dst[c] = val;
    }
}

// Push with the ring position known on the host (pushes are host-initiated, so the host mirrors
// [pos, size]): a workgroup assembles PT consecutive transitions' rows in LDS from coalesced reads
// of every field ([E][w] sources: PT*w contiguous elements each) and writes them as whole rows with
// 16-B stores; workgroup 0 stores the advanced [pos, size] for the sampler.  No read of meta, so no
// one-thread follow-up launch.
extern __shared__ float4 push_lds[];

__global__ void __launch_bounds__(LEARN_BLOCK) push_rows_kernel(float *ring, int rw, int64_t cap, int64_t pos,
                                                                int64_t *meta, int64_t new_pos, int64_t new_size,
                                                                int E, int PT, Fields F) {
    float *rows = reinterpret_cast<float *>(push_lds);
    const int e0 = blockIdx.x * PT;
    const int pt = min(PT, E - e0);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        meta[0] = new_pos;
        meta[1] = new_size;
    }
    for (int f = 0; f < F.n; ++f) {
        const int w = F.width[f], off = F.offset[f], n = pt * w;
        if (F.dtype[f] == 1) {
            const uint8_t *src = reinterpret_cast<const uint8_t *>(F.src[f]) + (size_t)e0 * w;
            for (int k = threadIdx.x; k < n; k += LEARN_BLOCK) rows[(k / w) * rw + off + k % w] = (float)src[k];
        } else {
            const float *src = reinterpret_cast<const float *>(F.src[f]) + (size_t)e0 * w;
            for (int k = threadIdx.x; k < n; k += LEARN_BLOCK) rows[(k / w) * rw + off + k % w] = src[k];
        }
    }
    const int dw = F.offset[F.n], pad = rw - dw;      // a padded row's tail: zeros
    for (int k = threadIdx.x; k < pt * pad; k += LEARN_BLOCK) rows[(k / pad) * rw + dw + k % pad] = 0.0f;
    __syncthreads();
    if ((rw & 3) == 0) {
        const int r4 = rw >> 2;
        for (int j = threadIdx.x; j < pt * r4; j += LEARN_BLOCK) {
            const int r = j / r4, c4 = j - r * r4;
            const int64_t row = (pos + e0 + r) % cap;
            reinterpret_cast<float4 *>(ring + row * rw)[c4] = push_lds[r * r4 + c4];
        }
    } else {
        for (int j = threadIdx.x; j < pt * rw; j += LEARN_BLOCK) {
            const int r = j / rw, c = j - r * rw;
            ring[((pos + e0 + r) % cap) * rw + c] = rows[j];
        }
    }
}

constexpr int TBL = 8192;

__device__ inline int64_t draw(uint64_t seed, uint64_t ctr, int idx, int att, int64_t size) {
    uint64_t h = mix64(mix64(mix64(seed) ^ ctr) ^ (((uint64_t)blockIdx.x << 44) | ((uint64_t)idx << 20) | (uint64_t)att));
    return (int64_t)(h % (uint64_t)size);
}

// (an in-kernel advance of meta by the last of the push's E workgroups to arrive measured ~90 us
// slower per step than this one-thread launch: E same-address atomics)
__global__ void meta_kernel(int64_t *meta, int64_t cap, int E) {
    meta[0] = (meta[0] + E) % cap;
    const int64_t s = meta[1] + E;
    meta[1] = s < cap ? s : cap;
}

__global__ void __launch_bounds__(1024) sample_kernel(const int64_t *meta, int B, uint64_t seed,
                                                     uint64_t *counter, int32_t *out_all) {
    int32_t *out = out_all + (size_t)blockIdx.x * B;   // one workgroup per batch
    __shared__ int keys[TBL];
    __shared__ int owner[TBL];
    // an empty ring still yields in-range rows (row 0): the host refuses to sample fewer rows than
    // B (DeviceReplay.sample_batch / the learners' plans), this only keeps a bad call in bounds
    const int64_t size = meta[1] > 0 ? meta[1] : 1;
    const uint64_t ctr = take_epoch(counter);     // the counter advances once per launch
    if (size < 2 * (int64_t)B) {
        // few spare rows (size < 2B <= 8192, the first updates after the len(memory) > B guard): a
        // redraw then hits a free row with probability (size - B) / size per round, so draw exactly
        // instead -- a partial Fisher-Yates shuffle of [0, size) in LDS (uniform ordered sample
        // without replacement, as random.sample), one thread, B swaps
        const int n = (int)size;
        for (int s = threadIdx.x; s < n; s += 1024) keys[s] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            const int m = B < n ? B : n;
            for (int i = 0; i < m; ++i) {
                const int j = i + (int)draw(seed, ctr, i, 0, n - i);
                const int t = keys[i];
                keys[i] = keys[j];
                keys[j] = t;
            }
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < B; idx += 1024) out[idx] = keys[idx < n ? idx : idx % n];
        return;
    }
    const int nv = (B + 1023) / 1024;
    int val[4], att[4];
    for (int u = 0; u < nv; ++u) {
        const int idx = threadIdx.x + u * 1024;
        att[u] = 0;
        val[u] = idx < B ? (int)draw(seed, ctr, idx, 0, size) : -1;
    }
    for (int round = 0; round < 64; ++round) {
        for (int s = threadIdx.x; s < TBL; s += 1024) {
            keys[s] = -1;
            owner[s] = INT_MAX;
        }
        __syncthreads();
        for (int u = 0; u < nv; ++u) {
            const int idx = threadIdx.x + u * 1024;
            if (idx >= B) continue;
            int h = (int)(mix64((uint64_t)val[u]) & (TBL - 1));
            while (true) {
                int old = atomicCAS(&keys[h], -1, val[u]);
                if (old == -1 || old == val[u]) {
                    atomicMin(&owner[h], idx);
                    break;
                }
                h = (h + 1) & (TBL - 1);
            }
        }
        __syncthreads();
        int redraw = 0;
        for (int u = 0; u < nv; ++u) {
            const int idx = threadIdx.x + u * 1024;
            if (idx >= B) continue;
            int h = (int)(mix64((uint64_t)val[u]) & (TBL - 1));
            while (keys[h] != val[u]) h = (h + 1) & (TBL - 1);
            if (owner[h] != idx) {
                ++att[u];
                val[u] = (int)draw(seed, ctr, idx, att[u], size);
                redraw = 1;
            }
        }
        if (!__syncthreads_or(redraw)) break;
    }
    for (int u = 0; u < nv; ++u) {
        const int idx = threadIdx.x + u * 1024;
        if (idx < B) out[idx] = val[u];
    }
}

__global__ void __launch_bounds__(LEARN_BLOCK) gather_kernel(const float *ring, int rw, const int32_t *idx, Fields F) {
    const int b = blockIdx.x;
    const float *src = ring + (int64_t)idx[b] * rw;
    for (int c = threadIdx.x; c < F.offset[F.n]; c += LEARN_BLOCK) {      // data columns (rw may be padded)
        int f = 0;
        while (c >= F.offset[f + 1]) ++f;
        const int w = F.width[f];
        F.dst[f][(size_t)b * w + (c - F.offset[f])] = src[c];
    }
}

// ------------------------------------------------------------------------------- optimiser
// gscale multiplies the gradient as it is read: 1 / world after a SUM all-reduce (the mean of the
// ranks' gradients without a separate division launch; exact for power-of-two worlds)
__global__ void adam_kernel(float *p, const float *g, float *m, float *v, int64_t n, float lr, float b1, float b2,
                            float eps, const int32_t *step, int step_add, float gscale) {
    const int t = *step + step_add;
    const double bc1 = 1.0 - pow((double)b1, (double)t);
    const double bc2 = 1.0 - pow((double)b2, (double)t);
    const float step_size = (float)((double)lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    const float w1 = (float)(1.0 - (double)b1), w2 = (float)(1.0 - (double)b2);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float gi = g[i] * gscale;
        float mi = m[i];
        mi = mi + w1 * (gi - mi);               // exp_avg.lerp_(grad, 1 - beta1)
        float vi = v[i] * b2;                   // exp_avg_sq.mul_(beta2)
        vi = vi + w2 * (gi * gi);               //   .addcmul_(grad, grad, 1 - beta2)
        const float den = sqrtf(vi) / bc2s + eps;
        p[i] = p[i] + (-step_size) * (mi / den);   // param.addcdiv_(exp_avg, denom, -step_size)
        m[i] = mi;
        v[i] = vi;
    }
}

// step (optional): the optimiser's device step counter, advanced by step_add in the same launch
// (the Polyak step is the last reader-free point of an update, ATT/maddpg:436-438)
// two networks in one launch: workgroups [0, g1) take (tgt1, src1), the rest (tgt2, src2)
__global__ void polyak2_kernel(float *tgt1, const float *src1, int64_t n1, int32_t *step1, float *tgt2,
                               const float *src2, int64_t n2, int32_t *step2, int g1, float keep, float tau,
                               int32_t step_add) {
    const bool first = (int)blockIdx.x < g1;
    float *tgt = first ? tgt1 : tgt2;
    const float *src = first ? src1 : src2;
    const int64_t n = first ? n1 : n2;
    int32_t *step = first ? step1 : step2;
    const int b = first ? blockIdx.x : blockIdx.x - g1, nb = first ? g1 : gridDim.x - g1;
    if (step && b == 0 && threadIdx.x == 0) step[0] += step_add;
    for (int64_t i = (int64_t)b * blockDim.x + threadIdx.x; i < n; i += (int64_t)nb * blockDim.x) {
        const float a = keep * tgt[i];
        const float c = tau * src[i];
        tgt[i] = a + c;
    }
}

__global__ void polyak_kernel(float *tgt, const float *src, int64_t n, float keep, float tau, int32_t *step,
                              int32_t step_add) {
    if (step && blockIdx.x == 0 && threadIdx.x == 0) step[0] += step_add;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float a = keep * tgt[i];
        const float b = tau * src[i];
        tgt[i] = a + b;
    }
}

// --------------------------------------------------------------------- activation backward
// gm[m][o] = gy[m][o] * act'(y[m][o]);  db[o] = sum_m gm[m][o]   (act: 0 identity, 1 relu, 2 tanh)
// Grid (ceil(O/64), ceil(M/32)).  Deterministic bias reduction in one launch: every workgroup
// writes its 64 column partials to ws, takes a ticket; the last workgroup of a column block sums
// the partials in row-block order (agent-scope release/acquire, MI355X_MICROARCH.md "Valid
// forms") and resets its ticket, so the kernel is graph-replayable.
template <int ACT>
__global__ void __launch_bounds__(LEARN_BLOCK) act_bgrad_kernel(const float *__restrict__ gy, int gys,
                                                               const float *__restrict__ y, int ys,
                                                               float *__restrict__ gm, int gms, float *db, int M,
                                                               int O, int rows_per_wg, float *ws,
                                                               unsigned *tickets) {
    __shared__ float part[4][64];
    __shared__ int s_last;
    const int lane = threadIdx.x & 63;
    const int col = blockIdx.x * 64 + lane;
    const int rg = threadIdx.x >> 6;
    const int m0 = blockIdx.y * rows_per_wg;
    const int m1 = min(M, m0 + rows_per_wg);
    float acc = 0.0f;
    if (col < O) {
#pragma unroll 8
        for (int m = m0 + rg; m < m1; m += 4) {
            float g = gy[(size_t)m * gys + col];
            if (ACT == 1) g = y[(size_t)m * ys + col] > 0.0f ? g : 0.0f;
            if (ACT == 2) {
                const float t = y[(size_t)m * ys + col];
                g = g * (1.0f - t * t);
            }
            if (gm) gm[(size_t)m * gms + col] = g;
            acc += g;
        }
    }
    if (!db) return;
    part[rg][lane] = acc;
    __syncthreads();
    if (rg == 0 && col < O) ws[(size_t)blockIdx.y * O + col] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = atomicAdd(&tickets[blockIdx.x], 1u);
        s_last = (t == gridDim.y - 1);
    }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float tot = 0.0f;
    if (col < O) {
#pragma unroll 8
        for (int r = rg; r < (int)gridDim.y; r += 4) tot += ws[(size_t)r * O + col];
    }
    part[rg][lane] = tot;
    __syncthreads();
    if (rg == 0 && col < O) db[col] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    if (threadIdx.x == 0) tickets[blockIdx.x] = 0;
}

// y[m][o] = act(y[m][o] + b[o]) in place
template <int ACT>
__global__ void bias_act_kernel(float *y, const float *__restrict__ b, int64_t n, int O) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float v = y[i] + b[i % O];
        if (ACT == 1) v = v > 0.0f ? v : 0.0f;
        if (ACT == 2) v = tanhf(v);
        y[i] = v;
    }
}

// ------------------------------------------------------------------------------ noise

__global__ void noise_kernel(float *act, int E, int N, const int32_t *episode, int eps_end, float noise_start,
                             float noise_end, uint64_t seed, uint64_t *counter, float *noise_out) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t ctr = take_epoch(counter);     // the counter advances once per launch
    if (row < (int64_t)E * N) {
        float n0, n1;
        row_noise(row, N, episode, eps_end, noise_start, noise_end, seed, ctr, n0, n1);
        float a0 = act[2 * row] + n0, a1 = act[2 * row + 1] + n1;
        a0 = fminf(fmaxf(a0, -1.0f), 1.0f);
        a1 = fminf(fmaxf(a1, -1.0f), 1.0f);
        act[2 * row] = a0;
        act[2 * row + 1] = a1;
        if (noise_out) {
            noise_out[2 * row] = n0;
            noise_out[2 * row + 1] = n1;
        }
    }
}

// The actor's output layer a = tanh(Wa h_a + ba) (ATT/nets:213, 256 -> 2) fused with the exploration
// noise and clamp of choose_action (ATT/maddpg:476-500).  A wave owns AON_RW = 16 consecutive agent
// rows: it issues the loads of all 16 rows (16 lanes per row, 16 features per lane: 1 KB row reads,
// coalesced), computes lane j's float64 Box-Muller noise for row j while they fly, then the dot
// pairs (sums over the 16-lane DPP rows) go through LDS to lane j, which finishes row j (tanh,
// noise, clamp).  One noise epoch per launch (take_epoch, one atomic per workgroup).  Replaces a
// grouped-GEMM launch with a 2-column output plus the noise launch.
constexpr int AON_RW = 16;

__global__ void __launch_bounds__(LEARN_BLOCK) actor_out_noise_kernel(const float *__restrict__ ha, int64_t R,
                                                                      const float *__restrict__ wa,
                                                                      const float *__restrict__ ba, float *act, int N,
                                                                      const int32_t *episode, int eps_end,
                                                                      float noise_start, float noise_end,
                                                                      uint64_t seed, uint64_t *counter, int noisy,
                                                                      float *noise_out) {
    __shared__ float2 xs[LEARN_BLOCK / 64][AON_RW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int q = lane >> 4, l16 = lane & 15;
    const int64_t base = ((int64_t)blockIdx.x * (LEARN_BLOCK / 64) + w) * AON_RW;
    float4 h[AON_RW / 4][4];
#pragma unroll
    for (int it = 0; it < AON_RW / 4; ++it) {
        const int64_t row = base + 4 * it + q;
        const float4 *hr = reinterpret_cast<const float4 *>(ha + (row < R ? row : 0) * 256) + l16 * 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) h[it][u] = hr[u];
    }
    const uint64_t ctr = noisy ? take_epoch(counter) : 0;      // the row loads fly across its barrier
    float4 w0[4], w1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        w0[u] = reinterpret_cast<const float4 *>(wa)[l16 * 4 + u];
        w1[u] = reinterpret_cast<const float4 *>(wa + 256)[l16 * 4 + u];
    }
    const int64_t myrow = base + lane;
    const bool mine = lane < AON_RW && myrow < R;
    float n0 = 0.0f, n1 = 0.0f;
    if (noisy && mine) row_noise(myrow, N, episode, eps_end, noise_start, noise_end, seed, ctr, n0, n1);
#pragma unroll
    for (int it = 0; it < AON_RW / 4; ++it) {
        float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float4 x = h[it][u];
            p0 = fmaf(x.w, w0[u].w, fmaf(x.z, w0[u].z, fmaf(x.y, w0[u].y, fmaf(x.x, w0[u].x, p0))));
            p1 = fmaf(x.w, w1[u].w, fmaf(x.z, w1[u].z, fmaf(x.y, w1[u].y, fmaf(x.x, w1[u].x, p1))));
        }
        p0 = aacw::rsum16(p0);
        p1 = aacw::rsum16(p1);
        if (l16 == 0) xs[w][4 * it + q] = make_float2(p0, p1);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");       // one wave's LDS operations run in order
    if (!mine) return;
    const float2 x = xs[w][lane];
    float a0 = tanhf(x.x + ba[0]), a1 = tanhf(x.y + ba[1]);
    if (noisy) {
        a0 = fminf(fmaxf(a0 + n0, -1.0f), 1.0f);
        a1 = fminf(fmaxf(a1 + n1, -1.0f), 1.0f);
        if (noise_out) reinterpret_cast<float2 *>(noise_out)[myrow] = make_float2(n0, n1);
    }
    reinterpret_cast<float2 *>(act)[myrow] = make_float2(a0, a1);
}

// The actor's merge layer, output layer and exploration noise (ATT/nets:211-213 + choose_action's noise
// and clamp, ATT/maddpg:476-500) over the E*N act rows in one weights-stationary launch: h_a =
// relu(Wm cat + bm) (192 -> 256), a = tanh(Wa h_a + ba) (256 -> 2), noise, clamp.  A 512-thread
// workgroup per CU; wave w owns merge features 32w .. 32w + 31 and keeps their Wm rows in registers
// (k order 48 kq + s: 16-B loads), the rows of a 16-row block on the MFMA's n axis (h_a^T = Wm cat^T
// on v_mfma_f32_16x16x4_f32).  The output layer's partial dots meet in LDS in a fixed wave order;
// h_a never reaches memory.  Replaces the merge layer's grouped-GEMM launch and actor_out_noise.
constexpr int AH_W = 8;                       // waves per workgroup
typedef float hf4 __attribute__((ext_vector_type(4)));

constexpr int AH_XS = 193;                   // LDS row stride of the staged input rows (odd: 2-way reads)
constexpr int AH_NB = 8;                     // blocks per workgroup whose noise is drawn up front

__global__ void __launch_bounds__(64 * AH_W) actor_head_ws_kernel(const float *__restrict__ cat, int ldc, int64_t R,
                                                                 const float *__restrict__ wm,
                                                                 const float *__restrict__ bm,
                                                                 const float *__restrict__ wa,
                                                                 const float *__restrict__ ba, float *act, int N,
                                                                 const int32_t *episode, int eps_end,
                                                                 float noise_start, float noise_end, uint64_t seed,
                                                                 uint64_t *counter, int noisy, float *noise_out) {
    __shared__ float sX[2][16 * AH_XS];      // the block's input rows, double-buffered
    __shared__ float2 sP[2][AH_W][16];
    __shared__ float2 sN[AH_NB * 16];        // the exploration noise of the workgroup's first AH_NB blocks
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, n = lane & 15, kq = lane >> 4;
    const int t = threadIdx.x;
    const uint64_t ctr = noisy ? take_epoch(counter) : 0;
    float a[2][48];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const hf4 *src = reinterpret_cast<const hf4 *>(wm + (size_t)(32 * w + 16 * tt + n) * 192 + 48 * kq);
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const hf4 v = src[j];
#pragma unroll
            for (int c = 0; c < 4; ++c) a[tt][4 * j + c] = v[c];
        }
    }
    // this lane's features 32w + 16tt + 4kq + v: bias and output-layer weights
    hf4 cb[2], u0[2], u1[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const int f = 32 * w + 16 * tt + 4 * kq;
        cb[tt] = *reinterpret_cast<const hf4 *>(bm + f);
        u0[tt] = *reinterpret_cast<const hf4 *>(wa + f);
        u1[tt] = *reinterpret_cast<const hf4 *>(wa + 256 + f);
    }
    const float ba0 = ba[0], ba1 = ba[1];
    const int64_t nblk = (R + 15) / 16;
    // the noise does not depend on h_a: the rows of the workgroup's first AH_NB blocks get theirs now,
    // one row per thread while the weight loads fly (in the block tail it was a float64 Box-Muller
    // chain on 16 lanes after every block's barrier)
    if (noisy && t < AH_NB * 16) {
        const int64_t row = (blockIdx.x + (int64_t)(t >> 4) * gridDim.x) * 16 + (t & 15);
        float n0 = 0.0f, n1 = 0.0f;
        if (row < R) row_noise(row, N, episode, eps_end, noise_start, noise_end, seed, ctr, n0, n1);
        sN[t] = make_float2(n0, n1);
    }
    // staging of a block's 16 x 192 input floats: 768 16-B items, items t and t + 512 of this thread
    hf4 pf[2];
    auto load_rows = [&](int64_t blk) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = t + 512 * u;
            const int row = i / 48, c4 = i - row * 48;
            int64_t r = blk * 16 + row;
            r = r < R ? r : R - 1;
            pf[u] = (i < 768) ? reinterpret_cast<const hf4 *>(cat + r * ldc)[c4] : hf4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    };
    auto store_rows = [&](float *dst) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = t + 512 * u;
            const int row = i / 48, c4 = i - row * 48;
            if (i < 768)
#pragma unroll
                for (int c = 0; c < 4; ++c) dst[row * AH_XS + 4 * c4 + c] = pf[u][c];
        }
    };
    if (blockIdx.x < nblk) {
        load_rows(blockIdx.x);
        store_rows(sX[0]);
    }
    __syncthreads();
    int cur = 0, kb = 0;
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x, ++kb) {
        const bool more = blk + gridDim.x < nblk;
        if (more) load_rows(blk + gridDim.x);      // in flight across the MFMA chain
        const float *x = sX[cur] + n * AH_XS + 48 * kq;
        hf4 acc[2] = {hf4{0.0f, 0.0f, 0.0f, 0.0f}, hf4{0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
        for (int s = 0; s < 48; ++s) {
            const float bv = x[s];
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tt][s], bv, acc[tt], 0, 0, 0);
        }
        float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                float h = acc[tt][v] + cb[tt][v];
                h = h > 0.0f ? h : 0.0f;
                p0 = fmaf(u0[tt][v], h, p0);
                p1 = fmaf(u1[tt][v], h, p1);
            }
        p0 += __shfl_xor(p0, 16, 64);
        p1 += __shfl_xor(p1, 16, 64);
        p0 += __shfl_xor(p0, 32, 64);
        p1 += __shfl_xor(p1, 32, 64);
        if (kq == 0) sP[cur][w][n] = make_float2(p0, p1);
        if (more) store_rows(sX[cur ^ 1]);        // read by the next block after the barrier
        __syncthreads();
        if (t < 16) {
            const int64_t row = blk * 16 + t;
            if (row < R) {
                float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
                for (int q = 0; q < AH_W; ++q) {
                    s0 += sP[cur][q][t].x;
                    s1 += sP[cur][q][t].y;
                }
                float a0 = tanhf(s0 + ba0), a1 = tanhf(s1 + ba1);
                if (noisy) {
                    float n0, n1;
                    if (kb < AH_NB) {
                        const float2 nz = sN[kb * 16 + t];
                        n0 = nz.x;
                        n1 = nz.y;
                    } else {
                        row_noise(row, N, episode, eps_end, noise_start, noise_end, seed, ctr, n0, n1);
                    }
                    a0 = fminf(fmaxf(a0 + n0, -1.0f), 1.0f);
                    a1 = fminf(fmaxf(a1 + n1, -1.0f), 1.0f);
                    if (noise_out) reinterpret_cast<float2 *>(noise_out)[row] = make_float2(n0, n1);
                }
                reinterpret_cast<float2 *>(act)[row] = make_float2(a0, a1);
            }
        }
        cur ^= 1;
    }
}

#define LHIP(x)                                                                                  \
    do {                                                                                         \
        hipError_t _e = (x);                                                                     \
        if (_e != hipSuccess) return lfail(std::string(#x) + ": " + hipGetErrorString(_e));     \
    } while (0)

int grid_for(int64_t n) {
    int64_t b = (n + LEARN_BLOCK - 1) / LEARN_BLOCK;
    return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

}  // namespace

extern "C" {

const char *aac_learn_last_error(void) { return l_err.c_str(); }

int aac_attn_fwd(const float *q, const float *k, const float *v, int32_t kvs, const float *nei, float *out,
                 int32_t outs, float *alpha, int32_t R, int32_t K, void *stream) {
    if (K < 1 || K > MAXK || R < 0) return lfail("attn: need 1 <= K <= 32");
    if (R == 0) return 0;
#define FWD(KM) hipLaunchKernelGGL(attn_fwd_kernel<KM>, dim3((R + 3) / 4), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, \
                                   q, k, v, kvs, nei, out, outs, alpha, R, K)
    if (K <= 4) FWD(4);
    else if (K <= 8) FWD(8);
    else if (K <= 16) FWD(16);
    else FWD(32);
#undef FWD
    LHIP(hipGetLastError());
    return 0;
}

int aac_attn_bwd(const float *q, const float *k, const float *v, int32_t kvs, const float *alpha, const float *dout,
                 int32_t douts, float *dq, float *dk, float *dv, int32_t R, int32_t K, void *stream) {
    if (K < 1 || K > MAXK || R < 0) return lfail("attn: need 1 <= K <= 32");
    if (R == 0) return 0;
#define BWD(KM) hipLaunchKernelGGL(attn_bwd_kernel<KM>, dim3((R + 3) / 4), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, \
                                   q, k, v, kvs, alpha, dout, douts, dq, dk, dv, R, K)
    if (K <= 4) BWD(4);
    else if (K <= 8) BWD(8);
    else if (K <= 16) BWD(16);
    else BWD(32);
#undef BWD
    LHIP(hipGetLastError());
    return 0;
}

static int make_fields(Fields &F, int n, const int32_t *widths, int rw) {
    if (n < 1 || n > AAC_MAX_FIELDS) return lfail("replay: 1..16 fields");
    F.n = n;
    F.offset[0] = 0;
    for (int f = 0; f < n; ++f) {
        F.width[f] = widths[f];
        F.offset[f + 1] = F.offset[f] + widths[f];
    }
    for (int f = n; f < AAC_MAX_FIELDS; ++f) F.offset[f + 1] = INT_MAX;
    // rw: the ring's row stride, the field widths' sum or more (rows padded to whole cache lines)
    if (F.offset[n] > rw) return lfail("replay: field widths exceed row_width");
    return 0;
}

int aac_replay_push(float *ring, int32_t rw, int64_t cap, int64_t *meta, int32_t n, const void *const *srcs,
                    const int32_t *widths, const int32_t *dtypes, int32_t E, void *stream) {
    Fields F{};
    if (make_fields(F, n, widths, rw)) return -1;
    if (E < 1 || E > cap) return lfail("replay: need 1 <= E <= capacity");
    for (int f = 0; f < n; ++f) {
        F.src[f] = srcs[f];
        F.dtype[f] = dtypes ? dtypes[f] : 0;
    }
    hipLaunchKernelGGL(push_kernel, dim3(E), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, ring, rw, cap, meta, F);
    hipLaunchKernelGGL(meta_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, meta, cap, E);
    LHIP(hipGetLastError());
    return 0;
}

int aac_replay_push_at(float *ring, int32_t rw, int64_t cap, int64_t *meta, int64_t pos, int64_t size, int32_t n,
                       const void *const *srcs, const int32_t *widths, const int32_t *dtypes, int32_t E,
                       void *stream) {
    Fields F{};
    if (make_fields(F, n, widths, rw)) return -1;
    if (E < 1 || E > cap) return lfail("replay: need 1 <= E <= capacity");
    if (pos < 0 || pos >= cap || size < 0 || size > cap) return lfail("replay: need 0 <= pos < capacity, size <= capacity");
    if ((reinterpret_cast<uintptr_t>(ring) & 15) != 0) return lfail("replay: ring must be 16-B aligned");
    for (int f = 0; f < n; ++f) {
        F.src[f] = srcs[f];
        F.dtype[f] = dtypes ? dtypes[f] : 0;
    }
    // transitions per workgroup: 4 (16 left one workgroup per CU: 14.2 us at E = 4096), rows within
    // 64 KB of LDS
    const int PT = std::max(1, std::min(4, (int)(65536 / (4 * (int64_t)rw))));
    const size_t lds = (size_t)PT * rw * 4;
    const int64_t np = (pos + E) % cap, ns = std::min<int64_t>(size + E, cap);
    hipLaunchKernelGGL(push_rows_kernel, dim3((E + PT - 1) / PT), dim3(LEARN_BLOCK), lds, (hipStream_t)stream, ring, rw,
                       cap, pos, meta, np, ns, E, PT, F);
    LHIP(hipGetLastError());
    return 0;
}

int aac_replay_sample(const int64_t *meta, int32_t B, int32_t nb, uint64_t seed, uint64_t *counter, int32_t *idx,
                      void *stream) {
    if (B < 1 || B > 4096) return lfail("replay: 1 <= B <= 4096");
    if (nb < 1) return lfail("replay: n_batches >= 1");
    hipLaunchKernelGGL(sample_kernel, dim3(nb), dim3(1024), 0, (hipStream_t)stream, meta, B, seed, counter, idx);
    LHIP(hipGetLastError());
    return 0;
}

int aac_replay_gather(const float *ring, int32_t rw, const int32_t *idx, int32_t B, int32_t n, float *const *dsts,
                      const int32_t *widths, void *stream) {
    Fields F{};
    if (make_fields(F, n, widths, rw)) return -1;
    for (int f = 0; f < n; ++f) F.dst[f] = dsts[f];
    hipLaunchKernelGGL(gather_kernel, dim3(B), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, ring, rw, idx, F);
    LHIP(hipGetLastError());
    return 0;
}

int aac_adam_flat(float *p, const float *g, float *m, float *v, int64_t n, float lr, float b1, float b2, float eps,
                  const int32_t *step, void *stream) {
    return aac_adam_flat_at(p, g, m, v, n, lr, b1, b2, eps, step, 0, stream);
}

int aac_adam_flat_at(float *p, const float *g, float *m, float *v, int64_t n, float lr, float b1, float b2,
                     float eps, const int32_t *step, int32_t step_add, void *stream) {
    return aac_adam_flat_at_scaled(p, g, m, v, n, lr, b1, b2, eps, step, step_add, 1.0f, stream);
}

int aac_adam_flat_at_scaled(float *p, const float *g, float *m, float *v, int64_t n, float lr, float b1, float b2,
                            float eps, const int32_t *step, int32_t step_add, float gscale, void *stream) {
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, p, g, m, v, n, lr,
                       b1, b2, eps, step, step_add, gscale);
    LHIP(hipGetLastError());
    return 0;
}

int aac_polyak_flat(float *tgt, const float *src, int64_t n, float tau, void *stream) {
    return aac_polyak_flat_step(tgt, src, n, tau, nullptr, 0, stream);
}

int aac_polyak_flat_step(float *tgt, const float *src, int64_t n, float tau, int32_t *step, int32_t step_add,
                         void *stream) {
    const float keep = (float)(1.0 - (double)tau);
    hipLaunchKernelGGL(polyak_kernel, dim3(grid_for(n)), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, tgt, src, n,
                       keep, tau, step, step_add);
    LHIP(hipGetLastError());
    return 0;
}

int aac_polyak_flat2(float *tgt1, const float *src1, int64_t n1, int32_t *step1, float *tgt2, const float *src2,
                     int64_t n2, int32_t *step2, float tau, int32_t step_add, void *stream) {
    if (n1 < 1 || n2 < 1) return lfail("polyak_flat2: both networks non-empty");
    const float keep = (float)(1.0 - (double)tau);
    const int g1 = grid_for(n1), g2 = grid_for(n2);
    hipLaunchKernelGGL(polyak2_kernel, dim3(g1 + g2), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, tgt1, src1, n1, step1,
                       tgt2, src2, n2, step2, g1, keep, tau, step_add);
    LHIP(hipGetLastError());
    return 0;
}

int aac_act_bgrad(const float *gy, int32_t gys, const float *y, int32_t ys, float *gm, int32_t gms, float *db,
                  int32_t M, int32_t O, int32_t act, float *ws, uint32_t *tickets, void *stream) {
    if (M <= 0 || O <= 0) return 0;
    const int rpw = 32;   // 8 rows per thread: larger tiles measured slower (latency-bound rows)
    dim3 grid((O + 63) / 64, (M + rpw - 1) / rpw);
    if (db && (!ws || !tickets)) return lfail("act_bgrad: db needs ws[ceil(M/32)][O] and tickets[ceil(O/64)]");
#define ABG(A) hipLaunchKernelGGL(act_bgrad_kernel<A>, grid, dim3(LEARN_BLOCK), 0, (hipStream_t)stream, gy, gys, y, ys, \
                                  gm, gms, db, M, O, rpw, ws, tickets)
    if (act == 0) ABG(0);
    else if (act == 1) ABG(1);
    else if (act == 2) ABG(2);
    else return lfail("act_bgrad: act must be 0, 1 or 2");
#undef ABG
    LHIP(hipGetLastError());
    return 0;
}

int aac_bias_act(float *y, const float *b, int64_t M, int32_t O, int32_t act, void *stream) {
    const int64_t n = M * O;
    if (n <= 0) return 0;
    if (act == 0) hipLaunchKernelGGL(bias_act_kernel<0>, dim3(grid_for(n)), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, y, b, n, O);
    else if (act == 1) hipLaunchKernelGGL(bias_act_kernel<1>, dim3(grid_for(n)), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, y, b, n, O);
    else if (act == 2) hipLaunchKernelGGL(bias_act_kernel<2>, dim3(grid_for(n)), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, y, b, n, O);
    else return lfail("bias_act: act must be 0, 1 or 2");
    LHIP(hipGetLastError());
    return 0;
}

int aac_noise_clamp(float *act, int32_t E, int32_t N, const int32_t *episode, int32_t eps_end, float noise_start,
                    float noise_end, uint64_t seed, uint64_t *counter, float *noise_out, void *stream) {
    const int64_t rows = (int64_t)E * N;
    hipLaunchKernelGGL(noise_kernel, dim3((unsigned)((rows + LEARN_BLOCK - 1) / LEARN_BLOCK)), dim3(LEARN_BLOCK), 0,
                       (hipStream_t)stream, act, E, N, episode, eps_end, noise_start, noise_end, seed, counter,
                       noise_out);
    LHIP(hipGetLastError());
    return 0;
}

int aac_actor_out_noise(const float *ha, int64_t R, const float *wa, const float *ba, float *act, int32_t N,
                        const int32_t *episode, int32_t eps_end, float noise_start, float noise_end, uint64_t seed,
                        uint64_t *counter, int32_t noisy, float *noise_out, void *stream) {
    if (R <= 0) return 0;
    if (N <= 0 || R % N) return lfail("actor_out_noise: R must be a multiple of N > 0");
    if (((reinterpret_cast<uintptr_t>(ha) | reinterpret_cast<uintptr_t>(wa)) & 15) != 0 ||
        (reinterpret_cast<uintptr_t>(act) & 7) != 0 || (reinterpret_cast<uintptr_t>(noise_out) & 7) != 0)
        return lfail("actor_out_noise: ha / wa 16-B, act / noise_out 8-B aligned");
    if (noisy && !counter) return lfail("actor_out_noise: noisy needs the counter");
    const int64_t wg = (R + 4 * AON_RW - 1) / (4 * AON_RW);
    hipLaunchKernelGGL(actor_out_noise_kernel, dim3((unsigned)wg), dim3(LEARN_BLOCK), 0, (hipStream_t)stream, ha, R, wa,
                       ba, act, N, episode, eps_end, noise_start, noise_end, seed, counter, noisy, noise_out);
    LHIP(hipGetLastError());
    return 0;
}

int aac_actor_head_ws(const float *cat, int32_t ldc, int64_t R, const float *wm, const float *bm, const float *wa,
                      const float *ba, float *act, int32_t N, const int32_t *episode, int32_t eps_end,
                      float noise_start, float noise_end, uint64_t seed, uint64_t *counter, int32_t noisy,
                      float *noise_out, void *stream) {
    if (R <= 0) return 0;
    if (N <= 0 || R % N) return lfail("actor_head_ws: R must be a multiple of N > 0");
    auto al = [](const void *p, int a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
    if (!cat || !wm || !bm || !wa || !ba || !act) return lfail("actor_head_ws: NULL operand");
    if (ldc < 192 || ldc % 4 || !al(cat, 16) || !al(wm, 16) || !al(bm, 16) || !al(wa, 16) || !al(act, 8) ||
        !al(noise_out, 8))
        return lfail("actor_head_ws: cat rows (ldc >= 192, % 4), wm, bm, wa 16-B aligned, act / noise_out 8-B");
    if (noisy && !counter) return lfail("actor_head_ws: noisy needs the counter");
    const int64_t nblk = (R + 15) / 16;
    const int wg = (int)std::min<int64_t>(nblk, 256);      // one workgroup per CU
    hipLaunchKernelGGL(actor_head_ws_kernel, dim3(wg), dim3(64 * AH_W), 0, (hipStream_t)stream, cat, ldc, R, wm, bm, wa,
                       ba, act, N, episode, eps_end, noise_start, noise_end, seed, counter, noisy, noise_out);
    LHIP(hipGetLastError());
    return 0;
}

}  // extern "C"
