// aac_uam_learn.hip -- the fused float64 learner of the UAM variant (include/aac_uam_learn.h;
// SURVEY.md section 8(f) f3).
//
// update_myown of UAM/maddpg:304-595 (shared ActorNetwork_TwoPortion + critic_single_TwoPortion,
// float64, one gradient iteration of B rows, Polyak tau) as grouped float64 GEMM launches with
// fused epilogues plus four small kernels; the launch list lives in uam_learner.FusedUamUpdate.
//
// gemm64_kernel: one 16x16 output tile per wave on v_mfma_f64_16x16x4_f64 (C/D: col = lane & 15,
// row = (lane >> 4) + 4 reg; A/B: lane holds op(A)[lane & 15][k] / op(B)[k][lane & 15] with
// k = 4 step + (lane >> 4)).  Operands are raw buffer loads whose out-of-range offsets return 0,
// so nothing touches a loaded value before its MFMA; two groups of 8 k-steps are in flight.  The
// UAM products are small (B = 512, widths 2 .. 256), so the kernel is built for many short waves:
// weight gradients split K = B into partial copies summed by the Adam kernel in fixed order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "../../include/aac_uam_learn.h"

namespace {

thread_local std::string g_lerr;

int lfail(const std::string &m) {
    g_lerr = m;
    return -1;
}

#define LHIP(x)                                                                                  \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) return lfail(std::string(#x) + ": " + hipGetErrorString(e_));      \
    } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef int i2 __attribute__((ext_vector_type(2)));
__device__ i2 buf_load_2i(i4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");

constexpr int OOB = 0x7ffffff0;     // byte offset past every operand (= num_records)
constexpr int G = 8;                // k steps (of 4) per prefetch group

struct Q64 {
    const double *A, *B;
    double *C;
    const double *bias, *addend, *mask;
    double *cextra;
    int64_t sstride;
    int M, N, K, lda, ldb, ldc, ldadd, ldmask, ta, tb, act, mact, ones, ks;
    int tiles_n, w_begin;           // w_begin in waves
    int kw;                         // waves per tile: 1, or 4 (a workgroup splits K and reduces in LDS)
    const double *dvec;             // dual output: C2[m][n] = C[m][n] > 0 ? dscale * dvec[n] : 0
    double *C2;
    double dscale;
};

struct Q64Batch {
    Q64 p[AAC_GEMM64_MAX];
    int n, waves;
};

__device__ __forceinline__ i4 rsrc64(const double *p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    i4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
    r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32));     // stride 0
    r.z = OOB;                                                 // num_records (bytes)
    r.w = 0x00020000;                                          // gfx9 dword3: 32-bit data format
    return r;
}

__device__ __forceinline__ double ld64(i4 r, int off) { return __builtin_bit_cast(double, buf_load_2i(r, off, 0, 0)); }

__global__ void __launch_bounds__(256) gemm64_kernel(Q64Batch g) {
    __shared__ d4 red[4][64];
    // the wave index is made wave-uniform so the product's fields are scalar loads (a per-lane
    // index turns every field access into a vector load with its own wait)
    const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (gw >= g.waves) return;
    int pi = 0;
    while (pi + 1 < g.n && gw >= g.p[pi + 1].w_begin) ++pi;
    const Q64 &P = g.p[pi];
    const int K = P.K, ks = P.ks, kw = P.kw;
    const int local = (gw - P.w_begin) / kw, wq = (gw - P.w_begin) % kw;     // tile-split, quarter
    const int s = local % ks, tile = local / ks;
    const int m0 = (tile / P.tiles_n) * 16, n0 = (tile % P.tiles_n) * 16;
    const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
    const int nreal = P.N - P.ones;
    const int nst = (K + 3) / 4, per = (nst + ks - 1) / ks;
    // kw = 4: the workgroup's four waves take consecutive quarters of the split's steps
    const int per4 = (per + kw - 1) / kw;
    const int sq0 = s * per, se = min(nst, sq0 + per);
    const int st0 = min(se, sq0 + wq * per4), st1 = min(se, st0 + per4);
    const i4 ra = rsrc64(P.A), rb = rsrc64(P.B);
    const int m = m0 + r, n = n0 + r;
    const bool mok = m < P.M, nok = n < nreal, isone = P.ones && n == nreal;
    // op(A)[m][k] = base_a + k * sa, op(B)[k][n] = base_b + k * sb (element offsets)
    const int sa = P.ta ? P.lda : 1, base_a = P.ta ? m : m * P.lda;
    const int sb = P.tb ? 1 : P.ldb, base_b = P.tb ? n * P.ldb : n;
    auto aoff = [&](int k) { return (mok && k < K) ? (base_a + k * sa) * 8 : OOB; };
    auto boff = [&](int k) { return (nok && k < K) ? (base_b + k * sb) * 8 : OOB; };
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    double a0[G], b0[G], a1[G], b1[G];
    auto load = [&](int sg, double(&a)[G], double(&b)[G]) {
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const int st = sg + q, k = 4 * st + kq;
            const bool on = st < st1;
            a[q] = ld64(ra, on ? aoff(k) : OOB);
            b[q] = ld64(rb, on ? boff(k) : OOB);
        }
    };
    auto comp = [&](int sg, const double(&a)[G], const double(&b)[G]) {
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const int st = sg + q;
            if (st >= st1) break;                    // wave-uniform
            const double bv = isone ? ((4 * st + kq < K) ? 1.0 : 0.0) : b[q];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], bv, acc, 0, 0, 0);
        }
    };
    load(st0, a0, b0);
    for (int sg = st0; sg < st1; sg += 2 * G) {
        load(sg + G, a1, b1);
        comp(sg, a0, b0);
        if (sg + G >= st1) break;
        load(sg + 2 * G, a0, b0);
        comp(sg + G, a1, b1);
    }
    if (kw > 1) {
        // the four quarters in wave order; wave 0 finishes the tile
        red[wq][lane] = acc;
        __syncthreads();
        if (wq != 0) return;
        acc = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    }
    double *C = P.C ? P.C + (int64_t)s * P.sstride : nullptr;
    double *cx = P.cextra ? P.cextra + (int64_t)s * P.sstride : nullptr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int mm = m0 + kq + 4 * j;              // f64 C/D layout
        if (mm >= P.M) continue;
        double v = acc[j];
        if (isone) {
            cx[mm] = v;
            continue;
        }
        if (!nok) continue;
        if (P.addend) v += P.addend[(size_t)mm * P.ldadd + n];
        if (P.bias) v += P.bias[n];
        if (P.act == 1) v = v > 0.0 ? v : 0.0;
        else if (P.act == 2) v = tanh(v);
        if (P.mact == 1) {
            v = P.mask[(size_t)mm * P.ldmask + n] > 0.0 ? v : 0.0;
        } else if (P.mact == 2) {
            const double t = P.mask[(size_t)mm * P.ldmask + n];
            v = v * (1.0 - t * t);
        }
        C[(size_t)mm * P.ldc + n] = v;
        if (P.C2) P.C2[(size_t)mm * P.ldc + n] = v > 0.0 ? P.dscale * P.dvec[n] : 0.0;
    }
}

// replay rows -> learner layouts (ROW = own 7 | radar 18 | a 2 | r | done | own' 7 | radar' 18)
__global__ void __launch_bounds__(64) uam_gather_kernel(const double *__restrict__ ring, const int32_t *__restrict__ idx,
                                                        int B, double *rows, double *xc, double *xt, double *xp) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (b >= B || t >= 54) return;
    const double v = ring[(int64_t)idx[b] * 54 + t];
    rows[(size_t)b * 54 + t] = v;
    if (t < 7) {
        xc[(size_t)b * 9 + t] = v;
        xp[(size_t)b * 9 + t] = v;
    } else if (t >= 25 && t < 27) {
        xc[(size_t)b * 9 + 7 + (t - 25)] = v;
    } else if (t >= 29 && t < 36) {
        xt[(size_t)b * 9 + (t - 29)] = v;
    }
}

// critic output layer, one wave per row (lane c holds features c, c + 64, c + 128, c + 192)
__global__ void __launch_bounds__(256) uam_head_kernel(const double *__restrict__ h, int B, const double *__restrict__ w,
                                                       const double *__restrict__ b, int mode, double *y,
                                                       const double *__restrict__ rew, const double *__restrict__ done,
                                                       int ldr, double gamma, double *dqo, double *dh,
                                                       double *lterm) {
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= B) return;
    const double *hr = h + (size_t)r * 256;
    double hv[4], p = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        hv[c] = hr[lane + 64 * c];
        p = fma(hv[c], w[lane + 64 * c], p);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
    const double q = p + b[0];
    if (mode == 2) {
        if (lane == 0) y[r] = rew[(size_t)r * ldr] + gamma * q * (1.0 - done[(size_t)r * ldr]);
        return;
    }
    double dq;
    if (mode == 0) {
        const double e = q - y[r];
        dq = (2.0 / B) * e;
        if (lane == 0) lterm[r] = e * e;
    } else {
        dq = -1.0 / B;
        if (lane == 0) lterm[r] = q;
    }
    if (dqo && lane == 0) dqo[r] = dq;
#pragma unroll
    for (int c = 0; c < 4; ++c) dh[(size_t)r * 256 + lane + 64 * c] = hv[c] > 0.0 ? dq * w[lane + 64 * c] : 0.0;
}

// the TD target (mode 2 on the target critic's rows ht) and the critic's mse head (mode 0 on h) of
// the same row in one pass: y[r] is computed and then used in-register (the values of the two
// launches of uam_head_kernel, bit for bit)
__device__ __forceinline__ double row_dot256(const double *__restrict__ hr, const double *__restrict__ w, int lane,
                                             double (&hv)[4]) {
    double p = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        hv[c] = hr[lane + 64 * c];
        p = fma(hv[c], w[lane + 64 * c], p);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
    return p;
}

__global__ void __launch_bounds__(256) uam_td_mse_head_kernel(const double *__restrict__ ht,
                                                              const double *__restrict__ wt,
                                                              const double *__restrict__ bt,
                                                              const double *__restrict__ rew,
                                                              const double *__restrict__ done, int ldr, double gamma,
                                                              double *y, const double *__restrict__ h,
                                                              const double *__restrict__ w,
                                                              const double *__restrict__ b, int B, double *dqo,
                                                              double *dh, double *lterm) {
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= B) return;
    double hv[4];
    const double qt = row_dot256(ht + (size_t)r * 256, wt, lane, hv) + bt[0];
    const double yv = rew[(size_t)r * ldr] + gamma * qt * (1.0 - done[(size_t)r * ldr]);
    if (lane == 0) y[r] = yv;
    const double q = row_dot256(h + (size_t)r * 256, w, lane, hv) + b[0];
    const double e = q - yv;
    const double dq = (2.0 / B) * e;
    if (lane == 0) lterm[r] = e * e;
    if (dqo && lane == 0) dqo[r] = dq;
#pragma unroll
    for (int c = 0; c < 4; ++c) dh[(size_t)r * 256 + lane + 64 * c] = hv[c] > 0.0 ? dq * w[lane + 64 * c] : 0.0;
}

__global__ void adam64_kernel(double *p, const double *__restrict__ gpart, int ns, double *m, double *v, int64_t n,
                              double lr, double b1, double b2, double eps, const int32_t *step, int step_add,
                              double gscale) {
    const int t = *step + step_add;
    const double bc1 = 1.0 - pow(b1, (double)t), bc2 = 1.0 - pow(b2, (double)t);
    const double step_size = lr / bc1, bc2s = sqrt(bc2);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double gi = gpart[i];
        int s = 1;
        for (; s + 8 <= ns; s += 8) {
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = gpart[(int64_t)(s + u) * n + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) gi += x[u];
        }
        for (; s < ns; ++s) gi += gpart[(int64_t)s * n + i];
        gi *= gscale;           // 1 / world after a SUM all-reduce (1 otherwise); the mean exactly for power-of-two worlds
        const double mi = b1 * m[i] + (1.0 - b1) * gi;
        const double vi = b2 * v[i] + (1.0 - b2) * gi * gi;
        const double den = sqrt(vi) / bc2s + eps;
        p[i] = p[i] - step_size * mi / den;
        m[i] = mi;
        v[i] = vi;
    }
}

// the fixed-order sum of ns partial copies (the adam64_kernel order): the gradient a multi-rank
// update all-reduces before its Adam step (aac_adam64_sum with nsplit = 1 on the result)
__global__ void sum64_kernel(double *out, const double *__restrict__ gpart, int ns, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double gi = gpart[i];
        int s = 1;
        for (; s + 8 <= ns; s += 8) {
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = gpart[(int64_t)(s + u) * n + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) gi += x[u];
        }
        for (; s < ns; ++s) gi += gpart[(int64_t)s * n + i];
        out[i] = gi;
    }
}

__global__ void uam_polyak_kernel(double *tgt, const double *__restrict__ src, int64_t n, double tau, int32_t *step,
                                  const double *lq, const double *la, int B, double *loss) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double t = tgt[i];
        tgt[i] = t + tau * (src[i] - t);
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        // the loss means: lane-strided partial sums then a fixed xor tree (deterministic; a single
        // thread walking the rows costs one dependent load latency per row, ~80 us at B = 512)
        const int lane = threadIdx.x;
        double sq = 0.0, sa = 0.0;
        for (int r = lane; r < B; r += 64) {
            if (lq) sq += lq[r];
            if (la) sa += la[r];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            sq += __shfl_xor(sq, o, 64);
            sa += __shfl_xor(sa, o, 64);
        }
        if (lane == 0) {
            if (step) *step += 1;
            if (loss) {
                loss[0] = sq / B;
                loss[1] = -(sa / B);
            }
        }
    }
}

// one replay row per aircraft (UamReplay.push_batch): a workgroup assembles 64 rows in LDS from
// coalesced reads of the seven sources, then writes them as 64 x 54 contiguous doubles (two ring
// segments at the wrap); thread 0 of workgroup 0 stores the ring's new [pos, size] (meta).
// done is uint8 (env output) or float64.  pos_in non-null (graph replays): the position is read from
// that device word and the advanced one stored to pos_out (another word: every workgroup reads pos_in),
// the size advanced in meta[1] by workgroup 0 alone.
constexpr int PR = 64;            // rows per workgroup
__global__ void __launch_bounds__(256) uam_push_kernel(double *ring, int64_t capacity, int64_t pos, int M,
                                                       const double *__restrict__ own, const double *__restrict__ radar,
                                                       const double *__restrict__ act, const double *__restrict__ rew,
                                                       const void *__restrict__ done, int done_u8,
                                                       const double *__restrict__ nown,
                                                       const double *__restrict__ nradar, int64_t *meta,
                                                       int64_t new_pos, int64_t new_size,
                                                       const int64_t *__restrict__ pos_in, int64_t *pos_out) {
    __shared__ double t[PR * 54];
    const int r0 = blockIdx.x * PR, nr = min(PR, M - r0), tid = threadIdx.x;
    if (pos_in) pos = *pos_in;
    if (blockIdx.x == 0 && tid == 0) {
        if (pos_in) {
            const int64_t np = pos + M >= capacity ? pos + M - capacity : pos + M;
            const int64_t ns = meta[1] + M;
            *pos_out = np;
            meta[0] = np;
            meta[1] = ns < capacity ? ns : capacity;
        } else if (meta) {
            meta[0] = new_pos;
            meta[1] = new_size;
        }
    }
    auto stage = [&](const double *src, int w, int c0) {
        for (int e = tid; e < nr * w; e += 256) {
            const int rr = e / w;
            t[rr * 54 + c0 + (e - rr * w)] = src[(size_t)r0 * w + e];
        }
    };
    stage(own, 7, 0);
    stage(radar, 18, 7);
    stage(act, 2, 25);
    stage(rew, 1, 27);
    for (int e = tid; e < nr; e += 256)
        t[e * 54 + 28] = done_u8 ? (double)static_cast<const uint8_t *>(done)[r0 + e]
                                 : static_cast<const double *>(done)[r0 + e];
    stage(nown, 7, 29);
    stage(nradar, 18, 36);
    __syncthreads();
    int64_t slot = pos + r0;
    if (slot >= capacity) slot -= capacity;
    const int first = (int)min<int64_t>(nr, capacity - slot);     // rows before the wrap
    for (int e = tid; e < nr * 54; e += 256) {
        const int rr = e / 54;
        double *dst = rr < first ? ring + slot * 54 : ring - (int64_t)first * 54;
        dst[e] = t[e];
    }
}

int env_i(const char *name, int dflt) {
    const char *v = getenv(name);
    return v ? atoi(v) : dflt;
}
const int g_kw4 = env_i("AAC_GEMM64_KW4", 1);
const int g_kw4_steps = env_i("AAC_GEMM64_KW4_STEPS", 16);
const int g_kw4_tiles = env_i("AAC_GEMM64_KW4_TILES", 1024);

int grid_of(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

}  // namespace

extern "C" {

const char *aac_uam_learn_last_error(void) { return g_lerr.c_str(); }

int aac_gemm64_batch(const aac_gemm64_prob *in, int32_t n, void *stream) {
    if (n < 1 || n > AAC_GEMM64_MAX) return lfail("gemm64_batch: 1 <= n <= AAC_GEMM64_MAX");
    Q64Batch g{};
    g.n = n;
    int64_t waves = 0;
    for (int i = 0; i < n; ++i) {
        const aac_gemm64_prob &s = in[i];
        Q64 &d = g.p[i];
        const std::string who = "gemm64_batch product " + std::to_string(i) + ": ";
        if (s.M <= 0 || s.N <= 0 || s.K <= 0) return lfail(who + "empty product");
        if (!s.A || !s.B) return lfail(who + "NULL operand");
        if (s.ones && !s.cextra) return lfail(who + "ones column needs cextra");
        if (s.N - s.ones > 0 && !s.C) return lfail(who + "NULL C");
        if (s.mact && !s.mask) return lfail(who + "mact needs mask");
        if (s.act < 0 || s.act > 2 || s.mact < 0 || s.mact > 2 || s.ones < 0 || s.ones > 1)
            return lfail(who + "bad act / mact / ones");
        const int ks = s.ksplit > 1 ? s.ksplit : 1;
        if (ks > 1 && (s.split_stride <= 0 || s.addend || s.bias || s.act || s.mact))
            return lfail(who + "ksplit > 1 needs split_stride and a plain epilogue");
        // every operand element is addressed by a 32-bit byte offset
        const int64_t nr = s.N - s.ones;
        const int64_t ea = s.ta ? (int64_t)s.K * s.lda : (int64_t)s.M * s.lda;
        const int64_t eb = s.tb ? nr * s.ldb : (int64_t)s.K * s.ldb;
        if (8 * ea >= OOB || 8 * eb >= OOB) return lfail(who + "operand larger than 2 GB");
        d.A = s.A; d.B = s.B; d.C = s.C; d.bias = s.bias; d.addend = s.addend; d.mask = s.mask;
        d.cextra = s.cextra;
        d.sstride = s.split_stride;
        d.M = s.M; d.N = s.N; d.K = s.K;
        d.lda = s.lda; d.ldb = s.ldb; d.ldc = s.ldc; d.ldadd = s.ldadd; d.ldmask = s.ldmask;
        d.ta = s.ta; d.tb = s.tb; d.act = s.act; d.mact = s.mact; d.ones = s.ones; d.ks = ks;
        if (s.C2 && (!s.dvec || ks > 1 || s.ones || !s.C)) return lfail(who + "dual output needs dvec, C, no split / ones");
        d.dvec = s.dvec; d.C2 = s.C2; d.dscale = s.dscale;
        const int tm = (s.M + 15) / 16, tn = (s.N + 15) / 16;
        d.tiles_n = tn;
        // long chains over few tiles: four waves per tile (K quarters, LDS reduction), the tile's
        // waves aligned to one workgroup
        const int steps = ((s.K + 3) / 4 + ks - 1) / ks;
        d.kw = (g_kw4 && steps >= g_kw4_steps && (int64_t)tm * tn * ks <= g_kw4_tiles) ? 4 : 1;
        if (d.kw == 4) waves = (waves + 3) / 4 * 4;
        d.w_begin = (int)waves;
        waves += (int64_t)tm * tn * ks * d.kw;
        if (waves > (1 << 26)) return lfail(who + "too many tiles");
    }
    g.waves = (int)waves;
    hipLaunchKernelGGL(gemm64_kernel, dim3((g.waves + 3) / 4), dim3(256), 0, (hipStream_t)stream, g);
    LHIP(hipGetLastError());
    return 0;
}

int aac_uam_push(double *ring, int64_t capacity, int64_t pos, int64_t M, const double *own, const double *radar,
                 const double *act, const double *rew, const void *done, int32_t done_u8, const double *nown,
                 const double *nradar, int64_t *meta, int64_t size, void *stream) {
    if (M <= 0) return 0;
    if (!ring || !own || !radar || !act || !rew || !done || !nown || !nradar) return lfail("uam_push: NULL argument");
    if (M > capacity || pos < 0 || pos >= capacity) return lfail("uam_push: M > capacity or pos out of range");
    if (M >= (int64_t)1 << 30) return lfail("uam_push: too many rows in one push");
    const int64_t np = (pos + M) % capacity, ns = std::min<int64_t>(size + M, capacity);
    hipLaunchKernelGGL(uam_push_kernel, dim3((unsigned)((M + PR - 1) / PR)), dim3(256), 0, (hipStream_t)stream, ring,
                       capacity, pos, (int)M, own, radar, act, rew, done, done_u8, nown, nradar, meta, np, ns,
                       (const int64_t *)nullptr, (int64_t *)nullptr);
    LHIP(hipGetLastError());
    return 0;
}

int aac_uam_push_io(double *ring, int64_t capacity, int64_t M, const double *own, const double *radar,
                    const double *act, const double *rew, const void *done, int32_t done_u8, const double *nown,
                    const double *nradar, int64_t *meta, const int64_t *pos_in, int64_t *pos_out, void *stream) {
    if (M <= 0) return 0;
    if (!ring || !own || !radar || !act || !rew || !done || !nown || !nradar || !meta || !pos_in || !pos_out)
        return lfail("uam_push_io: NULL argument");
    if (pos_in == pos_out) return lfail("uam_push_io: pos_in and pos_out must be two distinct words");
    if (M > capacity) return lfail("uam_push_io: M > capacity");
    if (M >= (int64_t)1 << 30) return lfail("uam_push_io: too many rows in one push");
    hipLaunchKernelGGL(uam_push_kernel, dim3((unsigned)((M + PR - 1) / PR)), dim3(256), 0, (hipStream_t)stream, ring,
                       capacity, (int64_t)0, (int)M, own, radar, act, rew, done, done_u8, nown, nradar, meta,
                       (int64_t)0, (int64_t)0, pos_in, pos_out);
    LHIP(hipGetLastError());
    return 0;
}

int aac_uam_gather(const double *ring, const int32_t *idx, int32_t B, double *rows, double *xc, double *xt, double *xp,
                   void *stream) {
    if (B <= 0) return 0;
    if (!ring || !idx || !rows || !xc || !xt || !xp) return lfail("uam_gather: NULL argument");
    hipLaunchKernelGGL(uam_gather_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, ring, idx, B, rows, xc, xt, xp);
    LHIP(hipGetLastError());
    return 0;
}

int aac_uam_head(const double *h, int32_t B, const double *w, const double *b, int32_t mode, double *y,
                 const double *rew, const double *done, int32_t ldr, double gamma, double *dq, double *dh,
                 double *lterm, void *stream) {
    if (B <= 0) return 0;
    if (!h || !w || !b || !y || mode < 0 || mode > 2) return lfail("uam_head: NULL argument or bad mode");
    if (mode == 2 && (!rew || !done)) return lfail("uam_head: mode 2 needs rew / done");
    if (mode < 2 && (!dh || !lterm)) return lfail("uam_head: modes 0 / 1 need dh / lterm");
    hipLaunchKernelGGL(uam_head_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, h, B, w, b, mode, y, rew,
                       done, ldr, gamma, dq, dh, lterm);
    LHIP(hipGetLastError());
    return 0;
}

int aac_uam_td_mse_head(const double *ht, const double *wt, const double *bt, const double *rew, const double *done,
                        int32_t ldr, double gamma, double *y, const double *h, const double *w, const double *b,
                        int32_t B, double *dq, double *dh, double *lterm, void *stream) {
    if (B <= 0) return 0;
    if (!ht || !wt || !bt || !rew || !done || !y || !h || !w || !b || !dh || !lterm)
        return lfail("uam_td_mse_head: bad argument");
    hipLaunchKernelGGL(uam_td_mse_head_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, ht, wt, bt, rew,
                       done, ldr, gamma, y, h, w, b, B, dq, dh, lterm);
    LHIP(hipGetLastError());
    return 0;
}

int aac_adam64_sum(double *param, const double *gpart, int32_t nsplit, double *exp_avg, double *exp_avg_sq, int64_t n,
                   double lr, double beta1, double beta2, double eps, const int32_t *step, int32_t step_add,
                   void *stream) {
    return aac_adam64_sum_scaled(param, gpart, nsplit, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, step, step_add,
                                 1.0, stream);
}

int aac_adam64_sum_scaled(double *param, const double *gpart, int32_t nsplit, double *exp_avg, double *exp_avg_sq,
                          int64_t n, double lr, double beta1, double beta2, double eps, const int32_t *step,
                          int32_t step_add, double gscale, void *stream) {
    if (n <= 0) return 0;
    if (nsplit < 1 || !param || !gpart || !exp_avg || !exp_avg_sq || !step) return lfail("adam64_sum: bad argument");
    hipLaunchKernelGGL(adam64_kernel, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, param, gpart, nsplit,
                       exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, step, step_add, gscale);
    LHIP(hipGetLastError());
    return 0;
}

int aac_sum64_partials(double *out, const double *gpart, int32_t nsplit, int64_t n, void *stream) {
    if (n <= 0) return 0;
    if (nsplit < 1 || !out || !gpart) return lfail("sum64_partials: bad argument");
    hipLaunchKernelGGL(sum64_kernel, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, out, gpart, nsplit, n);
    LHIP(hipGetLastError());
    return 0;
}

int aac_uam_polyak(double *target, const double *src, int64_t n, double tau, int32_t *step, const double *lq,
                   const double *la, int32_t B, double *loss, void *stream) {
    if (n <= 0 || !target || !src) return lfail("uam_polyak: bad argument");
    hipLaunchKernelGGL(uam_polyak_kernel, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, target, src, n, tau,
                       step, lq, la, B, loss);
    LHIP(hipGetLastError());
    return 0;
}

}  // extern "C"
