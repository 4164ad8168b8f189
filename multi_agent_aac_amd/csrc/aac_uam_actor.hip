// aac_uam_actor.hip -- the UAM learner's batched choose_action on the fp64 matrix cores
// (include/aac_uam.h ``aac_uam_actor``).
//
// ActorNetwork_TwoPortion (UAM/nets:167-190) in float64 for every aircraft of every env, then the
// exploration noise of choose_action (UAM/maddpg:597-676: act + randn * var, clamp to [-1, 1],
// var = get_custom_linear_scaling_factor of the env's own episode, UAM/maddpg:1399-1406):
//   h_o = relu(W1 own + b1) (7 -> 64), h_r = relu(W2 radar + b2) (18 -> 64),
//   h = relu(W3 [h_o | h_r] + b3) (128 -> 128), a = tanh(W4 h + b4) (128 -> 2).
// One wave per 16-row block: v_mfma_f64_16x16x4_f64 for the three wide layers (A fragments of
// the input rows from global memory, then from the wave's LDS slab of [h_o | h_r]; B fragments
// of the weights from L1 / L2, shared by four column tiles at a time so four accumulators are
// in flight), the 128 -> 2 output layer as per-lane partial dots reduced over the 16 lanes that
// hold one row.  The torch form of the same forward is ~13 launches with 64- and 128-wide
// float64 intermediates in HBM.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <string>

#include "../../include/aac_uam.h"
#include "aac_noise.h"
#include "aac_wave.h"

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int HLD = 132;     // LDS row stride (doubles) of a wave's 16 x 128 hidden slab

thread_local std::string g_aerr;
// 16-row tiles per block of the weights-stationary actor (aac_uam_actor_set_tiles; AAC_UAM_ACTOR_NT)
int g_actor_nt = [] {
    const char *v = getenv("AAC_UAM_ACTOR_NT");
    const int k = v ? atoi(v) : 4;
    return (k == 1 || k == 2 || k == 4) ? k : 4;
}();

__host__ __device__ inline uint64_t amix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct ActorArgs {
    const double *own, *radar, *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4;
    double *out;
    int R, N;
    const int32_t *episode;
    int eps_end, noisy;
    double noise_start, noise_end;
    uint64_t seed;
    uint64_t *counter;          // epoch | arrivals << 32 (aacn::take_epoch): advanced by the launch
};

// C tile of one 16-wide column block of a layer with K-contiguous weight rows W[o][k]: A
// fragments from ``a_of(k)`` (this lane's row l & 15), four column tiles at once
template <int KSTEPS, typename AF>
__device__ __forceinline__ void layer4(const double *W, int ldw, int K, int o0, int lane, AF a_of, d4 acc[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
    const int kl = lane >> 4, ol = lane & 15;
#pragma unroll 4
    for (int s = 0; s < KSTEPS; ++s) {
        const int k = 4 * s + kl;
        const double a = a_of(k);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double b = k < K ? W[(size_t)(o0 + 16 * c + ol) * ldw + k] : 0.0;
            acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
        }
    }
}

__global__ void __launch_bounds__(256) uam_actor_kernel(ActorArgs A) {
    __shared__ double slab[4][16 * HLD];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double *H = slab[w];
    const int rl = lane & 15, kl = lane >> 4;
    const uint64_t ctr = A.noisy ? aacn::take_epoch(A.counter) : 0;
    const int nblk = (A.R + 15) / 16;
    for (int blk = blockIdx.x * 4 + w; blk < nblk; blk += gridDim.x * 4) {
        // the slab is rewritten below; this wave's reads of the previous block come first (the
        // LDS executes one wave's instructions in order, the clobber keeps the compiler's order)
        asm volatile("" ::: "memory");
        const int r0 = blk * 16;
        const int ra = r0 + rl;                      // this lane's A row
        const bool rin = ra < A.R;
        d4 acc[4];
        // h_o = relu(W1 own + b1): K = 7 (2 steps), 64 outputs = four column tiles
        layer4<2>(A.w1, 7, 7, 0, lane, [&](int k) { return (rin && k < 7) ? A.own[(size_t)ra * 7 + k] : 0.0; }, acc);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = 16 * c + rl;
                const double v = acc[c][j] + A.b1[col];
                H[(kl + 4 * j) * HLD + col] = v > 0.0 ? v : 0.0;
            }
        // h_r = relu(W2 radar + b2): K = 18 (5 steps)
        layer4<5>(A.w2, 18, 18, 0, lane, [&](int k) { return (rin && k < 18) ? A.radar[(size_t)ra * 18 + k] : 0.0; },
                  acc);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = 16 * c + rl;
                const double v = acc[c][j] + A.b2[col];
                H[(kl + 4 * j) * HLD + 64 + col] = v > 0.0 ? v : 0.0;
            }
        asm volatile("" ::: "memory");      // slab writes before the other lanes' A reads
        // h = relu(W3 [h_o | h_r] + b3) in two passes of four column tiles; the output layer's
        // partial dots p[o][j] (row kl + 4 j) accumulate over this lane's 8 columns
        double p0[4] = {0.0, 0.0, 0.0, 0.0}, p1[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            layer4<32>(A.w3, 128, 128, 64 * half, lane, [&](int k) { return H[rl * HLD + k]; }, acc);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int col = 64 * half + 16 * c + rl;
                const double bb = A.b3[col], u0 = A.w4[col], u1 = A.w4[128 + col];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    double v = acc[c][j] + bb;
                    v = v > 0.0 ? v : 0.0;
                    p0[j] = fma(u0, v, p0[j]);
                    p1[j] = fma(u1, v, p1[j]);
                }
            }
        }
        // reduce over the 16 lanes of a row group (lane & 15), then lane (rl = 0) of group kl
        // finishes rows kl + 4 j
#pragma unroll
        for (int m = 1; m < 16; m <<= 1)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                p0[j] += __shfl_xor(p0[j], m, 64);
                p1[j] += __shfl_xor(p1[j], m, 64);
            }
        if (rl < 4) {
            // lane rl of group kl writes row kl + 4 rl (selects, not a dynamic register index)
            const double s0 = rl == 0 ? p0[0] : (rl == 1 ? p0[1] : (rl == 2 ? p0[2] : p0[3]));
            const double s1 = rl == 0 ? p1[0] : (rl == 1 ? p1[1] : (rl == 2 ? p1[2] : p1[3]));
            const int r = r0 + kl + 4 * rl;
            if (r < A.R) {
                double a0 = tanh(s0 + A.b4[0]), a1 = tanh(s1 + A.b4[1]);
                if (A.noisy) {
                    const int e = r / A.N;
                    const int ep = A.episode ? A.episode[e] : 1;
                    double var;
                    if (ep <= A.eps_end) {
                        const double slope = (A.noise_end - A.noise_start) / (double)(A.eps_end - 1);
                        var = A.noise_start + slope * (double)(ep - 1);
                    } else {
                        var = A.noise_end;
                    }
                    const uint64_t h1 = amix64(amix64(amix64(A.seed) ^ ctr) ^ (uint64_t)(2 * (int64_t)r));
                    const uint64_t h2 = amix64(h1 ^ 0xD1B54A32D192ED03ull);
                    const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);   // (0, 1]
                    const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
                    const double rr = sqrt(-2.0 * log(u1));
                    a0 = fmin(fmax(a0 + rr * cos(6.283185307179586 * u2) * var, -1.0), 1.0);
                    a1 = fmin(fmax(a1 + rr * sin(6.283185307179586 * u2) * var, -1.0), 1.0);
                }
                A.out[2 * (size_t)r] = a0;
                A.out[2 * (size_t)r + 1] = a1;
            }
        }
    }
}

// Weights-stationary form (the default): a workgroup keeps every weight fragment it needs in
// registers and walks 16-row blocks.  The layers run transposed (h^T = W x^T, the block's rows on
// the MFMA's n axis; A = weight fragments, B = activations), so wave w owns output features
// 16w..16w+15 of the two 64-wide encoders and 32w..32w+31 of the 128-wide merge layer, and the
// activations pass between layers through a [feature][row] LDS image.  The per-block form above
// re-reads the 128 KB merge weights from L2 for every 16 rows (~1 GB per launch at 131 072 rows).
constexpr int TI = 17;                       // row stride of the [feature][16 rows] image

__device__ __forceinline__ double row_noise(const ActorArgs &A, int r, uint64_t ctr, double &n1) {
    const int e = r / A.N;
    const int ep = A.episode ? A.episode[e] : 1;
    double var;
    if (ep <= A.eps_end) {
        const double slope = (A.noise_end - A.noise_start) / (double)(A.eps_end - 1);
        var = A.noise_start + slope * (double)(ep - 1);
    } else {
        var = A.noise_end;
    }
    const uint64_t h1 = amix64(amix64(amix64(A.seed) ^ ctr) ^ (uint64_t)(2 * (int64_t)r));
    const uint64_t h2 = amix64(h1 ^ 0xD1B54A32D192ED03ull);
    const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);   // (0, 1]
    const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
    const double rr = sqrt(-2.0 * log(u1));
    n1 = rr * sin(6.283185307179586 * u2) * var;
    return rr * cos(6.283185307179586 * u2) * var;
}

// NT 16-row tiles per block (the rows of the block on the MFMA's n axis, NT independent accumulator
// chains per weight fragment): each merge-layer weight fragment held in registers feeds NT MFMAs per
// k step, so the block's latency chain (loads, two barriers, the 32-step merge chain, the output
// reduction, the noise) is paid once per 16 NT rows.  NT = 1 was the first form: ~10 k cycles per
// 16 rows at one wave per SIMD.  Every row's arithmetic is the same for any NT (bit-identical).
// AAC_UAM_ACT_PF (default 1): the next block's own / radar rows are loaded while this block's merge
// chain runs (spare registers of the one-wave-per-SIMD launch; LDS-only barriers keep them in flight),
// and the exploration noise of the workgroup's first NBN blocks is drawn up front into LDS by all 256
// threads (the fp64 Box-Muller off the per-block output stage, which one wave ran after the chain).
// Same arithmetic per row: bit-identical to the form without either.
#ifndef AAC_UAM_ACT_PF
#define AAC_UAM_ACT_PF 1
#endif
#if AAC_UAM_ACT_PF
#define UACT_BARRIER() aacw::lds_barrier()
#else
#define UACT_BARRIER() __syncthreads()
#endif
// AAC_UAM_ACT_EPOCH_END: the noise epoch read with one load at the start and the launch's arrival
// counted at its end (aacn::read_epoch / end_epoch) instead of an atomic round trip before the
// first block (aacn::take_epoch); the same counter sequence
#ifndef AAC_UAM_ACT_EPOCH_END
#define AAC_UAM_ACT_EPOCH_END 1
#endif
constexpr int NBN = 8;      // blocks per workgroup whose noise is drawn up front (config 5: 8 per workgroup)

template <int NT>
__global__ void __launch_bounds__(256) uam_actor_ws_kernel(ActorArgs A) {
    constexpr int ROWS = 16 * NT, TS = ROWS + 1;       // TS: row stride of the [feature][rows] image
    __shared__ double sH[128 * TS];          // [h_o | h_r] of the block, [feature][row]
    __shared__ double sP[4][ROWS][2];        // per-wave partial output dots
    __shared__ double2 sN[AAC_UAM_ACT_PF ? NBN * ROWS : 1];     // up-front noise, [block of the wg][row]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, n = lane & 15, kq = lane >> 4;
    // A fragments (lane: output row 16 t + n of the tile, k slot kq of each 4-step)
    double a1[2], a2[5], a3[2][32];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int k = 4 * s + kq;
        a1[s] = k < 7 ? A.w1[(16 * w + n) * 7 + k] : 0.0;
    }
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int k = 4 * s + kq;
        a2[s] = k < 18 ? A.w2[(16 * w + n) * 18 + k] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 32; ++s) a3[t][s] = A.w3[(32 * w + 16 * t + n) * 128 + 4 * s + kq];
    // epilogue constants of this lane's outputs: feature 16 t + kq + 4 j of a tile (f64 C layout)
    double c1[4], c2[4], c3[2][4], u0[2][4], u1[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        c1[j] = A.b1[16 * w + kq + 4 * j];
        c2[j] = A.b2[16 * w + kq + 4 * j];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int o = 32 * w + 16 * t + kq + 4 * j;
            c3[t][j] = A.b3[o];
            u0[t][j] = A.w4[o];
            u1[t][j] = A.w4[128 + o];
        }
    }
    const double b40 = A.b4[0], b41 = A.b4[1];
    // the launch's noise epoch (one atomic per workgroup), after the weight loads are in flight
    const uint64_t ctr = !A.noisy ? 0 : (AAC_UAM_ACT_EPOCH_END ? aacn::read_epoch(A.counter) : aacn::take_epoch(A.counter));
    const int nblk = (A.R + ROWS - 1) / ROWS;
    auto load_rows = [&](int blk, double (&bo)[NT][2], double (&br)[NT][5]) {
        const int r0 = blk * ROWS;
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            const int r = r0 + 16 * q + n;
            const int rc = r < A.R ? r : A.R - 1;        // rows past R feed only their own column
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int k = 4 * s + kq;
                bo[q][s] = A.own[(size_t)rc * 7 + (k < 7 ? k : 6)];
            }
#pragma unroll
            for (int s = 0; s < 5; ++s) {
                const int k = 4 * s + kq;
                br[q][s] = A.radar[(size_t)rc * 18 + (k < 18 ? k : 17)];
            }
        }
    };
    double bo[NT][2], br[NT][5];
    if (AAC_UAM_ACT_PF && (int)blockIdx.x < nblk) load_rows(blockIdx.x, bo, br);
    if (AAC_UAM_ACT_PF && A.noisy) {
        for (int i = threadIdx.x; i < NBN * ROWS; i += 256) {
            const int bi = i / ROWS, x = i - bi * ROWS;
            const int rr = (blockIdx.x + bi * gridDim.x) * ROWS + x;
            if (rr < A.R) {
                double e1;
                const double e0 = row_noise(A, rr, ctr, e1);
                sN[i] = make_double2(e0, e1);
            }
        }
    }
    for (int blk = blockIdx.x, bi = 0; blk < nblk; blk += gridDim.x, ++bi) {
        const int r0 = blk * ROWS;
        double nbo[NT][2], nbr[NT][5];
        if (!AAC_UAM_ACT_PF) load_rows(blk, bo, br);
        else if (blk + (int)gridDim.x < nblk) load_rows(blk + gridDim.x, nbo, nbr);
        // h_o^T = relu(W1 own^T + b1), h_r^T = relu(W2 radar^T + b2): padded k slots have a zero A
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 2; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s], bo[q][s], acc, 0, 0, 0);
            d4 acr = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 5; ++s) acr = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s], br[q][s], acr, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const double v = acc[j] + c1[j];
                sH[(16 * w + kq + 4 * j) * TS + 16 * q + n] = v > 0.0 ? v : 0.0;
                const double u = acr[j] + c2[j];
                sH[(64 + 16 * w + kq + 4 * j) * TS + 16 * q + n] = u > 0.0 ? u : 0.0;
            }
        }
        UACT_BARRIER();
        // h^T = relu(W3 [h_o | h_r]^T + b3), two output tiles per wave and NT row tiles, then this
        // lane's share of the 128 -> 2 output layer
        d4 h0[NT], h1[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            h0[q] = d4{0.0, 0.0, 0.0, 0.0};
            h1[q] = d4{0.0, 0.0, 0.0, 0.0};
        }
#pragma unroll
        for (int s = 0; s < 32; ++s) {
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                const double b = sH[(4 * s + kq) * TS + 16 * q + n];
                h0[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a3[0][s], b, h0[q], 0, 0, 0);
                h1[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a3[1][s], b, h1[q], 0, 0, 0);
            }
        }
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            double p0 = 0.0, p1 = 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double v = h0[q][j] + c3[0][j];
                v = v > 0.0 ? v : 0.0;
                p0 = fma(u0[0][j], v, p0);
                p1 = fma(u1[0][j], v, p1);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double v = h1[q][j] + c3[1][j];
                v = v > 0.0 ? v : 0.0;
                p0 = fma(u0[1][j], v, p0);
                p1 = fma(u1[1][j], v, p1);
            }
            // sum over the four lane groups that hold row n, then (below) over the waves in order
            p0 += __shfl_xor(p0, 16, 64);
            p1 += __shfl_xor(p1, 16, 64);
            p0 += __shfl_xor(p0, 32, 64);
            p1 += __shfl_xor(p1, 32, 64);
            if (kq == 0) {
                sP[w][16 * q + n][0] = p0;
                sP[w][16 * q + n][1] = p1;
            }
        }
        UACT_BARRIER();
        for (int x = threadIdx.x; x < ROWS; x += 256) {
            const int rr = r0 + x;
            if (rr < A.R) {
                const double s0 = ((sP[0][x][0] + sP[1][x][0]) + sP[2][x][0]) + sP[3][x][0];
                const double s1 = ((sP[0][x][1] + sP[1][x][1]) + sP[2][x][1]) + sP[3][x][1];
                double x0 = tanh(s0 + b40), x1 = tanh(s1 + b41);
                if (A.noisy) {
                    double e0, e1;
                    if (AAC_UAM_ACT_PF && bi < NBN) {
                        const double2 z = sN[bi * ROWS + x];
                        e0 = z.x;
                        e1 = z.y;
                    } else {
                        e0 = row_noise(A, rr, ctr, e1);
                    }
                    x0 = fmin(fmax(x0 + e0, -1.0), 1.0);
                    x1 = fmin(fmax(x1 + e1, -1.0), 1.0);
                }
                A.out[2 * (size_t)rr] = x0;
                A.out[2 * (size_t)rr + 1] = x1;
            }
        }
        if (AAC_UAM_ACT_PF) {
#pragma unroll
            for (int q = 0; q < NT; ++q) {
#pragma unroll
                for (int s = 0; s < 2; ++s) bo[q][s] = nbo[q][s];
#pragma unroll
                for (int s = 0; s < 5; ++s) br[q][s] = nbr[q][s];
            }
        }
    }
    if (AAC_UAM_ACT_EPOCH_END && A.noisy) aacn::end_epoch(A.counter, ctr);
}

}  // namespace

extern "C" {

const char *aac_uam_actor_last_error(void) { return g_aerr.c_str(); }

int aac_uam_actor_set_tiles(int32_t nt) {
    if (nt != 1 && nt != 2 && nt != 4) {
        g_aerr = "aac_uam_actor_set_tiles: 1, 2 or 4 row tiles per block";
        return AAC_E_INVALID;
    }
    g_actor_nt = nt;
    return 0;
}

int aac_uam_actor(const double *own, const double *radar, int32_t R, const double *w1, const double *b1,
                  const double *w2, const double *b2, const double *w3, const double *b3, const double *w4,
                  const double *b4, double *out, int32_t N, const int32_t *episode, int32_t eps_end,
                  double noise_start, double noise_end, uint64_t seed, uint64_t *counter, int32_t noisy,
                  void *stream) {
    if (R <= 0) return 0;
    if (!own || !radar || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !w4 || !b4 || !out || N <= 0) {
        g_aerr = "aac_uam_actor: null argument or N <= 0";
        return AAC_E_INVALID;
    }
    if (noisy && (!counter || eps_end < 2)) {
        g_aerr = "aac_uam_actor: noisy needs a counter and eps_end >= 2";
        return AAC_E_INVALID;
    }
    ActorArgs A{own, radar, w1, b1, w2, b2, w3, b3, w4, b4, out, R, N, episode, eps_end, noisy ? 1 : 0,
                noise_start, noise_end, seed, counter};
    const int nblk = (R + 15) / 16;
    static const int per_block = [] {
        const char *v = getenv("AAC_UAM_ACTOR_V1");
        return v && atoi(v) != 0;
    }();
    if (per_block) {
        int wgs = (nblk + 3) / 4;
        wgs = wgs > 2048 ? 2048 : wgs;
        hipLaunchKernelGGL(uam_actor_kernel, dim3(wgs), dim3(256), 0, (hipStream_t)stream, A);
    } else {
        static const int cap = [] {
            const char *v = getenv("AAC_UAM_ACTOR_WGS");
            return v ? atoi(v) : 256;     // one workgroup per CU (> 256 VGPRs: one wave per SIMD)
        }();
        const int nt = g_actor_nt;
        const int nb = (R + 16 * nt - 1) / (16 * nt);
        const int wgs = nb < cap ? nb : cap;
        switch (nt) {
            case 1: hipLaunchKernelGGL(uam_actor_ws_kernel<1>, dim3(wgs), dim3(256), 0, (hipStream_t)stream, A); break;
            case 2: hipLaunchKernelGGL(uam_actor_ws_kernel<2>, dim3(wgs), dim3(256), 0, (hipStream_t)stream, A); break;
            default: hipLaunchKernelGGL(uam_actor_ws_kernel<4>, dim3(wgs), dim3(256), 0, (hipStream_t)stream, A); break;
        }
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_aerr = std::string("aac_uam_actor: ") + hipGetErrorString(e);
        return AAC_E_HIP;
    }
    return 0;
}

}  // extern "C"
