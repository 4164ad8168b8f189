// aac_gru.hip -- GRU-cell row kernel of the GRU-actor MADDPG (include/aac_gru.h).
//
// One wave per row, lane u = hidden unit (H = 64).  Per row the wave reads gi, gh (2 x 768 B) and
// h (256 B), evaluates the three gates in torch's GRUCell order (ATen gru_cell: the reset and
// update gates from gh + gi, the new gate as gi_n + gh_n * r, h' = (h - n) z + n), the O-unit
// output layer by DPP wave sums, and, by mode, the loss gradient and the gate backward:
//   dn = dh' - dh' z,  dz = dh' (h - n),  da_n = dn (1 - n^2),  dr = da_n gh_n,
//   da_r = dr r (1 - r),  da_z = dz z (1 - z)
//   dgi = [da_r, da_z, da_n],  dgh = [da_r, da_z, da_n r]
// so a training step of all N agents' GRU cells is one launch per direction, and the input
// projections / weight gradients stay grouped MFMA GEMMs.  HBM-bound: ~2 KB read per row.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/aac_gru.h"
#include "aac_wave.h"
#include "aac_noise.h"

namespace {

thread_local std::string g_err;

int gfail(const std::string &m) {
    g_err = m;
    return -1;
}

using aacw::wsum;

constexpr int H = AAC_GRU_HIDDEN;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// one row r of aac_gru_cell (one wave, lane u = hidden unit).  tgt_in: the CRITIC target of this
// row in a register (a chained launch) instead of a.target[r]; returns the TD value (TD mode) to
// every lane
__device__ __forceinline__ float cell_row(const aac_gru_args &a, int r, int u, const float *tgt_in) {
    float td = 0.0f;
    const float *gi = a.gi + (size_t)r * a.ldg, *gh = a.gh + (size_t)r * a.ldg;
    const float ir = gi[u], iz = gi[H + u], in = gi[2 * H + u];
    const float hr = gh[u], hz = gh[H + u], hn = gh[2 * H + u];
    const float hv = a.h[(size_t)r * a.ldh + u];
    const float rg = sigm(hr + ir);
    const float zg = sigm(hz + iz);
    const float ng = tanhf(in + hn * rg);
    const float hp = (hv - ng) * zg + ng;
    const int agent = r % a.N;
    const float *W = a.wout + (size_t)agent * a.wstride;
    const float *b = a.bout + (size_t)agent * a.bstride;
    const bool two = a.O == 2;          // wave-uniform; O is 1 or 2
    float y0 = wsum(W[u] * hp) + b[0];
    float y1 = two ? wsum(W[H + u] * hp) + b[1] : 0.0f;
    if (a.act == 2) {
        y0 = tanhf(y0);
        y1 = tanhf(y1);
    }
    if (a.hout) a.hout[(size_t)r * a.ldho + u] = hp;
    float dh;
    if (a.mode == AAC_GRU_FWD) {
        const float yu = u == 0 ? y0 : y1;
        if (a.y && u < a.O) a.y[(size_t)r * a.ldy + u] = yu;
        if (a.pack_dst) {
            float *d = a.pack_dst + (size_t)r * a.ld_pack_dst;
            if (u < a.npack) d[u] = a.pack_src[(size_t)r * a.ld_pack_src + u];
            if (u < a.O) d[a.npack + u] = yu;
        }
        return td;
    }
    if (a.mode == AAC_GRU_TD) {
        td = a.rew[r] + (a.gamma * y0) * (1.0f - a.done[r]);
        if (u == 0) a.yout[r] = td;
        return td;
    }
    if (a.mode == AAC_GRU_CRITIC || a.mode == AAC_GRU_ACTLOSS) {
        const float tg = a.mode == AAC_GRU_CRITIC ? (tgt_in ? *tgt_in : a.target[r]) : 0.0f;
        const float g = a.mode == AAC_GRU_CRITIC ? (2.0f * a.inv_m) * (y0 - tg) : -a.inv_m;
        if (u == 0) {
            if (a.y) a.y[r] = y0;
            if (a.dq) a.dq[r] = g;
        }
        dh = g * W[u];
    } else {   // AAC_GRU_ACTBWD: tanh output layer backward
        float da0, da1 = 0.0f;
        if (a.dsa) {      // d a = dsa . W_sa[:, col:col+2] of this row's agent (lane u = k)
            const float s = a.dsa[(size_t)r * a.lddsa + u];
            const float *ws = a.wsa + (size_t)agent * a.wsa_stride + (size_t)u * a.ldwsa + a.wsa_col;
            da0 = wsum(s * ws[0]);
            if (two) da1 = wsum(s * ws[1]);
        } else {
            da0 = a.da[(size_t)r * a.ldda];
            if (two) da1 = a.da[(size_t)r * a.ldda + 1];
        }
        const float d0 = da0 * (1.0f - y0 * y0);
        dh = d0 * W[u];
        if (u == 0) a.dq[(size_t)r * a.O] = d0;
        if (two) {
            const float d1 = da1 * (1.0f - y1 * y1);
            dh = fmaf(d1, W[H + u], dh);
            if (u == 0) a.dq[(size_t)r * a.O + 1] = d1;
        }
    }
    const float dn = dh - dh * zg;
    const float dz = dh * (hv - ng);
    const float dan = dn * (1.0f - ng * ng);
    const float dr = dan * hn;
    const float dar = dr * (1.0f - rg) * rg;
    const float daz = dz * (1.0f - zg) * zg;
    float *dgi = a.dgi + (size_t)r * a.ldd;
    dgi[u] = dar;
    dgi[H + u] = daz;
    dgi[2 * H + u] = dan;
    if (a.dgh) {
        float *dgh = a.dgh + (size_t)r * a.ldd;
        dgh[u] = dar;
        dgh[H + u] = daz;
        dgh[2 * H + u] = dan * rg;
    }
    return td;
}

__global__ void __launch_bounds__(256) gru_cell_kernel(aac_gru_args a) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= a.R) return;
    cell_row(a, r, threadIdx.x & 63, nullptr);
}

// two argument sets in one launch: independent (chain 0: set k takes workgroups [k G, (k + 1) G)) or
// chained per row (chain 1: set 0 in TD mode, then set 1 in CRITIC mode on the same row with the TD
// value from the register -- the TD target and the critic's mse head of one update, WGRU/maddpg:280-291)
struct GruCellPair {
    aac_gru_args s0, s1;
    int chain;
};
__global__ void __launch_bounds__(256) gru_cell2_kernel(GruCellPair P) {
    const int u = threadIdx.x & 63;
    if (P.chain) {
        const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
        if (r >= P.s0.R) return;
        const float td = cell_row(P.s0, r, u, nullptr);
        cell_row(P.s1, r, u, &td);
        return;
    }
    const int g0 = (P.s0.R + 3) / 4;
    if ((int)blockIdx.x < g0) {
        const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
        if (r < P.s0.R) cell_row(P.s0, r, u, nullptr);
    } else {
        const int r = (blockIdx.x - g0) * 4 + (threadIdx.x >> 6);
        if (r < P.s1.R) cell_row(P.s1, r, u, nullptr);
    }
}

// ------------------------------------------------------------ weights-stationary actor forward
// The act path of config 4 (E x N rows, every agent its own network): a workgroup takes one agent
// and walks blocks of 16 NT envs; wave w owns hidden units 16w .. 16w + 15.  The layers run
// transposed on v_mfma_f32_16x16x4_f32 (y^T = W x^T: A = weight fragments held in registers for the
// whole launch, B = activations, the block's rows on the n axis), so lane (n, kq) ends with units
// 16w + 4kq .. + 3 of row n of each gate -- all six gate pre-activations of a unit meet in one lane
// and the GRU cell runs in registers.  The encoders' outputs pass to the input projection through a
// [feature][row] LDS image; the output layer's partial dots through LDS in a fixed wave order.
typedef float f4 __attribute__((ext_vector_type(4)));
// GNT 16-row tiles per block (2 for the act path; 1 for the projection mode at B = 512 rows per agent,
// so that every CU gets a workgroup); PROJ: write cat / gi / gh, no cell.
// Up to GMAX argument sets per launch (projection mode: independent network evaluations of one
// update_myown, e.g. the target actor on s', the critic on (s, a) and the actor on s): blocks of set
// k are [k G N, (k + 1) G N).
constexpr int GMAX = 3;
struct GruActorBatch {
    aac_gru_actor_args s[GMAX];
    int n;
};
template <int GNT, bool PROJ>
__global__ void __launch_bounds__(256) gru_actor_fwd_kernel(GruActorBatch Pb) {
    const int per = gridDim.x / Pb.n;                        // workgroups per set
    const int set = (int)blockIdx.x / per, bx = (int)blockIdx.x - set * per;
    // the set's arguments by value, selected with uniform branches (indexing the by-value kernel
    // argument would move it to scratch)
    const aac_gru_actor_args A = set == 0 ? Pb.s[0] : (set == 1 ? Pb.s[1] : Pb.s[2]);
    constexpr int GROWS = 16 * GNT, GTS = GROWS + 1;
    __shared__ float sCat[128 * GTS];         // [e_o | e_g] of the block, [feature][row]
    __shared__ float sP[4][GROWS][2];         // per-wave partial output dots
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, n = lane & 15, kq = lane >> 4;
    const int G = per / A.N;                  // workgroups per agent
    const int ag = bx / G, g = bx - ag * G;
    const size_t po = (size_t)ag * A.pstride;
    const float *Wo = A.Wo + po, *Wg = A.Wg + po, *Wih = A.Wih + po, *Whh = A.Whh + po, *Wout = A.Wout + po;
    const int d = A.d_own;
    // A fragments: lane (n, kq) holds W[feature 16t + n][k] for its k of step s.  The encoders take
    // k = 4s + kq; the input projections k = 32 kq + s (W_ih) and 16 kq + s (W_hh), the same k order
    // on the B side, so that a lane's weights and h values are consecutive floats (16-B loads: the
    // 4-B form issued ~190 loads per wave against a limit of 63 in flight)
    float ao[2], ag5[5], ai[3][32], ah[3][16];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int k = 4 * s + kq;
        ao[s] = k < d ? Wo[(16 * w + n) * d + k] : 0.0f;
    }
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int k = 4 * s + kq;
        ag5[s] = k < 18 ? Wg[(16 * w + n) * 18 + (k < 18 ? k : 0)] : 0.0f;
    }
#pragma unroll
    for (int gt = 0; gt < 3; ++gt) {
        const f4 *wi = reinterpret_cast<const f4 *>(Wih + (64 * gt + 16 * w + n) * 128 + 32 * kq);
        const f4 *wh = reinterpret_cast<const f4 *>(Whh + (64 * gt + 16 * w + n) * 64 + 16 * kq);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const f4 v = wi[j];
#pragma unroll
            for (int c = 0; c < 4; ++c) ai[gt][4 * j + c] = v[c];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f4 v = wh[j];
#pragma unroll
            for (int c = 0; c < 4; ++c) ah[gt][4 * j + c] = v[c];
        }
    }
    // epilogue constants of this lane's features 16w + 4kq + v (f32 C layout)
    const int u0 = 16 * w + 4 * kq;
    f4 cbo, cbg, cbi[3], cbh[3], wo0, wo1;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        cbo[v] = A.bo[po + u0 + v];
        cbg[v] = A.bg[po + u0 + v];
#pragma unroll
        for (int gt = 0; gt < 3; ++gt) {
            cbi[gt][v] = A.bih[po + 64 * gt + u0 + v];
            cbh[gt][v] = A.bhh[po + 64 * gt + u0 + v];
        }
        wo0[v] = PROJ ? 0.0f : Wout[u0 + v];
        wo1[v] = PROJ ? 0.0f : Wout[64 + u0 + v];
    }
    const float bout0 = PROJ ? 0.0f : A.bout[po], bout1 = PROJ ? 0.0f : A.bout[po + 1];
    const uint64_t ctr = (!PROJ && A.noisy) ? aacn::take_epoch(A.counter) : 0;     // one epoch per launch
    // the noise of the workgroup's first GNB blocks, one row per thread up front (its fp64 Box-Muller
    // beside the weight loads instead of 32 threads per block on the output stage's chain)
    constexpr int GNB = 256 / GROWS;
    __shared__ float2 sN[PROJ ? 1 : GNB][PROJ ? 1 : GROWS];
    if (!PROJ && A.noisy) {
        const int bi = threadIdx.x / GROWS, x = threadIdx.x - bi * GROWS;
        const int e = (g + bi * G) * GROWS + x;
        if (e < A.E) {
            float n0, n1;
            aacn::row_noise((int64_t)e * A.N + ag, A.N, A.episode, A.eps_end, A.noise_start, A.noise_end, A.seed,
                            ctr, n0, n1);
            sN[bi][x] = make_float2(n0, n1);
        }
    }
    const int nblk = (A.E + GROWS - 1) / GROWS;
    for (int blk = g, bi = 0; blk < nblk; blk += G, ++bi) {
        const int e0 = blk * GROWS;
        float bo_[GNT][2], br[GNT][5], bh[GNT][16];
        f4 hv[GNT];
#pragma unroll
        for (int q = 0; q < GNT; ++q) {
            const int e = e0 + 16 * q + n;
            const size_t r = (size_t)(e < A.E ? e : A.E - 1) * A.N + ag;    // rows past E: their own column only
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int k = 4 * s + kq;
                bo_[q][s] = A.own[r * A.ld_own + (k < d ? k : 0)];
            }
#pragma unroll
            for (int s = 0; s < 5; ++s) {
                const int k = 4 * s + kq;
                br[q][s] = A.radar[r * A.ld_radar + (k < 18 ? k : 0)];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const f4 v = *reinterpret_cast<const f4 *>(A.h + r * A.ldh + 16 * kq + 4 * j);
#pragma unroll
                for (int c = 0; c < 4; ++c) bh[q][4 * j + c] = v[c];
            }
            hv[q] = *reinterpret_cast<const f4 *>(A.h + r * A.ldh + u0);
        }
        // e_o^T = relu(Wo own^T + bo), e_g^T = relu(Wg radar^T + bg) -> sCat (padded k: zero A)
#pragma unroll
        for (int q = 0; q < GNT; ++q) {
            f4 acc = {0.0f, 0.0f, 0.0f, 0.0f}, acr = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < 2; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ao[s], bo_[q][s], acc, 0, 0, 0);
#pragma unroll
            for (int s = 0; s < 5; ++s) acr = __builtin_amdgcn_mfma_f32_16x16x4f32(ag5[s], br[q][s], acr, 0, 0, 0);
            f4 co, cg;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const float x = acc[v] + cbo[v], y = acr[v] + cbg[v];
                co[v] = x > 0.0f ? x : 0.0f;
                cg[v] = y > 0.0f ? y : 0.0f;
                sCat[(u0 + v) * GTS + 16 * q + n] = co[v];
                sCat[(64 + u0 + v) * GTS + 16 * q + n] = cg[v];
            }
            const int e = e0 + 16 * q + n;
            if (PROJ && A.cat && e < A.E) {
                float *c = A.cat + ((size_t)e * A.N + ag) * A.ldc;
                *reinterpret_cast<f4 *>(c + u0) = co;
                *reinterpret_cast<f4 *>(c + 64 + u0) = cg;
            }
        }
        __syncthreads();
        // gi^T = W_ih cat^T, gh^T = W_hh h^T for this wave's units of the three gates
        f4 gi[3][GNT], gh[3][GNT];
#pragma unroll
        for (int gt = 0; gt < 3; ++gt)
#pragma unroll
            for (int q = 0; q < GNT; ++q) {
                gi[gt][q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
                gh[gt][q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
        for (int s = 0; s < 32; ++s)
#pragma unroll
            for (int q = 0; q < GNT; ++q) {
                const float b = sCat[(32 * kq + s) * GTS + 16 * q + n];
#pragma unroll
                for (int gt = 0; gt < 3; ++gt)
                    gi[gt][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ai[gt][s], b, gi[gt][q], 0, 0, 0);
            }
#pragma unroll
        for (int s = 0; s < 16; ++s)
#pragma unroll
            for (int q = 0; q < GNT; ++q)
#pragma unroll
                for (int gt = 0; gt < 3; ++gt)
                    gh[gt][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ah[gt][s], bh[q][s], gh[gt][q], 0, 0, 0);
        if (PROJ) {      // gi / gh rows with their biases, for aac_gru_cell and the weight gradients
#pragma unroll
            for (int q = 0; q < GNT; ++q) {
                const int e = e0 + 16 * q + n;
                if (e >= A.E) continue;
                const size_t r = (size_t)e * A.N + ag;
#pragma unroll
                for (int gt = 0; gt < 3; ++gt) {
                    *reinterpret_cast<f4 *>(A.gi + r * A.ldg + 64 * gt + u0) = gi[gt][q] + cbi[gt];
                    *reinterpret_cast<f4 *>(A.gh + r * A.ldg + 64 * gt + u0) = gh[gt][q] + cbh[gt];
                }
            }
            __syncthreads();      // sCat is rewritten by the next block
            continue;
        }
        // the cell (torch's GRUCell order, as gru_cell_kernel) and this lane's share of the output layer
#pragma unroll
        for (int q = 0; q < GNT; ++q) {
            const int e = e0 + 16 * q + n;
            f4 hp;
            float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const float ir = gi[0][q][v] + cbi[0][v], iz = gi[1][q][v] + cbi[1][v], in = gi[2][q][v] + cbi[2][v];
                const float hr = gh[0][q][v] + cbh[0][v], hz = gh[1][q][v] + cbh[1][v], hn = gh[2][q][v] + cbh[2][v];
                const float rg = sigm(hr + ir);
                const float zg = sigm(hz + iz);
                const float ng = tanhf(in + hn * rg);
                hp[v] = (hv[q][v] - ng) * zg + ng;
                p0 = fmaf(wo0[v], hp[v], p0);
                p1 = fmaf(wo1[v], hp[v], p1);
            }
            if (e < A.E) *reinterpret_cast<f4 *>(A.hout + ((size_t)e * A.N + ag) * A.ldho + u0) = hp;
            p0 += __shfl_xor(p0, 16, 64);
            p1 += __shfl_xor(p1, 16, 64);
            p0 += __shfl_xor(p0, 32, 64);
            p1 += __shfl_xor(p1, 32, 64);
            if (kq == 0) {
                sP[w][16 * q + n][0] = p0;
                sP[w][16 * q + n][1] = p1;
            }
        }
        __syncthreads();
        if (threadIdx.x < GROWS) {
            const int x = threadIdx.x, e = e0 + x;
            if (e < A.E) {
                const float s0 = ((sP[0][x][0] + sP[1][x][0]) + sP[2][x][0]) + sP[3][x][0];
                const float s1 = ((sP[0][x][1] + sP[1][x][1]) + sP[2][x][1]) + sP[3][x][1];
                const size_t row = (size_t)e * A.N + ag;
                float *yo = A.y + row * A.ldy;
                float y0 = tanhf(s0 + bout0), y1 = tanhf(s1 + bout1);
                if (A.noisy) {       // noise_kernel's arithmetic on the stored tanh values
                    float n0, n1;
                    if (bi < GNB) {
                        n0 = sN[bi][x].x;
                        n1 = sN[bi][x].y;
                    } else {
                        aacn::row_noise((int64_t)row, A.N, A.episode, A.eps_end, A.noise_start, A.noise_end, A.seed,
                                        ctr, n0, n1);
                    }
                    y0 = fminf(fmaxf(y0 + n0, -1.0f), 1.0f);
                    y1 = fminf(fmaxf(y1 + n1, -1.0f), 1.0f);
                    if (A.noise_out) {
                        A.noise_out[2 * row] = n0;
                        A.noise_out[2 * row + 1] = n1;
                    }
                }
                yo[0] = y0;
                yo[1] = y1;
            }
        }
    }
}

__global__ void pack_rows_kernel(float *dst, int ldd, const float *a, int lda, int n0, const float *b, int ldb, int n1,
                                 int R) {
    const int w = n0 + n1;
    const int64_t total = (int64_t)R * w;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(e / w), c = (int)(e % w);
        dst[(size_t)r * ldd + c] = c < n0 ? a[(size_t)r * lda + c] : b[(size_t)r * ldb + (c - n0)];
    }
}

__global__ void reset_hidden_kernel(float *h, int E, int width, const uint8_t *done) {
    const int64_t total = (int64_t)E * width;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        if (done[i / width]) h[i] = 0.0f;
}

}  // namespace

extern "C" {

const char *aac_gru_last_error(void) { return g_err.c_str(); }

static int cell_check(const aac_gru_args &a) {
    if (a.R <= 0 || a.N <= 0) return gfail("gru_cell: R, N > 0");
    if (a.O < 1 || a.O > 2) return gfail("gru_cell: 1 <= O <= 2");
    if (!a.gi || !a.gh || !a.h || !a.wout || !a.bout) return gfail("gru_cell: NULL input");
    if (a.mode < AAC_GRU_FWD || a.mode > AAC_GRU_ACTBWD) return gfail("gru_cell: bad mode");
    if (a.mode == AAC_GRU_TD && (!a.rew || !a.done || !a.yout || a.O != 1)) return gfail("gru_cell: TD needs rew, done, yout, O = 1");
    if (a.mode == AAC_GRU_CRITIC && (!a.target || a.O != 1)) return gfail("gru_cell: CRITIC needs target, O = 1");
    if (a.mode == AAC_GRU_ACTLOSS && a.O != 1) return gfail("gru_cell: ACTLOSS needs O = 1");
    if (a.mode == AAC_GRU_ACTBWD && ((!a.da && !(a.dsa && a.wsa)) || !a.dq))
        return gfail("gru_cell: ACTBWD needs da (or dsa and wsa), dq");
    if (a.mode >= AAC_GRU_CRITIC && !a.dgi) return gfail("gru_cell: backward modes need dgi");
    if (a.pack_dst && (!a.pack_src || a.npack < 0 || a.npack + a.O > 64)) return gfail("gru_cell: bad pack");
    return 0;
}

int aac_gru_cell(const aac_gru_args *args, void *stream) {
    const aac_gru_args &a = *args;
    if (int rc = cell_check(a)) return rc;
    hipLaunchKernelGGL(gru_cell_kernel, dim3((a.R + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gfail(std::string("gru_cell: ") + hipGetErrorString(e));
    return 0;
}

int aac_gru_cell2(const aac_gru_args *a0, const aac_gru_args *a1, int32_t chain, void *stream) {
    if (!a0 || !a1) return gfail("gru_cell2: null arguments");
    if (int rc = cell_check(*a0)) return rc;
    if (chain) {
        if (a0->mode != AAC_GRU_TD || a1->mode != AAC_GRU_CRITIC || a0->R != a1->R)
            return gfail("gru_cell2: chain needs set 0 TD and set 1 CRITIC over the same rows");
        aac_gru_args b = *a1;
        if (!b.target) b.target = a0->yout;      // validated below; the chained value is used instead
        if (int rc = cell_check(b)) return rc;
    } else if (int rc = cell_check(*a1)) {
        return rc;
    }
    GruCellPair P{*a0, *a1, chain ? 1 : 0};
    const int grid = chain ? (a0->R + 3) / 4 : (a0->R + 3) / 4 + (a1->R + 3) / 4;
    hipLaunchKernelGGL(gru_cell2_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gfail(std::string("gru_cell: ") + hipGetErrorString(e));
    return 0;
}

static int actor_fwd_check(const aac_gru_actor_args &a) {
    const bool proj = a.gi != nullptr;
    auto al16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (a.E <= 0 || a.N <= 0) return gfail("gru_actor_fwd: E, N > 0");
    if (a.d_own < 1 || a.d_own > 8 || a.ld_own < a.d_own || a.ld_radar < 18 || a.ldh < H)
        return gfail("gru_actor_fwd: 1 <= d_own <= 8 and row strides >= the used widths");
    if (!a.own || !a.radar || !a.h || !a.Wo || !a.bo || !a.Wg || !a.bg || !a.Wih || !a.bih || !a.Whh || !a.bhh)
        return gfail("gru_actor_fwd: NULL operand");
    if (a.ldh % 4 || !al16(a.h)) return gfail("gru_actor_fwd: h rows must be 16-B aligned");
    if (proj) {
        if (!a.gh || a.ldg < 3 * H || a.ldg % 4 || !al16(a.gi) || !al16(a.gh) ||
            (a.cat && (a.ldc < 128 || a.ldc % 4 || !al16(a.cat))))
            return gfail("gru_actor_fwd: projection outputs gi, gh (and cat) with 16-B aligned rows");
    } else {
        if (!a.hout || !a.y || !a.Wout || !a.bout || a.ldy < 2) return gfail("gru_actor_fwd: NULL output operand");
        if (a.ldho % 4 || a.ldho < H || !al16(a.hout)) return gfail("gru_actor_fwd: hout rows must be 16-B aligned");
        if (a.noisy && (!a.counter || a.ldy != 2)) return gfail("gru_actor_fwd: noisy needs a counter and ldy == 2");
    }
    return 0;
}

int aac_gru_actor_fwd(const aac_gru_actor_args *args, void *stream) {
    if (!args) return gfail("gru_actor_fwd: null arguments");
    const aac_gru_actor_args &a = *args;
    if (int rc = actor_fwd_check(a)) return rc;
    const bool proj = a.gi != nullptr;
    // one workgroup per CU in all (one wave per SIMD: ~250 registers of weights per lane)
    const int rows = proj ? 16 : 32;
    const int blocks = (a.E + rows - 1) / rows;
    const int G = std::max(1, std::min(blocks, 256 / a.N));
    GruActorBatch b{};
    b.s[0] = b.s[1] = b.s[2] = a;
    b.n = 1;
    if (proj) hipLaunchKernelGGL((gru_actor_fwd_kernel<1, true>), dim3(G * a.N), dim3(256), 0, (hipStream_t)stream, b);
    else hipLaunchKernelGGL((gru_actor_fwd_kernel<2, false>), dim3(G * a.N), dim3(256), 0, (hipStream_t)stream, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gfail(std::string("gru_actor_fwd: ") + hipGetErrorString(e));
    return 0;
}

int aac_gru_actor_proj_multi(const aac_gru_actor_args *args, int32_t n, void *stream) {
    if (!args || n < 1 || n > GMAX) return gfail("gru_actor_proj_multi: 1 <= n <= 3 argument sets");
    GruActorBatch b{};
    for (int k = 0; k < n; ++k) {
        if (int rc = actor_fwd_check(args[k])) return rc;
        if (!args[k].gi) return gfail("gru_actor_proj_multi: projection mode (gi != NULL) only");
        if (args[k].E != args[0].E || args[k].N != args[0].N) return gfail("gru_actor_proj_multi: equal E and N");
        b.s[k] = args[k];
    }
    for (int k = n; k < GMAX; ++k) b.s[k] = args[0];
    b.n = n;
    // the 256 CUs shared by the sets: each workgroup keeps its weights for several 16-row blocks
    const int blocks = (args[0].E + 15) / 16;
    const int G = std::max(1, std::min(blocks, 256 / (args[0].N * n)));
    hipLaunchKernelGGL((gru_actor_fwd_kernel<1, true>), dim3(G * args[0].N * n), dim3(256), 0, (hipStream_t)stream, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gfail(std::string("gru_actor_proj_multi: ") + hipGetErrorString(e));
    return 0;
}

int aac_pack_rows(float *dst, int32_t ldd, const float *a, int32_t lda, int32_t n0, const float *b, int32_t ldb,
                  int32_t n1, int32_t R, void *stream) {
    if (R <= 0 || n0 < 0 || n1 < 0 || n0 + n1 > ldd) return gfail("pack_rows: bad shape");
    const int64_t total = (int64_t)R * (n0 + n1);
    int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(pack_rows_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, (hipStream_t)stream, dst, ldd, a, lda,
                       n0, b, ldb, n1, R);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gfail(std::string("pack_rows: ") + hipGetErrorString(e));
    return 0;
}

int aac_gru_reset_hidden(float *h, int32_t E, int32_t width, const uint8_t *env_done, void *stream) {
    if (E <= 0 || width <= 0 || !h || !env_done) return gfail("gru_reset_hidden: bad arguments");
    const int64_t total = (int64_t)E * width;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(reset_hidden_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, h, E, width, env_done);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gfail(std::string("gru_reset_hidden: ") + hipGetErrorString(e));
    return 0;
}

}  // extern "C"
