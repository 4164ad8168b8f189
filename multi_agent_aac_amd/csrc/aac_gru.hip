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
#include <string>

#include "../../include/aac_gru.h"
#include "aac_wave.h"

namespace {

thread_local std::string g_err;

int gfail(const std::string &m) {
    g_err = m;
    return -1;
}

using aacw::wsum;

constexpr int H = AAC_GRU_HIDDEN;

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void __launch_bounds__(256) gru_cell_kernel(aac_gru_args a) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int u = threadIdx.x & 63;
    if (r >= a.R) return;
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
        return;
    }
    if (a.mode == AAC_GRU_TD) {
        if (u == 0) a.yout[r] = a.rew[r] + (a.gamma * y0) * (1.0f - a.done[r]);
        return;
    }
    if (a.mode == AAC_GRU_CRITIC || a.mode == AAC_GRU_ACTLOSS) {
        const float g = a.mode == AAC_GRU_CRITIC ? (2.0f * a.inv_m) * (y0 - a.target[r]) : -a.inv_m;
        if (u == 0) {
            if (a.y) a.y[r] = y0;
            if (a.dq) a.dq[r] = g;
        }
        dh = g * W[u];
    } else {   // AAC_GRU_ACTBWD: tanh output layer backward
        const float d0 = a.da[(size_t)r * a.ldda] * (1.0f - y0 * y0);
        dh = d0 * W[u];
        if (u == 0) a.dq[(size_t)r * a.O] = d0;
        if (two) {
            const float d1 = a.da[(size_t)r * a.ldda + 1] * (1.0f - y1 * y1);
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

int aac_gru_cell(const aac_gru_args *args, void *stream) {
    const aac_gru_args &a = *args;
    if (a.R <= 0 || a.N <= 0) return gfail("gru_cell: R, N > 0");
    if (a.O < 1 || a.O > 2) return gfail("gru_cell: 1 <= O <= 2");
    if (!a.gi || !a.gh || !a.h || !a.wout || !a.bout) return gfail("gru_cell: NULL input");
    if (a.mode < AAC_GRU_FWD || a.mode > AAC_GRU_ACTBWD) return gfail("gru_cell: bad mode");
    if (a.mode == AAC_GRU_TD && (!a.rew || !a.done || !a.yout || a.O != 1)) return gfail("gru_cell: TD needs rew, done, yout, O = 1");
    if (a.mode == AAC_GRU_CRITIC && (!a.target || a.O != 1)) return gfail("gru_cell: CRITIC needs target, O = 1");
    if (a.mode == AAC_GRU_ACTLOSS && a.O != 1) return gfail("gru_cell: ACTLOSS needs O = 1");
    if (a.mode == AAC_GRU_ACTBWD && (!a.da || !a.dq)) return gfail("gru_cell: ACTBWD needs da, dq");
    if (a.mode >= AAC_GRU_CRITIC && !a.dgi) return gfail("gru_cell: backward modes need dgi");
    if (a.pack_dst && (!a.pack_src || a.npack < 0 || a.npack + a.O > 64)) return gfail("gru_cell: bad pack");
    hipLaunchKernelGGL(gru_cell_kernel, dim3((a.R + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gfail(std::string("gru_cell: ") + hipGetErrorString(e));
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
