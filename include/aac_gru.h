/* aac_gru.h -- C ABI of the GRU-cell row kernel in libaac_env.so (gfx950): the recurrent core of
 * the GRU-actor MADDPG.
 *
 * It replaces, for every agent at once (agent of row r = r % N):
 *   nn.GRUCell(128, 64) + outlay Linear(64, 2) + Tanh of GRUCELL_actor_TwoPortion
 *       (MADDPG_ownENV_randomOD_Wgru_radar/Nnetworks_randomOD_Wgru_radar.py:181-198)
 *   nn.GRUCell(128, 64) + own_fc_outlay Linear(64, 1) of critic_single_obs_wGRU_TwoPortion
 *       (same file :428-446)
 * and their backward inside update_myown (maddpg_agent_randomOD_Wgru_radar.py:211-326).  The two
 * input projections gi = x W_ih^T + b_ih and gh = h W_hh^T + b_hh come from aac_gemm_batch; this
 * kernel does the gates (torch's GRUCell order: r = sig(gi_r + gh_r), z = sig(gi_z + gh_z),
 * n = tanh(gi_n + r gh_n), h' = (h - n) z + n), the output layer, the loss gradient and the gate
 * backward, one wave per row with lane = hidden unit.
 *
 * Conventions as aac_env.h: device pointers, stream = hipStream_t as void*, 0 = ok, message in
 * aac_gru_last_error().
 */
#ifndef AAC_GRU_H
#define AAC_GRU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AAC_GRU_HIDDEN 64 /* actor_hidden_state (WGRU/ma_main:389) */

enum {
    AAC_GRU_FWD = 0,     /* y = act(W_out h' + b_out); optional h' and packed [src | y] rows */
    AAC_GRU_TD = 1,      /* yout = rew + (gamma q')(1 - done)          (WGRU/maddpg:280-282) */
    AAC_GRU_CRITIC = 2,  /* MSE: dq = 2(q - target)/M, gate gradients    (WGRU/maddpg:284-291) */
    AAC_GRU_ACTLOSS = 3, /* 3 - mean q: dq = -1/M, gate gradients        (WGRU/maddpg:302-305) */
    AAC_GRU_ACTBWD = 4   /* d a -> tanh output layer -> gate gradients   (WGRU/nets:196-197) */
};

typedef struct {
    const float *gi, *gh; /* [R][192] pre-activations incl. biases, rows ldg apart */
    int32_t ldg;
    const float *h; /* [R][64] hidden state in, rows ldh apart */
    int32_t ldh;
    const float *wout, *bout; /* agent n: [O][64] weights at wout + n*wstride, O biases at bout + n*bstride */
    int32_t wstride, bstride;
    int32_t O;                /* output units: 2 actor, 1 critic */
    int32_t act;              /* output activation: 0 none, 2 tanh */
    int32_t R, N, mode;
    float *hout; /* h' rows (may be NULL), ldho apart */
    int32_t ldho;
    float *y; /* FWD: outputs [R][O] (ldy); CRITIC / ACTLOSS: q [R] (may be NULL) */
    int32_t ldy;
    const float *pack_src; /* FWD (may be NULL): pack_dst[r] = [pack_src[r][0 .. npack-1], y_r] */
    int32_t ld_pack_src, npack;
    float *pack_dst;
    int32_t ld_pack_dst;
    const float *target;      /* CRITIC: TD target [R] */
    const float *rew, *done;  /* TD: [R] each */
    float gamma, inv_m;       /* TD discount; 1 / rows of the per-agent loss mean */
    float *yout;              /* TD: [R] */
    const float *da;          /* ACTBWD: d loss / d a [R][O] rows ldda apart */
    int32_t ldda;
    float *dq;                /* CRITIC / ACTLOSS: dq [R]; ACTBWD: dout [R][O] */
    float *dgi, *dgh;         /* gate gradients [R][192] rows ldd apart (dgh may be NULL) */
    int32_t ldd;
    /* ACTBWD with dsa != NULL (da == NULL): d a computed here as the critic input layer's backward,
     * da[r][j] = sum_k dsa[r][k] wsa[agent][k][col + j] over k < 64 (dsa rows lddsa apart; agent n's
     * [64][ldwsa] matrix at wsa + n*wsa_stride) -- in place of a product launch (WGRU/maddpg:302-305) */
    const float *dsa;
    int32_t lddsa;
    const float *wsa;
    int32_t wsa_stride, ldwsa, wsa_col;
} aac_gru_args;

const char *aac_gru_last_error(void);

int aac_gru_cell(const aac_gru_args *args, void *stream);

/* Two aac_gru_cell argument sets in one launch: chain == 0, independent sets (e.g. the target actor's
 * and the actor's forward cells of one update); chain != 0, per row: set 0 in TD mode, then set 1 in
 * CRITIC mode with that row's TD target taken from the register (a1->target may be NULL).  Same
 * results as two aac_gru_cell calls. */
int aac_gru_cell2(const aac_gru_args *a0, const aac_gru_args *a1, int32_t chain, void *stream);

/* The whole GRUCELL_actor_TwoPortion forward (WGRU/Nnetworks:181-198: own_fc + own_grid encoders,
 * GRUCell(128, 64), outlay Linear(64, 2) + Tanh) for E envs x N agents in one launch: rows
 * r = e*N + i of agent i (own rows ld_own apart, the first d_own <= 8 columns read; radar rows 18
 * wide; hidden rows 64 wide).  Weights-stationary: a workgroup takes one agent, keeps every weight
 * fragment of its wave's 16 hidden units in registers and walks 32-row blocks; the input projections
 * run on the fp32 matrix cores and never reach memory.  Replaces the act path's two grouped-GEMM
 * launches (encoders, gates) and its aac_gru_cell launch.  Agent i's parameters are at the agent-0
 * pointers + i*pstride floats.  hout (h', 64 wide, ldho % 4 == 0) and y (tanh actions, 2 wide). */
typedef struct {
    const float *own;
    int32_t ld_own, d_own;
    const float *radar;
    int32_t ld_radar;
    const float *h;
    int32_t ldh;
    const float *Wo, *bo, *Wg, *bg, *Wih, *bih, *Whh, *bhh, *Wout, *bout;
    int32_t pstride;
    int32_t E, N;
    float *hout;
    int32_t ldho;
    float *y;
    int32_t ldy;
    /* projection mode (gi != NULL; any GRU network of this shape, e.g. update_myown's critics with
     * d_own = 8 input columns): no cell and no output layer -- cat = [e_o | e_g] (ldc), gi = cat W_ih^T
     * + b_ih and gh = h W_hh^T + b_hh (ldg) are written for aac_gru_cell and the weight gradients,
     * in place of the encoder and gate grouped-GEMM launches; hout, y, Wout, bout are not used. */
    float *cat, *gi, *gh;
    int32_t ldc, ldg;
    /* act mode, noisy != 0: the exploration noise and clamp of choose_action (WGRU/maddpg:336-428) on y
     * in the same launch -- exactly aac_noise_clamp(y, E, N, episode, eps_end, noise_start, noise_end,
     * seed, counter, noise_out) after it (same per-row noise, the counter's epoch advances once) */
    int32_t noisy;
    const int32_t *episode;
    int32_t eps_end;
    float noise_start, noise_end;
    uint64_t seed;
    uint64_t *counter;
    float *noise_out;
} aac_gru_actor_args;

int aac_gru_actor_fwd(const aac_gru_actor_args *args, void *stream);

/* n <= 3 projection-mode argument sets (gi != NULL, equal E and N) in one launch: independent
 * network evaluations of one update_myown (WGRU/maddpg:242-310: the target actor on s', the critic on
 * (s, a), the actor on s), the CUs shared between them so that each workgroup keeps its weights for
 * several row blocks.  Same results as n aac_gru_actor_fwd calls. */
int aac_gru_actor_proj_multi(const aac_gru_actor_args *args, int32_t n, void *stream);

/* dst[r][0 .. n0-1] = a[r*lda + ...], dst[r][n0 .. n0+n1-1] = b[r*ldb + ...] for R rows (ldd):
 * the [own, a] critic input rows of critic_single_obs_wGRU_TwoPortion (WGRU/nets:441). */
int aac_pack_rows(float *dst, int32_t ldd, const float *a, int32_t lda, int32_t n0, const float *b, int32_t ldb,
                  int32_t n1, int32_t R, void *stream);

/* h[e][0 .. width-1] = 0 for every env e < E with env_done[e] != 0: a finished episode starts the
 * next one from zero hidden states (WGRU/ma_main:476-478). */
int aac_gru_reset_hidden(float *h, int32_t E, int32_t width, const uint8_t *env_done, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* AAC_GRU_H */
