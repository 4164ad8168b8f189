/* aac_fused.h -- C ABI of the fused learner kernels in libaac_env.so (gfx950).
 *
 * The MADDPG update of the reference (update_myown, ATT/maddpg:219-440) is a chain of small
 * nn.Linear forward/backward products over B = 1024 samples x N agents.  On MI355X the cost is
 * the number of launches, not the FLOPs, so the learner is expressed as ~25 launches per
 * gradient iteration of two kinds:
 *
 *   aac_gemm_batch   up to AAC_GEMM_MAX independent fp32 products in ONE launch (grouped GEMM on
 *                    v_mfma_f32_16x16x4_f32, one 32x32 tile per wave), each with a fused epilogue
 *                      C = mact( act( A.B + addend + bias ) )
 *                    act = ReLU / tanh of the layer (ATT/nets:180-184, :699-701); mact multiplies
 *                    by the derivative of the layer that produced ``mask`` (relu' or 1 - t^2),
 *                    i.e. the backward of the activation; ``ones`` appends a virtual column of
 *                    ones to B so a weight-gradient product dW = G^T X also yields the bias
 *                    gradient sum_rows G (written to cextra).  Large-K weight-gradient products
 *                    split K into ``ksplit`` partial copies of C (split_stride apart) that the
 *                    optimiser kernel sums in fixed order (aac_adam_flat_sum), so no cross-
 *                    workgroup reduction or fence is needed inside the launch.
 *   aac_critic_head  the critic's 256 -> 1 output layer per row (one wave per row) fused with
 *                    the loss gradient: mse (ATT/maddpg:386) / -mean Q (ATT/maddpg:424) / the
 *                    TD target r + gamma Q'(1 - done_any) (ATT/maddpg:355-370).
 *
 * Conventions as in aac_env.h: plain device pointers, ``stream`` = hipStream_t as void*,
 * 0 = ok, message in aac_fused_last_error().
 */
#ifndef AAC_FUSED_H
#define AAC_FUSED_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AAC_GEMM_MAX 16

/* C[M][N] (row-major, ldc) = epilogue(op(A)[M][K] . op(B)[K][N]).
 * op(A)[m][k] = ta ? A[k*lda + m] : A[m*lda + k];  op(B)[k][n] = tb ? B[n*ldb + k] : B[k*ldb + n].
 * ones = 1: column N-1 of op(B) is a virtual column of ones and C column N-1 goes to cextra[m]
 * (no epilogue on it); the real B / C have N-1 columns.
 * act: 0 none, 1 relu, 2 tanh.  mact: 0 none, 1 x (mask > 0), 2 x (1 - mask^2); mask[m*ldmask+n].
 * addend (may be NULL): added before bias.
 * ksplit <= 1: one pass over K.  ksplit > 1: split s of K writes its partial product to
 * C + s*split_stride (and cextra + s*split_stride); no addend / bias / act / mact allowed. */
typedef struct {
    const float *A, *B;
    float *C;
    const float *bias, *addend, *mask;
    float *cextra;
    int64_t split_stride;
    int32_t M, N, K;
    int32_t lda, ldb, ldc, ldadd, ldmask;
    int32_t ta, tb, act, mact, ones, ksplit;
    /* dual output (may be NULL): C2[m*ldc + n] = C[m][n] > 0 ? dscale * dvec[n] : 0 -- the critic
     * head's actor-loss gradient dh = dq w (h > 0) with the constant dq = -1/B (ATT/maddpg:424)
     * written by the combine layer's epilogue; needs ksplit <= 1 and no ones column */
    const float *dvec;
    float *C2;
    float dscale;
} aac_gemm_prob;

/* A critic-head job (the arguments of aac_critic_head) that runs inside a grouped GEMM launch,
 * beside products it does not depend on (aac_gemm_batch_heads). */
typedef struct {
    const float *h;
    int32_t ldh, M;
    const float *w, *b;
    int32_t mode;
    const float *y, *rew, *done;
    int32_t B, N;
    float gamma;
    float *q, *dq, *dh, *yout;
    /* mode 2 only (M2 > 0): the critic step's mse head (mode 0 with M = M2) on rows r < M2 of h2
     * (w2, b2: the current critic's output layer; q2, dq2, dh2 as q, dq, dh), chained on the TD
     * target just computed for row r -- the TD target of update_myown's first batch and its critic
     * loss gradient in one pass */
    const float *h2, *w2, *b2;
    float *q2, *dq2, *dh2;
    int32_t M2;
} aac_head_job;

#define AAC_HEAD_MAX 1

const char *aac_fused_last_error(void);

/* n <= AAC_GEMM_MAX products in one launch. */
int aac_gemm_batch(const aac_gemm_prob *probs, int32_t n, void *stream);
/* The same launch with nh <= AAC_HEAD_MAX critic-head jobs (without a chained head) appended as
 * extra workgroups (four rows each; the arithmetic of aac_critic_head).  The jobs must not read what the products write, nor
 * the products what the jobs write: one launch, no ordering between them.  n may be 0. */
int aac_gemm_batch_heads(const aac_gemm_prob *probs, int32_t n, const aac_head_job *heads, int32_t nh, void *stream);
/* aac_gemm_batch with an explicit workgroup order: xcd_order != 0 hands each of the 8 XCDs (workgroup
 * b runs on XCD b % 8) a contiguous range of the launch's workgroups, so the tiles of one product share
 * one XCD's L2 and read their operands from HBM about once.  Same arithmetic, bit-identical results.
 * For the GRU learner's launches (16 equal per-agent products each) it cuts grouped-GEMM HBM traffic
 * 3.06x -> 1.19x the algorithmic bytes (profiles/r03_gemm_pmc_gru_xcd_*.json) but costs ~1 % of the
 * config-4 step, so the learner uses it only with AAC_GRU_XCD=1.  xcd_order == 0 forces the
 * round-robin order (also under AAC_GEMM_XCD_ALL). */
int aac_gemm_batch_ordered(const aac_gemm_prob *probs, int32_t n, int32_t xcd_order, void *stream);
/* The launch plan of aac_gemm_batch without launching (host only): per product 0 (register
 * fragments, 32x32 wave tiles) or 1 + cfg (LDS-staged workgroup tile: cfg >> 2 = 64x64 / 64x32 /
 * 32x64 / 32x32, cfg & 3 = operand layouts); *workgroups = the grid (may be NULL). */
int aac_gemm_plan(const aac_gemm_prob *probs, int32_t n, int32_t *lds_cfg, int32_t *workgroups);
/* Process-wide tile policy (default from AAC_GEMM_LDS_MIN_WG = 256, AAC_GEMM_LDS_SMALL = 0): an
 * eligible product takes the largest LDS workgroup tile (64x64, then 64x32 / 32x64) that gives at
 * least min_workgroups workgroups, else the register path; small_tiles != 0 falls back to 32x32 LDS
 * tiles instead; min_workgroups = -1 - c forces tile c (0 64x64, 1 64x32, 2 32x64, 3 32x32) on every
 * eligible product.  For tests and measurement tools; plans built afterwards use it. */
void aac_gemm_set_lds_policy(int32_t min_workgroups, int32_t small_tiles);

/* Diagnostic builds only (-DAAC_GEMM_STAMPS): per-workgroup stamps of the last gemm launch,
 * 5 uint64 per workgroup [memrealtime entry, memtime entry, memtime after MFMA loop, memtime exit,
 * memrealtime exit]; returns -1 in a normal build. */
int aac_gemm_stamps(unsigned long long *out, int32_t n_wg);

/* torch.optim.Adam step (as aac_adam_flat_at) whose gradient is the fixed-order sum of nsplit
 * partial copies gpart[s*n + i]; grad_out (may be NULL) receives that sum. */
int aac_adam_flat_sum(float *param, const float *gpart, int32_t nsplit, float *grad_out, float *exp_avg,
                      float *exp_avg_sq, int64_t n, float lr, float beta1, float beta2, float eps,
                      const int32_t *step, int32_t step_add, void *stream);
/* The same with the partial copies gstride floats apart (>= n; the learners pad it to a multiple of
 * 4 so that the copy-parallel kernel's 16-B loads stay aligned). */
int aac_adam_flat_sum_strided(float *p, const float *gpart, int32_t ns, int64_t gstride, float *gout, float *m,
                              float *v, int64_t n, float lr, float b1, float b2, float eps, const int32_t *step,
                              int32_t step_add, void *stream);

/* One network's Adam job for aac_adam_flat_sum_pair (arguments as aac_adam_flat_sum_strided). */
typedef struct aac_adam_job {
    float *param;
    const float *gpart;
    int32_t nsplit;
    int64_t gstride;
    float *grad_out;
    float *exp_avg, *exp_avg_sq;
    int64_t n;
    float lr, beta1, beta2, eps;
    const int32_t *step;
    int32_t step_add;
} aac_adam_job;
/* Two networks' Adam steps over split-K copies in one launch (the copy-parallel kernel for both:
 * nsplit >= 2, gstride % 4 == 0, 16-B aligned copies; AAC_ADAM4 on); each job's arithmetic is
 * that of aac_adam_flat_sum_strided. */
int aac_adam_flat_sum_pair(const aac_adam_job *a, const aac_adam_job *b, void *stream);

/* out[i] = sum_{s < nsplit} gpart[s*n + i] in split order (before a gradient all-reduce). */
int aac_sum_partials(float *out, const float *gpart, int32_t nsplit, int64_t n, void *stream);
int aac_sum_partials_strided(float *out, const float *gpart, int32_t nsplit, int64_t gstride, int64_t n, void *stream);

/* Critic output layer + loss gradient, rows of 256 features h[r*ldh + j]:
 *   q[r] = h[r] . w + b[0]
 *   mode 0 (critic loss, mse):  dq = (2/M)(q - y[r])      dh = dq w * (h > 0)
 *   mode 1 (actor loss, -mean): dq = -(1/M)               dh = dq w * (h > 0)
 *   mode 2 (TD target):  yout[r] = rew[r*N + r/B] + (gamma q)(1 - any_n(done[r*N + n] == 1))
 * q, dq, dh, yout may be NULL where unused. */
int aac_critic_head(const float *h, int32_t ldh, int32_t M, const float *w, const float *b, int32_t mode,
                    const float *y, const float *rew, const float *done, int32_t B, int32_t N, float gamma, float *q,
                    float *dq, float *dh, float *yout, void *stream);

/* One head job as its own launch (the arithmetic of aac_critic_head; with M2 > 0 the chained mse
 * head of the job's mode 2, which aac_gemm_batch_heads does not take). */
int aac_critic_head_job(const aac_head_job *job, void *stream);

/* Backward of the critic's action inputs into the actor's output layer, one row r = b*N + n per
 * actor row (R = B*N): da_j = df[b][n*128 .. +128] . W_enc_n[:, d0 + j] (wenc = N stacked
 * [128][din] encoder weights), dout[r][j] = da_j (1 - a_j^2) with a_j = X[(b*N + n)*din + d0 + j],
 * dha[r][c] = (dout_0 wa[c] + dout_1 wa[256 + c]) * (ha[r][c] > 0), ha / dha rows of 256. */
int aac_actor_out_bwd(const float *df, int32_t ldf, const float *wenc, int32_t din, int32_t d0, const float *X,
                      const float *wa, const float *ha, int32_t N, int32_t R, float *dout, float *dha, void *stream);

/* The actor step's critic data gradient and aac_actor_out_bwd in one launch (ATT/maddpg:421-425
 * backward): df = (dh Wc) * (f > 0) over B samples (dh [B][256], Wc the combine weight [256][ldw =
 * 128 N], f [B][ldw] the encoder outputs), reduced straight into da_j = df[b][n*128 ..] . W_enc_n[:, d0 + j]
 * (df is not stored), then dout / dha as aac_actor_out_bwd for the rows r = b*N + n.  head (may be
 * NULL, no chained head): a critic-head job as extra workgroups, independent of this work. */
typedef struct {
    const float *dh, *Wc, *f, *wenc, *X, *wa, *ha;
    float *dout, *dha;
    int32_t ldw, din, d0, N, B;
} aac_dcomb_aob_args;
int aac_actor_dcomb_out_bwd(const aac_dcomb_aob_args *args, const aac_head_job *head, void *stream);

/* Training form of the actor's neighbour attention (ATT/nets:186-210) over R rows of K neighbour
 * features xn[(r*K + j)*64] (mask from nei rows, nei_j.mean() != 0), e_o rows eo + r*lde:
 * q = Wq e_o, qk = Wk^T q, alpha = masked softmax(x_j . qk / 8), xb = sum alpha_j x_j,
 * vout[r*ldv + c] = (Wv xb)[c]; q, qk, xb [R][64] and alpha [R][K] are kept for the backward.
 * Wq, Wk, Wv: the 64x64 q / k / v weights (row-major, nn.Linear layout). */
int aac_attn_train_fwd(const float *eo, int32_t lde, const float *xn, const float *nei, const float *Wq,
                       const float *Wk, const float *Wv, float *q, float *qk, float *alpha, float *xb, float *vout,
                       int32_t ldv, int32_t R, int32_t K, void *stream);
/* Its backward from dv (= d v_att, rows dv + r*lddv): dxn = d x_j * (x_j > 0) [R*K][64],
 * dqk, dq [R][64], deo = (dcat_o + Wq^T dq) * (e_o > 0) [R][64] (dcat_o rows + r*ldd: the
 * merge layer's gradient into e_o). */
int aac_attn_train_bwd(const float *dv, int32_t lddv, const float *xn, const float *alpha, const float *qk,
                       const float *eo, int32_t lde, const float *dcat_o, int32_t ldd, const float *Wq, const float *Wk,
                       const float *Wv, float *dxn, float *dqk, float *dq, float *deo, int32_t R, int32_t K,
                       void *stream);

/* The same backward (K <= 8, the MFMA path) that also accumulates the neighbour encoder's weight
 * gradient: pwn [aac_attn_train_bwd_partials(R)][448] gets one partial row per workgroup, row p =
 * [sum dx_j^T nei_j (64 x 6, f * 6 + c) | sum dx_j (64)] over the workgroup's rows (nei rows
 * [(r*K + j)*6]); the rows sum to dWn | dbn (ATT/nets:186-190) in a fixed order.  dxn may be NULL. */
int aac_attn_train_bwd_wn(const float *dv, int32_t lddv, const float *xn, const float *alpha, const float *qk,
                          const float *eo, int32_t lde, const float *dcat_o, int32_t ldd, const float *Wq,
                          const float *Wk, const float *Wv, float *dxn, float *dqk, float *dq, float *deo, int32_t R,
                          int32_t K, const float *nei, float *pwn, void *stream);
int32_t aac_attn_train_bwd_partials(int32_t R);

/* Inference form of the actor's neighbour attention (ATT/nets:186-210) for R rows, K <= 32:
 * x_j = relu(Wn nei_j + bn) computed from the 6-wide rows nei[(r*K + j)*6], scores
 * x_j . (Wqk e_o) / 8 with Wqk = Wk^T Wq (64x64, precomputed), masked softmax (mask
 * nei_j.mean() != 0), out[r*ldo + c] = (Wv sum_j a_j x_j)[c]; e_o rows at eo + r*lde. */
int aac_attn_block(const float *eo, int32_t lde, const float *nei, const float *Wn, const float *bn,
                   const float *Wqk, const float *Wv, float *out, int32_t ldo, int32_t R, int32_t K, void *stream);

/* The actor's encoders fused into its neighbour attention (ATT/nets:194-210), K <= 8:
 *   e_o = relu(Wo own[:d_own] + bo), e_g = relu(Wg radar + bg)  -> cat[r][0:64], cat[r][64:128]
 *   x_j = relu(Wn nei_j + bn)                                    -> xn[(r*K + j)*64] (train)
 *   q = Wq e_o, qk = Wk^T q, alpha = masked softmax(x_j . qk / 8), xb = sum alpha_j x_j
 *   v_att = Wv xb                                                -> cat[r][128:192]
 * (q, qk, alpha, xb kept for aac_attn_train_bwd when xn != NULL; inference leaves them NULL).  The
 * encoders' GEMM launch before the attention disappears.  Optional riding job in the same launch
 * (c_rows > 0): the critic's per-agent encoders f[b][n*128 + c] = relu(W_n x_bn + b_n) (ATT/nets:
 * 697-701, R3) of rows x_bn = cx + b*cx_ld + n*c_din, W_n = cW + n*128*c_din, b_n = cb + n*128,
 * f = cf + b*c_n*128 + n*128 -- independent work that shares the launch; R = 0 runs it alone. */
typedef struct {
    const float *own; int32_t ld_own; int32_t d_own;
    const float *radar; int32_t ld_radar;
    const float *nei;
    const float *Wo, *bo, *Wg, *bg, *Wn, *bn, *Wq, *Wk, *Wv;
    float *cat; int32_t ld_cat;
    float *xn, *q, *qk, *alpha, *xb;
    int32_t R, K;
    const float *cx; int32_t cx_ld; int32_t c_din;
    const float *cW, *cb;
    float *cf;
    int32_t c_rows, c_n;
    /* optional (o_h != NULL): the actor's tanh output layer (ATT/nets:213) folded into the riding
     * job -- the action columns of its input rows are computed first, a_j = tanh(o_h[(b*c_n + n)*256] .
     * o_w[j*256] + o_b[j]) for j < 2, stored to o_x + b*cx_ld + n*c_din + o_d0 + j (o_x = the
     * writable view of cx) and used as the encoder's inputs.  The output layer's launch disappears. */
    const float *o_h, *o_w, *o_b;
    float *o_x;
    int32_t o_d0;
} aac_attn_enc_args;
/* nset = 1 or 2 independent argument sets in one launch (e.g. the target actor's inference pass
 * beside a training forward; K <= 8 each). */
int aac_attn_enc_fwd(const aac_attn_enc_args *args, int32_t nset, void *stream);
/* The same launch with a critic-head job (no chained head) appended as extra workgroups (four rows
 * each; the arithmetic of aac_critic_head); head may be NULL.  The job must not read what the sets
 * write, nor the sets what the job writes. */
int aac_attn_enc_fwd_head(const aac_attn_enc_args *args, int32_t nset, const aac_head_job *head, void *stream);

/* Replay gather with interleaved destinations: element c of field f of sampled row b goes to
 * dsts[f][b*(widths[f]/chunks[f])*dstrides[f] + (c/chunks[f])*dstrides[f] + c%chunks[f]]
 * (chunks = widths, dstrides = widths gives aac_replay_gather), and to the same place in
 * dsts2[f] when dsts2 and dsts2[f] are not NULL.  Lets [own_n | a_n] land as the critic's
 * (D0 + 2)-wide encoder input rows without a concat. */
int aac_replay_gather_strided(const float *ring, int32_t row_width, const int32_t *idx, int32_t B, int32_t n_fields,
                              float *const *dsts, float *const *dsts2, const int32_t *widths,
                              const int32_t *chunks, const int32_t *dstrides, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* AAC_FUSED_H */
