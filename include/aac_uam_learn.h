/* aac_uam_learn.h -- C ABI of the fused float64 UAM learner in libaac_env.so (gfx950).
 *
 * The UAM variant's update_myown (UAM/maddpg:304-595: one gradient iteration of a shared
 * ActorNetwork_TwoPortion and a shared critic_single_TwoPortion in float64, B = 512 rows, then the
 * Polyak update) is ~20 launches of five kinds instead of ~100 torch kernels:
 *
 *   aac_gemm64_batch  up to AAC_GEMM64_MAX independent float64 products in ONE launch (grouped GEMM
 *                     on v_mfma_f64_16x16x4_f64, one 16x16 output tile per wave) with the same
 *                     fused epilogue, ``ones`` bias-gradient column and ``ksplit`` partial copies
 *                     as aac_gemm_batch (include/aac_fused.h); the struct is aac_gemm_prob with
 *                     double pointers.
 *   aac_uam_push      one replay row per aircraft into the device ring.
 *   aac_uam_gather    sampled replay rows -> the learner's input layouts.
 *   aac_uam_head      the critic's 256 -> 1 output layer per row with the TD target, the mse
 *                     gradient or the -mean Q gradient, and the per-row loss terms.
 *   aac_adam64_sum    torch fused Adam (float64, capturable) on the fixed-order sum of partial
 *                     gradient copies.
 *   aac_uam_polyak    soft update of both targets, the step counter, and the two losses.
 *
 * Conventions as in aac_env.h: plain device pointers, ``stream`` = hipStream_t as void*,
 * 0 = ok, message in aac_uam_learn_last_error().
 */
#ifndef AAC_UAM_LEARN_H
#define AAC_UAM_LEARN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AAC_GEMM64_MAX 16

/* C[M][N] = mact(act(op(A) op(B) + addend + bias)) in float64; fields as aac_gemm_prob. */
typedef struct {
    const double *A, *B;
    double *C;
    const double *bias, *addend, *mask;
    double *cextra;
    int64_t split_stride;
    int32_t M, N, K;
    int32_t lda, ldb, ldc, ldadd, ldmask;
    int32_t ta, tb, act, mact, ones, ksplit;
    /* dual output (may be NULL): C2[m*ldc + n] = C[m][n] > 0 ? dscale * dvec[n] : 0 -- the actor
     * loss's critic head dh = -1/B w (h > 0) from the merge layer's epilogue (UAM/maddpg:512) */
    const double *dvec;
    double *C2;
    double dscale;
} aac_gemm64_prob;

const char *aac_uam_learn_last_error(void);

int aac_gemm64_batch(const aac_gemm64_prob *probs, int32_t n, void *stream);

/* Appends M transitions (one per aircraft) to the float64 replay ring at slots (pos + i) % capacity
 * as rows [own 7 | radar 18 | a 2 | r | done | own' 7 | radar' 18]; done is uint8 (done_u8 = 1)
 * or float64.  meta (may be NULL) receives the ring's new [pos, size] = [(pos + M) % capacity,
 * min(size + M, capacity)] for the device sampler.  Replaces UamReplay.push_batch's torch.cat
 * (UAM/main:582-603 pushes one Experience per aircraft). */
int aac_uam_push(double *ring, int64_t capacity, int64_t pos, int64_t M, const double *own, const double *radar,
                 const double *act, const double *rew, const void *done, int32_t done_u8, const double *nown,
                 const double *nradar, int64_t *meta, int64_t size, void *stream);

/* aac_uam_push with the ring position on the device (graph replays of whole training steps): the
 * position is read from *pos_in and the advanced one, (pos + M) % capacity, stored to *pos_out (a
 * different word); meta (required) receives [new pos, min(meta[1] + M, capacity)].  Alternate the
 * two words between consecutive pushes. */
int aac_uam_push_io(double *ring, int64_t capacity, int64_t M, const double *own, const double *radar,
                    const double *act, const double *rew, const void *done, int32_t done_u8, const double *nown,
                    const double *nradar, int64_t *meta, const int64_t *pos_in, int64_t *pos_out, void *stream);

/* Replay rows ring[idx[b]] (row width 54: own 7 | radar 18 | a 2 | r | done | own' 7 | radar' 18,
 * uam_learner.ROW) -> rows[b][54], xc[b] = [own | a] (9), xt[b][0:7] = own', xp[b][0:7] = own. */
int aac_uam_gather(const double *ring, const int32_t *idx, int32_t B, double *rows, double *xc, double *xt,
                   double *xp, void *stream);

/* Critic output layer q[r] = h[r] . w + b[0] over B rows of 256 features (h row stride 256):
 *   mode 0 (critic loss, mse):   e = q - y[r], dq = (2/B) e, dh = dq w (h > 0), lterm[r] = e^2
 *   mode 1 (actor loss, -mean):  dq = -1/B, dh = dq w (h > 0), lterm[r] = q
 *   mode 2 (TD target):          y[r] = rew[r*ldr] + gamma q (1 - done[r*ldr])
 * y is read in mode 0 and written in mode 2; dq (may be NULL) gets dq[r]; dq / dh / lterm are
 * unused in mode 2. */
int aac_uam_head(const double *h, int32_t B, const double *w, const double *b, int32_t mode, double *y,
                 const double *rew, const double *done, int32_t ldr, double gamma, double *dq, double *dh,
                 double *lterm, void *stream);

/* aac_uam_head mode 2 on the target critic's rows ht (TD target into y) and mode 0 on the critic's
 * rows h chained in one launch: for each row r, y[r] = rew[r*ldr] + gamma Q'(1 - done[r*ldr]), then
 * the mse head of Q(h[r]) against that y (dq, dh, lterm = e^2) -- the values of the two launches. */
int aac_uam_td_mse_head(const double *ht, const double *wt, const double *bt, const double *rew, const double *done,
                        int32_t ldr, double gamma, double *y, const double *h, const double *w, const double *b,
                        int32_t B, double *dq, double *dh, double *lterm, void *stream);
/* torch.optim.Adam(fused, capturable) step for float64 parameters: g = sum of nsplit partial
 * copies gpart[s*n + i] in copy order; t = *step + step_add, bias corrections in float64:
 *   m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= (lr/(1-b1^t)) m / (sqrt(v)/sqrt(1-b2^t) + eps) */
int aac_adam64_sum(double *param, const double *gpart, int32_t nsplit, double *exp_avg, double *exp_avg_sq,
                   int64_t n, double lr, double beta1, double beta2, double eps, const int32_t *step,
                   int32_t step_add, void *stream);
/* Same on the summed gradient times gscale (1 / world after a SUM all-reduce of the ranks' sums). */
int aac_adam64_sum_scaled(double *param, const double *gpart, int32_t nsplit, double *exp_avg, double *exp_avg_sq,
                          int64_t n, double lr, double beta1, double beta2, double eps, const int32_t *step,
                          int32_t step_add, double gscale, void *stream);

/* out[i] = the sum of the nsplit partial copies gpart[s*n + i] in aac_adam64_sum's order: the
 * gradient a multi-rank update all-reduces before aac_adam64_sum(..., out, nsplit = 1, ...). */
int aac_sum64_partials(double *out, const double *gpart, int32_t nsplit, int64_t n, void *stream);

/* target[i] += tau (src[i] - target[i]) over n parameters (torch._foreach_lerp_); then one wave
 * adds 1 to *step and writes loss[0] = mean(lq[0..B)), loss[1] = -mean(la[0..B)) with a fixed
 * summation order (lq / la / loss may be NULL). */
int aac_uam_polyak(double *target, const double *src, int64_t n, double tau, int32_t *step, const double *lq,
                   const double *la, int32_t B, double *loss, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* AAC_UAM_LEARN_H */
