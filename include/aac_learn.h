/* aac_learn.h -- C ABI of the learner-side kernels in libaac_env.so (gfx950).
 *
 * They replace the pieces of the reference's MADDPG path that are not plain GEMMs
 * (SURVEY.md section 8(a) rows a9-a14):
 *   aac_attn_fwd/bwd     masked single-head attention of ActorNetwork_ATT_TwoPortion
 *                        (ATT/nets:194-210: mask = nei.mean(-1) != 0, softmax(k.q / 8) over K,
 *                        masked weights zeroed, v_att = sum alpha v)
 *   aac_replay_push/...  ReplayMemory (ATT/mem:6-23) as a device ring of fixed-width fp32 rows;
 *                        sample = uniform without replacement like random.sample (ATT/mem:19)
 *   aac_adam_flat        torch.optim.Adam step (ATT/maddpg:93-94, :387, :425) on one flat buffer
 *   aac_polyak_flat      soft_update (ATT/maddpg:18-22) on one flat buffer
 *   aac_polyak_flat_step the same, advancing the optimiser step counter in the same launch
 *   aac_noise_clamp      choose_action exploration: act + randn * var, clamp [-1, 1]
 *                        (ATT/maddpg:476-500, var schedule :563-570)
 * Conventions as in aac_env.h: plain device pointers, ``stream`` = hipStream_t as void*, 0 = ok.
 */
#ifndef AAC_LEARN_H
#define AAC_LEARN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AAC_MAX_FIELDS 16

const char *aac_learn_last_error(void);

/* q [R][64]; k, v rows of 64 floats at k + (r*K + j) * kv_stride (same for v); nei [R][K][6]
 * (mask source, may be NULL = no mask); out rows of 64 at out + r * out_stride; alpha [R][K]. */
int aac_attn_fwd(const float *q, const float *k, const float *v, int32_t kv_stride, const float *nei, float *out,
                 int32_t out_stride, float *alpha, int32_t R, int32_t K, void *stream);
/* dout rows at dout + r * dout_stride; writes dq [R][64], dk/dv rows with kv_stride. */
int aac_attn_bwd(const float *q, const float *k, const float *v, int32_t kv_stride, const float *alpha,
                 const float *dout, int32_t dout_stride, float *dq, float *dk, float *dv, int32_t R, int32_t K,
                 void *stream);

/* One transition = one ring row made of n_fields consecutive fields; field f has widths[f]
 * elements per transition, source srcs[f] ([E][widths[f]]), dtype[f] 0 = fp32, 1 = uint8.
 * meta (device int64[2]) = {next write position, current size}; updated on the device. */
int aac_replay_push(float *ring, int32_t row_width, int64_t capacity, int64_t *meta, int32_t n_fields,
                    const void *const *srcs, const int32_t *widths, const int32_t *dtypes, int32_t E, void *stream);
/* The same push with the ring position and size known to the caller (pushes are host-initiated,
 * so the host mirrors them): rows (pos + e) % capacity, then meta = {(pos + E) % capacity,
 * min(size + E, capacity)} stored by the launch itself (one launch instead of two).  ring 16-B
 * aligned. */
int aac_replay_push_at(float *ring, int32_t row_width, int64_t capacity, int64_t *meta, int64_t pos, int64_t size,
                       int32_t n_fields, const void *const *srcs, const int32_t *widths, const int32_t *dtypes,
                       int32_t E, void *stream);
/* n_batches independent batches of B distinct indices uniform in [0, meta[1]) (B <= 4096,
 * meta[1] >= B) into idx[n_batches][B]; deterministic in (seed, *counter); *counter (device
 * uint64, < 2^32; its high half counts arriving workgroups inside the launch) is advanced by one per
 * call in the same launch. */
int aac_replay_sample(const int64_t *meta, int32_t B, int32_t n_batches, uint64_t seed, uint64_t *counter,
                      int32_t *idx, void *stream);
/* dsts[f][b][widths[f]] = ring[idx[b]][field f]. */
int aac_replay_gather(const float *ring, int32_t row_width, const int32_t *idx, int32_t B, int32_t n_fields,
                      float *const *dsts, const int32_t *widths, void *stream);

/* torch.optim.Adam (no weight decay, no amsgrad); step (device int32) is the step number
 * AFTER increment, read on the device so the call can be graph-captured. */
int aac_adam_flat(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float lr,
                  float beta1, float beta2, float eps, const int32_t *step, void *stream);
/* Same with step number *step + step_add (several optimiser steps per captured update read
 * one device counter that is advanced once afterwards). */
int aac_adam_flat_at(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float lr,
                     float beta1, float beta2, float eps, const int32_t *step, int32_t step_add, void *stream);
/* Same on the gradient grad * gscale: gscale = 1 / world after a SUM all-reduce of the ranks'
 * gradients (the data-parallel mean of SURVEY.md section 8(e) without a separate division launch). */
int aac_adam_flat_at_scaled(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float lr,
                            float beta1, float beta2, float eps, const int32_t *step, int32_t step_add, float gscale,
                            void *stream);
/* tgt = (1 - tau) * tgt + tau * src */
int aac_polyak_flat(float *tgt, const float *src, int64_t n, float tau, void *stream);
/* Same, and *step += step_add in the same launch (the optimiser step counter of this network,
 * advanced once per captured update after every Adam step that reads it; NULL: no counter). */
int aac_polyak_flat_step(float *tgt, const float *src, int64_t n, float tau, int32_t *step, int32_t step_add,
                         void *stream);
/* Both networks' soft updates (critic, actor: ATT/maddpg:436-438) and their step counters in one
 * launch; the same arithmetic per element as two aac_polyak_flat_step calls. */
int aac_polyak_flat2(float *tgt1, const float *src1, int64_t n1, int32_t *step1, float *tgt2, const float *src2,
                     int64_t n2, int32_t *step2, float tau, int32_t step_add, void *stream);

/* Fused activation backward + bias gradient of y = act(x W^T + b) (nn.Linear + ReLU/Tanh of
 * ATT/nets:180-184, ATT/nets:699-701): gm = gy * act'(y) (rows of O at the given strides; gm may
 * be NULL) and db[o] = sum_m gm[m][o] (db may be NULL), reduced deterministically in the same
 * launch through ws (>= ceil(M/32) * O floats) and tickets (>= ceil(O/64) zeroed uint32 that the
 * kernel leaves zeroed).  act: 0 identity, 1 ReLU, 2 tanh. */
int aac_act_bgrad(const float *gy, int32_t gy_stride, const float *y, int32_t y_stride, float *gm,
                  int32_t gm_stride, float *db, int32_t M, int32_t O, int32_t act, float *ws, uint32_t *tickets,
                  void *stream);

/* y[M][O] = act(y + b) in place (bias + activation epilogue of a bias-less GEMM). */
int aac_bias_act(float *y, const float *b, int64_t M, int32_t O, int32_t act, void *stream);

/* act [E*N][2] += (float)(randn * var_e); clamp to [-1, 1]; var_e from episode[e] (device):
 * var = noise_start + ((noise_end - noise_start)/(eps_end - 1)) * (ep - 1) if ep <= eps_end else
 * noise_end (get_custom_linear_scaling_factor: end_scale 0 in ATT/maddpg:563-570, 0.03 in
 * MADDPG_ownENV_randomOD_Wgru_radar/maddpg_agent_randomOD_Wgru_radar.py:432-439).  Deterministic in
 * (seed, *counter); *counter (device uint64 < 2^32, as for aac_replay_sample) advances by one per call
 * in the same launch. */
int aac_noise_clamp(float *act, int32_t E, int32_t N, const int32_t *episode, int32_t eps_end, float noise_start,
                    float noise_end, uint64_t seed, uint64_t *counter, float *noise_out, void *stream);
/* The actor's output layer fused with that noise: act[r] = tanh(wa . ha[r] + ba) for R = E*N agent
 * rows of 256 features (wa = the [2][256] act_out weight, ATT/nets:213), then, with noisy != 0, the
 * noise and clamp of aac_noise_clamp (the same per-row draw; the counter advances by one per call).
 * ha and wa 16-B aligned. */
int aac_actor_out_noise(const float *ha, int64_t R, const float *wa, const float *ba, float *act, int32_t N,
                        const int32_t *episode, int32_t eps_end, float noise_start, float noise_end, uint64_t seed,
                        uint64_t *counter, int32_t noisy, float *noise_out, void *stream);

/* The actor's merge + output layers with that noise in one weights-stationary launch (ATT/nets:211-213,
 * ATT/maddpg:476-500): h_a = relu(wm cat[r] + bm) (wm [256][192], cat rows ldc apart = [e_o | e_g |
 * v_att]), act[r] = tanh(wa h_a + ba), then with noisy != 0 the noise and clamp of aac_noise_clamp (the
 * same per-row draw; the counter advances by one per call).  Replaces the merge layer's grouped-GEMM
 * launch and aac_actor_out_noise on the act path; h_a is not stored. */
int aac_actor_head_ws(const float *cat, int32_t ldc, int64_t R, const float *wm, const float *bm, const float *wa,
                      const float *ba, float *act, int32_t N, const int32_t *episode, int32_t eps_end,
                      float noise_start, float noise_end, uint64_t seed, uint64_t *counter, int32_t noisy,
                      float *noise_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* AAC_LEARN_H */
