/* aac_uam.h -- C ABI of the UAM environment in
 * libaac_env.so: the MI355X (gfx950) implementation of env_simulator.reset_world_change_skin /
 * step / ss_reward_Mar_changeskin of MADDPG_ownENV_randomOD_radar_N_model_use_tdCPA_forV2_changeskin_UAM
 * (UAM/ below).  Conventions as in aac_env.h: plain pointers, a
 * hipStream_t passed as void*, 0 / negative AAC_E* return codes, aac_uam_last_error().
 *
 * Layouts (E envs, N aircraft, K = N-1, R = 18 rays), all double (the UAM networks and their
 * inputs are float64, UAM/maddpg:148-180):
 *   own    double[E][N][7]    [nmlz_pos, vel / vmax, nmlz_pos(goal) - nmlz_pos, heading]
 *   radar  double[E][N][18]   raw distances (m), default the ray length (~5)
 *   nei    double[E][N][K][5] neighbours sorted by distance: [nmlz_pos - nmlz_pos_j, vel_j / vmax, heading]
 *   nei6   double[E][N][K][6] the p3 neighbour rows (UAM/env:1775-1788), sorted
 *   reward double[E][N] (individual, full_observable_critic_flag = False); done uint8[E][N]
 *   mask   uint8[E][N]: bit0 bound crash, bit1 cloud / runway conflict, bit2 drone collision,
 *          bit3 goal touch, bit4 goal branch taken (check_goal), bit5 collided with one of the two
 *          previously nearest neighbours (bound_building_check[3])
 *   env_done uint8[E] (UAM/main:624-637); bbc uint8[E][4]
 *   tcpa/dcpa double[E][N][K], conf_cur/conf_pre int32[E][N] (UAM/env:1745-1750), optional
 *   state: pos/vel/pre_pos/pre_vel/goal/start double[E][N][2], heading double[E][N],
 *          reach uint8[E][N], clouds double[E][2][2] (cloud / go-around aircraft centres),
 *          cloud_kind int32[E][2] (cloud_a|b, go_0..3), cloud_tgt int32[E], step int32[E],
 *          top2 uint8[E][N][2] (the two nearest neighbours of the last observation: the
 *          pre_surroundingNeighbor order ss_reward reads, UAM/env:4084-4093; 255 = none)
 */
#ifndef AAC_UAM_H
#define AAC_UAM_H

#include <stdint.h>

#include "aac_env.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct aac_uam aac_uam;

/* Replaces env_simulator.__init__ + create_world for the UAM map (UAM/env:45-207, UAM/params:14-46). */
typedef struct {
    int32_t E, N;               /* envs, aircraft per env (2 <= N <= 64)                    */
    int32_t episode_length;     /* --episode_length (UAM/main:1222)                         */
    double dt, acc_max, vmax, pB, radar_len;   /* 0.5, 0.5, 1, 0.5, 5                        */
    double bound[4];            /* 0, 40, 0, 40                                             */
} aac_uam_cfg;

typedef struct {
    double *own, *radar, *nei, *nei6, *reward;   /* nei, nei6 may be NULL                   */
    uint8_t *done, *mask, *env_done, *bbc;       /* required for step                       */
    double *tcpa, *dcpa;                          /* optional, both or neither               */
    int32_t *conf_cur, *conf_pre;                 /* optional, both or neither               */
} aac_uam_out;

int aac_uam_create(const aac_uam_cfg *cfg, int device, aac_uam **out);
void aac_uam_destroy(aac_uam *env);
const char *aac_uam_last_error(void);

/* reset_world_change_skin (UAM/env:551-771) for envs with env_mask_dev[e] != 0 (NULL = all):
 * starts / goals double[E][N][2], clouds int32[E][2] = (cloud_0 in {0: cloud_a, 1: cloud_b},
 * cloud_1 in {0..3}: go_0..go_3); writes those envs' observation rows. */
int aac_uam_reset(aac_uam *env, const uint8_t *env_mask_dev, const double *start_dev, const double *goal_dev,
                  const int32_t *clouds_dev, const aac_uam_out *out, void *stream);

/* step (UAM/env:4667-4904) + ss_reward_Mar_changeskin (UAM/env:3892-4629) + the episode
 * termination of UAM/main:624-637.  actions double[E][N][2] in [-1, 1]. */
int aac_uam_step(aac_uam *env, const double *actions_dev, const aac_uam_out *out, void *stream);

/* Episode bank for the GPU auto-reset: n whole episodes (start / goal double[n][N][2], clouds
 * int32[n][2]), host pointers.  aac_uam_auto_reset resets every env with env_done_dev[e] != 0
 * to bank entry hash(seed, e, episode[e]) (the reference draws a fresh episode per reset). */
int aac_uam_set_bank(aac_uam *env, const double *start, const double *goal, const int32_t *clouds, int32_t n,
                     uint64_t seed);
int aac_uam_auto_reset(aac_uam *env, const uint8_t *env_done_dev, const aac_uam_out *out, void *stream);
/* Process-wide: on != 0 (default, unless AAC_UAM_RESET_CONTIGUOUS=1) the auto-reset first packs the
 * resetting envs into an ordered list (one extra launch) so every reset workgroup holds epb of
 * them; 0 resets over contiguous env ranges.  Results are identical either way. */
void aac_uam_set_reset_compact(int32_t on);
/* From now on the per-env episode counter (int32[E], advanced by every auto-reset of an env) lives
 * in the caller's device buffer episode_dev (the current counts are copied into it); the caller
 * keeps it alive while the handle exists.  The copy is enqueued on `stream`. */
int aac_uam_use_episode_buffer(aac_uam *env, int32_t *episode_dev, void *stream);

/* Host: draw n episodes with the reference's rules (UAM/env:575-747, UAM/util:165-237): cloud
 * choices, starts in the two start zones re-drawn until > 3 pB from earlier starts, ends uniform
 * over the no-spawn-subtracted regions on the start's side of the runway. */
int aac_uam_bank_build(int32_t n, int32_t N, uint64_t seed, double *start, double *goal, int32_t *clouds);

/* Batched choose_action of the UAM learner (UAM/maddpg:597-676) on the fp64 matrix cores:
 * ActorNetwork_TwoPortion (UAM/nets:167-190) over R = E * N rows own double[R][7], radar
 * double[R][18] with torch nn.Linear weights (w1 [64][7], w2 [64][18], w3 [128][128], w4 [2][128],
 * row-major, float64), then (noisy != 0) + randn * var and clamp to [-1, 1], var from the row's
 * env episode[r / N] (get_custom_linear_scaling_factor, UAM/maddpg:1399-1406); counter is a
 * device uint64 incremented after the launch.  out double[R][2]. */
int aac_uam_actor(const double *own, const double *radar, int32_t R, const double *w1, const double *b1,
                  const double *w2, const double *b2, const double *w3, const double *b3, const double *w4,
                  const double *b4, double *out, int32_t N, const int32_t *episode, int32_t eps_end,
                  double noise_start, double noise_end, uint64_t seed, uint64_t *counter, int32_t noisy,
                  void *stream);
const char *aac_uam_actor_last_error(void);
/* 16-row tiles per block of aac_uam_actor (1, 2 or 4; default 4, or AAC_UAM_ACTOR_NT): the same
 * arithmetic per row for every value (tests compare them bit for bit). */
int aac_uam_actor_set_tiles(int32_t nt);

/* Device-to-device copies of the state (NULL = skip), for tests and the reference facade. */
int aac_uam_get_state(aac_uam *env, double *pos, double *vel, double *pre_pos, double *pre_vel, double *goal,
                      double *start, double *heading, uint8_t *reach, double *clouds, int32_t *cloud_kind,
                      int32_t *cloud_tgt, int32_t *step, uint8_t *top2, void *stream);
int aac_uam_set_state(aac_uam *env, const double *pos, const double *vel, const double *pre_pos,
                      const double *pre_vel, const double *goal, const double *start, const double *heading,
                      const uint8_t *reach, const double *clouds, const int32_t *cloud_kind, const int32_t *cloud_tgt,
                      const int32_t *step, const uint8_t *top2, void *stream);

/* Diagnostic (tests): n random segments of length len against a 64-gon of radius r, the radar's
 * fast ray-vs-polygon paths against the full 64-edge clip; *bad = cases whose hit flag or t differ
 * in any bit.  Synchronous (allocates, launches on the null stream, copies back). */
int aac_uam_ray_gon_check(int64_t n, uint64_t seed, double r, double len, uint64_t *bad);

#ifdef __cplusplus
}
#endif
#endif
