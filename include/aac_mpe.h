/* aac_mpe.h -- C ABI of the batched MPE simple_spread environment in libaac_env.so (gfx950):
 * SURVEY.md section 8(f) row f4 (config 1, MADDPG_SS_baseV3, ``SS/`` below).
 *
 * It replaces, for E environments at once, MultiAgentEnv.step (SS/env/multiagent/environment.py:
 * 80-103) with World.step (SS/env/multiagent/core.py:116-195) and the simple_spread reward /
 * observation (SS/env/multiagent/scenarios/simple_spread.py:46-100), and reset_world (:32-44).
 * State is fp64 as the reference's numpy; the action force is the float32 product u * 5 of
 * _set_action (environment.py:193-197).  One thread per environment.
 *
 * Layouts (device pointers): pos, vel [E][N][2] f64; lmk [E][L][2] f64; act [E][N][2] f32;
 * obs [E][N][4 + 2L + 4(N-1)] f32 = [vel, pos, lmk_j - pos, pos_k - pos (k != i), comm_k (zeros)];
 * rew [E][N] f64.  N <= AAC_MPE_MAX_AGENTS, L <= AAC_MPE_MAX_LANDMARKS.
 */
#ifndef AAC_MPE_H
#define AAC_MPE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AAC_MPE_MAX_AGENTS 8
#define AAC_MPE_MAX_LANDMARKS 8

const char *aac_mpe_last_error(void);

/* One step of every environment: physics, then obs and rewards of the new state. */
int aac_mpe_step(double *pos, double *vel, const double *lmk, const float *act, int32_t E, int32_t N, int32_t L,
                 float *obs, double *rew, void *stream);

/* Observation and rewards of the current state (after a reset). */
int aac_mpe_observe(const double *pos, const double *vel, const double *lmk, int32_t E, int32_t N, int32_t L,
                    float *obs, double *rew, void *stream);

/* reset_world for envs with env_mask[e] != 0 (NULL = all): agent then landmark positions uniform
 * in [-1, 1) from a counter-based hash RNG (seed, *counter, env, draw index), velocities 0;
 * *counter is incremented on the stream. */
int aac_mpe_reset(double *pos, double *vel, double *lmk, int32_t E, int32_t N, int32_t L, const uint8_t *env_mask,
                  uint64_t seed, uint64_t *counter, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* AAC_MPE_H */
