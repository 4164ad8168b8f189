/* aac_env.h -- C ABI of libaac_env.so, the MI355X (gfx950) implementation of the
 * Multi_agent_AAC ``one_model_att`` environment hot path.
 *
 * The reference has no FFI: its boundary is a Python method surface that ma_main drives
 * (SURVEY.md section 8(b)).  Each entry point below replaces one reference interface; the
 * Python facade ``multi_agent_aac_amd.env`` binds them with ctypes (INTEGRATION.md shows the
 * binding).  Conventions:
 *   - plain pointers and sizes only; ``stream`` is a hipStream_t passed as void* (NULL = default);
 *   - pointers named *_dev are device pointers, caller-owned (e.g. torch data_ptr());
 *   - every function returns 0 on success, a negative AAC_E* code on failure, and sets a
 *     thread-local message readable with aac_last_error();
 *   - one handle = one device, not thread-safe (the reference is single-threaded).
 *
 * Layouts (E envs, N agents, K = N-1 neighbours, D0 = 6 + 4K (6 in variant 1), R = 18 rays, W = max_wp):
 *   own  float[E][N][D0]   radar float[E][N][R]   nei float[E][N][K][6]
 *   reward float[E][N] (team sum, identical across an env's agents)
 *   done uint8[E][N]; mask uint8[E][N] bit0 bound-crash, bit1 drone-collision, bit2 goal-touch,
 *        bit3 building, bit4 waypoint-in-range, bit5 check_goal (goal branch taken)
 *   env_done uint8[E] (ATT/main:448-462 termination); bbc uint8[E][4] (bound_building_check)
 *   state: pos/vel/pre_pos/pre_vel/goal double[E][N][2]; wp double[E][N][W][2];
 *          wp_cur/wp_cnt/wall int32[E][N]; reach uint8[E][N]; step int32[E]; map_idx int32[E]
 */
#ifndef AAC_ENV_H
#define AAC_ENV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AAC_OK 0
#define AAC_E_INVALID (-1)
#define AAC_E_HIP (-2)
#define AAC_E_NOMEM (-3)
#define AAC_E_STATE (-4)

#define AAC_RADAR_DRONES 0     /* ATT/env:1051-1170 (active in one_model_att)        */
#define AAC_RADAR_OBSTACLES 1  /* OM/env:1049-1148 (occupied cells + 4 bound lines)   */
#define AAC_RADAR_COMBINED 2   /* ATT/env:879-1048 (min of both; contract R6)         */

typedef struct aac_env aac_env;

/* Static configuration; replaces env_simulator.__init__ (ATT/env:41) + create_world (ATT/env:84). */
typedef struct {
    int32_t E, N, R;            /* envs, agents per env, radar rays (must be 18)            */
    int32_t radar_mode;         /* AAC_RADAR_*                                              */
    int32_t compat;             /* 1: keep the reference's observation quirks (R7)          */
    int32_t team_reward;        /* 1: every agent gets the team sum (full_observable_critic_flag,
                                      ATT/env:2602-2603); 0: per-agent reward                 */
    int32_t max_wp;             /* waypoint capacity W per agent                            */
    int32_t episode_length;     /* --episode_length (ATT/main:918)                          */
    int32_t grid_w, grid_h;     /* occupancy grid, 23 x 13 for bound [455,680]x[255,385]    */
    int32_t n_maps;             /* >= 1 occupancy maps (multi-map configs)                  */
    double dt, acc_max, vmax, pB, radar_len;   /* 0.5, 8, 5, 2.5, 15                        */
    double bound[4];            /* xlow, xhigh, ylow, yhigh                                 */
    double cell;                /* grid length, 10 m                                        */
    const uint8_t *occ;         /* HOST: n_maps * grid_w * grid_h bytes, x-major [i][j]     */
    int32_t variant;            /* 0: one_model_att (ATT/env); 1: randomOD_Wgru_radar (config 4,
                                      WGRU/env:824-2131): requires radar_mode OBSTACLES,
                                      team_reward 0, max_wp <= 32; own rows are 6 wide (D0 = 6,
                                      scale_vel), reward per agent (WGRU/env:1666-2039), wp_cur
                                      holds the removed-waypoint bits of the goal list, bbc =
                                      [bound, building, 0, 0]; typically vmax 10, episode_length 150 */
} aac_env_cfg;

/* Caller-owned device output buffers of one step / reset. tcpa..conf_pre may be NULL. */
typedef struct {
    float *own, *radar, *nei, *reward;
    uint8_t *done, *mask, *env_done, *bbc;
    double *tcpa, *dcpa;        /* [E][N][K] current-state t_cpa / d_cpa (ATT/util:308-329) */
    int32_t *conf_cur, *conf_pre;  /* [E][N] potential-conflict counts, current / previous    */
} aac_step_out;

int aac_env_create(const aac_env_cfg *cfg, int device, aac_env **out);
void aac_env_destroy(aac_env *env);
const char *aac_last_error(void);

/* Replaces reset_world (ATT/env:199-511) for the envs with env_mask_dev[e] != 0 (NULL = all):
 * installs the given OD (start_dev [E][N][2], wps_dev [E][N][W][2], wp_cnt_dev [E][N],
 * map_idx_dev [E] or NULL = map 0) and writes those envs' observation rows to ``out``. */
int aac_env_reset(aac_env *env, const uint8_t *env_mask_dev, const double *start_dev, const double *wps_dev,
                  const int32_t *wp_cnt_dev, const int32_t *map_idx_dev, const aac_step_out *out, void *stream);

/* Replaces env.step (ATT/env:2627) + env.ss_reward (ATT/env:2105) + the termination test of
 * ATT/main:448-462 for all E envs: actions_dev float[E][N][2] in [-1, 1]. */
int aac_env_step(aac_env *env, const float *actions_dev, const aac_step_out *out, void *stream);

/* The rest of one ma_main iteration after the env step, fused into the step launch (each step
 * workgroup does it for its own envs): the replay push of the E transitions (ReplayMemory.push,
 * ATT/mem:12-15, ATT/main:363-400 -- the rows aac_replay_push_at writes), rows zeroed for the
 * finished envs (e.g. the GRU actor's next hidden states, WGRU/ma_main:476-478), and the OD-bank
 * auto-reset of the finished envs (reset_world, ATT/env:199-511).  The results equal aac_env_step,
 * then aac_replay_push_at(ring, ...), then the zeroing, then aac_env_auto_reset(env_done, out). */
typedef struct {
    float *ring;                /* replay ring float[capacity][row_width] (device); NULL = no push     */
    int32_t row_width;
    int64_t capacity, pos, size;   /* the host mirror of the ring position / fill before this push  */
    int64_t *meta;              /* device int64[2] [pos, size], advanced by the launch (for the sampler) */
    int32_t n_fields;           /* 1..12 sources, in row order                                         */
    const void *const *srcs;    /* HOST array of device pointers, source f is [E][widths[f]]; a source
                                   may be one of this step's outputs (``out``), read after the step   */
    const int32_t *widths;      /* HOST, sum = row_width                                               */
    const int32_t *dtypes;      /* HOST, 0 float32, 1 uint8 (stored as 0.0 / 1.0); NULL = all float32  */
    float *zero_rows;           /* device float[E][zero_width], rows of finished envs set to 0; or NULL */
    int32_t zero_width;
    int32_t auto_reset;         /* 1: redraw the finished envs from the OD bank (after the push)        */
    /* graph replays: when pos_in != NULL the ring position is read from that device word (pos and
     * size above are ignored); the launch stores the advanced position to pos_out (a different word)
     * and to meta[0], and the advanced size to meta[1].  Alternate the two words between steps. */
    const int64_t *pos_in;
    int64_t *pos_out;
} aac_step_tail;
int aac_env_step_tail(aac_env *env, const float *actions_dev, const aac_step_out *out, const aac_step_tail *tail,
                      void *stream);

/* Device-resident OD bank for GPU auto-reset.  Host arrays:
 * start [P][2], wps [P][W][2], cnt [P]; one entry = one agent's (start, A* waypoint list). */
int aac_env_set_od_bank(aac_env *env, const double *start, const double *wps, const int32_t *cnt,
                        int32_t n_pairs, uint64_t seed);
/* Multi-map form (MADDPG_ownENV_randomOD_radar_multipleMap: random_map_idx =
 * random.randrange(len(world_map_2D_collection)) per episode, ma_main:464-465): one bank per map of
 * the handle's map stack, concatenated map-major (n_per_map[m] entries for map m).  Each auto-reset
 * draws the env's map uniformly, then its agents' ODs from that map's bank; the env's map_idx is
 * updated.  aac_env_set_od_bank is this with n_maps = 1 (it refuses a handle with n_maps > 1). */
int aac_env_set_od_banks(aac_env *env, int32_t n_maps, const double *start, const double *wps, const int32_t *cnt,
                         const int32_t *n_per_map, uint64_t seed);

/* Re-draws the OD of every env with env_done_dev[e] != 0 from the bank (reference rule: starts
 * more than 2 pB apart, ATT/env:258-268) and overwrites those envs' rows of ``out``. */
int aac_env_auto_reset(aac_env *env, const uint8_t *env_done_dev, const aac_step_out *out, void *stream);
/* Process-wide: on > 0 the auto-reset first packs the done envs into an ordered list (one extra
 * launch) so that each reset workgroup holds epb of them; 0 resets over contiguous env ranges; < 0
 * (the default, or AAC_ENV_RESET_PACKED=0 / 1) packs for the WGRU variant only, where a large
 * share of the envs ends every step.  Results are identical either way. */
void aac_env_set_reset_compact(int32_t on);
/* Diagnostic builds only (-DAAC_ENV_STAMPS): per-workgroup phase stamps of the last step launch
 * (7 uint64 per workgroup); returns an error in a normal build. */
int aac_env_stamps(unsigned long long *out, int32_t n_wg);
/* The same for the reset kernel (7 uint64 per workgroup: realtime at entry, memtime at entry / after
 * the OD draw / after the state writes / after the radar / after the observation, realtime at exit;
 * all zero for a workgroup without a resetting env); an error in a normal build. */
int aac_env_reset_stamps(unsigned long long *out, int32_t n_wg);
/* From now on the per-env episode counter (int32[E], advanced by every auto-reset of an env) lives
 * in the caller's device buffer episode_dev (the current counts are copied into it); the caller
 * keeps it alive while the handle exists.  A trainer's noise schedule can read it directly.  The copy
 * is enqueued on `stream` (ordered after the caller's pending resets and its fill of the buffer). */
int aac_env_use_episode_buffer(aac_env *env, int32_t *episode_dev, void *stream);

/* State export / import (device pointers, each may be NULL to skip).  `start` (double2[E][N]) is
 * the episode start: the reference-path origin of the WGRU variant's cross-track reward
 * (WGRU/env:2621-2632, `ref_line` of reset_world); a state injected from another OD must carry it. */
int aac_env_get_state(aac_env *env, double *pos, double *vel, double *pre_pos, double *pre_vel, double *goal,
                      double *wp, int32_t *wp_cur, int32_t *wp_cnt, uint8_t *reach, int32_t *wall, int32_t *step,
                      int32_t *map_idx, double *start, void *stream);
int aac_env_set_state(aac_env *env, const double *pos, const double *vel, const double *pre_pos,
                      const double *pre_vel, const double *goal, const double *wp, const int32_t *wp_cur,
                      const int32_t *wp_cnt, const uint8_t *reach, const int32_t *wall, const int32_t *step,
                      const int32_t *map_idx, const double *start, void *stream);

/* Exact radar threshold bands: the most radar rays one launch flagged for the exact fix-up (a ray within
 * ~1e-9 of touching another agent's 64-gon or a cell corner, ATT/env:1089-1164, OM/env:1100-1141) and the
 * list's capacity (more would keep their float values); for variant 1 also the most rewards one step
 * listed for recomputation from the exact radar minimum (the larger of the two).  Synchronises the stream. */
int aac_env_band_max(aac_env *env, int32_t *out, int32_t *cap, void *stream);

/* Host utilities (no GPU). A* restates ATT/jps_straight.py:17-72 on a grid_w x grid_h x-major
 * grid (0 = free); writes up to max_len (x, y) cells, returns the path length or 0 if none. */
int aac_astar(const uint8_t *grid, int32_t w, int32_t h, int32_t sx, int32_t sy, int32_t ex, int32_t ey,
              int32_t *path_xy, int32_t max_len);

/* Builds an OD bank of n_pairs entries drawn with the reference rule (ATT/env:251-347): start
 * quadrant uniform, target quadrant uniform among the other three, cells uniform in the
 * ``target_pool`` lists, A* + turning-point refinement.  Returns the largest waypoint count
 * seen (> max_wp means entries were truncated: treat as an error), or < 0 on error. */
int aac_od_bank_build(const uint8_t *occ, int32_t w, int32_t h, const double *bound, double cell,
                      int32_t n_pairs, uint64_t seed, int32_t max_wp, double *start, double *wps, int32_t *cnt);

#ifdef __cplusplus
}
#endif
#endif /* AAC_ENV_H */
