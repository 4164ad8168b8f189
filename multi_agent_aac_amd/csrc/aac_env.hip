// aac_env.hip -- gfx950 kernels + C ABI for the one_model_att environment hot path.
//
// One thread per (env, agent); a 256-thread workgroup owns floor(256/N) whole envs, so every
// neighbour interaction (radar vs other drones, tdCPA, collisions, team reward) stays inside the
// workgroup and goes through LDS -- no inter-workgroup communication at all.  State is SoA double2
// in HBM (16 B per lane, coalesced), observations are written as fp32.  No MFMA: this is byte- and
// fp64-branch work bounded by HBM.
//
// Arithmetic contract (shared with oracle/aac_oracle.c, compiled -ffp-contract=off):
//   np.linalg.norm([x,y]) = sqrt(fma(y,y,x*x)); np.dot = fma(a1,b1,a0*b0); GEOS distance has no FMA;
//   np.sum over the N team rewards = numpy pairwise summation.
// Reference: ATT/env:2627-2713 kinematics, :758-773 neighbours, :1051-1170 radar (drones),
// OM/env:1049-1148 radar (obstacles), :1285-1469 observation, ATT/util:308-329 tdCPA,
// ATT/env:2105-2618 ss_reward, ATT/main:448-462 termination, ATT/env:199-405 reset.
// variant 1 = the randomOD_Wgru_radar env of config 4 (WGRU/env:824-1054 observation, :1666-2039
// ss_reward, :2048-2131 step, WGRU/ma_main:653-661 termination): obstacle radar, 6-wide own rows,
// per-agent reward against the next waypoint and the reference path (oracle/wgru_env_ref.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/aac_env.h"
#include "aac_geom.h"
#include "aac_wave.h"

#define BLOCK 256
// the exact goal / building threshold tests as real calls (1) or inline (0), per env variant: whichever
// the variant's step kernel runs faster with (they only execute within 1e-9 of a threshold)
#ifndef AAC_EXACT_COLD_ATT
#define AAC_EXACT_COLD_ATT 0
#endif
#ifndef AAC_EXACT_COLD_WGRU
#define AAC_EXACT_COLD_WGRU 1
#endif
#define EXACT_COLD(V) ((V) == 0 ? AAC_EXACT_COLD_ATT != 0 : AAC_EXACT_COLD_WGRU != 0)
#define MAX_MAP_BYTES 8192
#ifndef AAC_ENV_MIN_WAVES         // minimum waves per SIMD the step kernel is compiled for: 4 keeps
#define AAC_ENV_MIN_WAVES 4       // 4 workgroups per CU resident (179 -> 128 VGPRs, a few spilled to
#endif                            // scratch on cold paths); 2 waves: 1.75x slower at 262 144 envs
// observation rows staged in LDS for coalesced 16-B stores (floats per workgroup, else direct)
#define OBS_STAGE_FLOATS 2560
#define WPC 8            // variant 1: waypoints per agent kept in LDS by the step kernel

namespace {

struct Args {
    int E, N, K, D0, W, radar_mode, compat, team_reward, episode_length, gw, gh, n_maps, epb, variant;
    double bound[4];
    double gx0, gy0, xs, ys;
    double dt, acc_max, vmax, pb, radar_len;
    double2 *pos, *vel, *pre_pos, *pre_vel, *goal, *wp, *start;
    double2 *wp0;        // [E][N] = wp[cur] (variant 0): the step reads it coalesced instead of gathering
    int32_t *wp_cur, *wp_cnt, *wall, *step, *map_idx;   // variant 1: wp_cur = removed-waypoint bits
    uint8_t *reach;
    const uint8_t *occ;  // n_maps * gw * gh
    const unsigned long long *occ_rows;   // n_maps * gw row bit masks (bit j = cell (i, j)); gh <= 64
    float *own, *radar, *nei, *reward;
    uint8_t *done, *mask, *env_done, *bbc;
    double *tcpa, *dcpa;
    int32_t *conf_cur, *conf_pre;
    // radar rays with a threshold-band case (radar_phase): header + the env's N positions per entry,
    // resolved exactly by band_fix_kernel after the launch
    struct BandHdr *band_hdr;
    double2 *band_pos;
    int32_t *band_cnt;   // [0] entries this launch (zeroed by band_fix_kernel), [1] most ever (overflow check),
                         // [2] / [3] the same for rfix
    int band_cap;
    // variant 1 step: agents with a flagged ray, whose reward's near-building penalty (the radar minimum)
    // band_fix_kernel recomputes from the exact radar (the kernel's minimum is the float one)
    struct RewFix *rfix;
};

// a variant-1 agent whose reward band_fix_kernel recomputes: r = rp - nbp(rmin) (kind 1), (rp - nbp) +
// 0.0 (kind 2, the normal-step branch), rp (kind 0: no penalty term), rmin over the agent's exact rays
struct RewFix {
    int32_t e, i, map, kind;
    double rp;
    double2 pos;
    int64_t row;          // ring row of the env's transition (reward column), -1: none
};

// one flagged radar ray: env, agent, ray, kind (0 step: radar output + ring column, 1 reset: radar
// output), the env's map, the ring row of its transition (-1: none)
struct BandHdr {
    int32_t e, i, r, kind, map, pad;
    int64_t row;
};

struct ResetArgs {
    int mode;                 // 0 explicit OD, 1 bank
    const uint8_t *mask;      // env mask (explicit) or env_done (bank); NULL = all
    const double2 *start;     // explicit [E][N]
    const double2 *wps;       // explicit [E][N][W]
    const int32_t *cnt;       // explicit [E][N]
    const int32_t *map_idx;   // explicit [E] or NULL
    const double2 *bank_start, *bank_wp;
    const int32_t *bank_cnt;
    int32_t bank_n;
    const int32_t *bank_off;  // [bank_maps + 1] first entry of each map's bank (multi-map)
    int32_t bank_maps;        // 1: one bank, every env on map 0; > 1: map drawn per episode
    uint64_t seed;
    int32_t *episode;         // [E] per-env episode counter (bank mode)
    const int32_t *list;      // [count, env...] of the resetting envs (env_compact_kernel); NULL:
                              // workgroup b takes envs b*epb ... (mask-filtered)
};

// The fused step tail (aac_env_step_tail): the replay push of this step's transitions, rows zeroed for
// the finished envs, and their auto-reset, run by each step workgroup for its own envs.  The push's
// fields are split by the host: "early" fields (sources written by earlier launches: the current
// observations, the actions, hidden states) are copied at kernel start; the fields that are this
// step's outputs (next own / radar / nei rows, reward, done) are written into the ring where the
// step produces them ("late" columns), so nothing is read back.
#define TAIL_MAX_FIELDS 12
enum { LATE_OWN, LATE_RADAR, LATE_NEI, LATE_REW, LATE_DONE, LATE_N };
struct Tail {
    float *ring;              // replay ring [cap][rw]; null = no push
    int rw, nf;               // row width; number of early fields
    int64_t cap, pos;         // host mirror of the ring position before this push
    int64_t *meta;            // device [pos, size] for the sampler, stored by workgroup 0
    int64_t new_pos, new_size;
    const int64_t *pos_in;    // non-null: the position is read here (ignoring pos) and the advanced one is
    int64_t *pos_out;         // stored to pos_out (another word: every workgroup reads pos_in), size in meta
    const void *src[TAIL_MAX_FIELDS];          // early fields: [E][width] sources
    int width[TAIL_MAX_FIELDS], col[TAIL_MAX_FIELDS], dtype[TAIL_MAX_FIELDS];   // col: first ring column
    int cum[TAIL_MAX_FIELDS + 1];              // early fields' running column counts (cum[nf] = n_early)
    int late[LATE_N];         // first ring column of each step output, -1 = not pushed
    float *zero_rows;         // [E][zero_w] rows zeroed for the finished envs (after the push); null = none
    int zero_w;
    int reset;                // 1: auto-reset the finished envs from the OD bank (after the push)
    int spec;                 // 1: their OD draws made during the step by the agent-free waves (spec_draw)
    int tab_off;              // float offset of the early fields' column table in the staging area (its end)
    int late_copy;            // 1: the early fields are copied by the agent-free waves during the agent phase
};

// ring row of env e for this push (pos < cap, e < E <= cap)
__device__ inline float *ring_row(const Tail &T, int64_t pos, int e) {
    int64_t row = pos + e;
    if (row >= T.cap) row -= T.cap;
    return T.ring + row * T.rw;
}

// LineString([p0,p1]).buffer(pB) meets one of the 4 infinite bound lines (ATT/env:2507)
__device__ inline bool bound_crash(const Args &A, double x0, double y0, double x1, double y1) {
    return capsule_crash(A.pb, A.bound, x0, y0, x1, y1);
}

// 64-gon(pos, pB) meets 64-gon(goal, 1) (ATT/env:2266-2269); exact within the threshold band
template <bool COLD>
__device__ inline bool goal_reached(double px, double py, double gx, double gy, double pb) {
    return goal_meet_exact<COLD>(px, py, gx, gy, pb);
}

// 64-gon(pos, pB) meets the closed square cell (ATT/env:2243-2250): separating axes; an axis within
// EXACT_BAND of separating hands the decision to the exact test on the GEOS float vertices
template <bool COLD>
__device__ __attribute__((always_inline)) bool building_hit(double px, double py, double cx, double cy, double pb) {
    double dx = cx - px, dy = cy - py;
    if (fabs(dx) > 5.0 + pb + EXACT_BAND || fabs(dy) > 5.0 + pb + EXACT_BAND) return false;
    bool unsure = fabs(dx) > 5.0 + pb - EXACT_BAND || fabs(dy) > 5.0 + pb - EXACT_BAND;
    // the 64-gon lies between its inscribed (pb cos(pi/64)) and circumscribed (pb) circles:
    // away from that band the distance to the square decides
    {
        const double ox = fmax(fabs(dx) - 5.0, 0.0), oy = fmax(fabs(dy) - 5.0, 0.0);
        const double dist = sqrt(ox * ox + oy * oy);
        if (dist > pb * (1.0 + 1e-12) + 1e-12) return false;
        if (dist < pb * c_tab.apothem * (1.0 - 1e-12) - 1e-12) return true;
    }
    // not unrolled: unrolled, the compiler hoisted the 32 loop-invariant limits out of the caller's
    // cell loop and kept them live across the whole agent phase (64 VGPRs, spilled to scratch)
#pragma unroll 1
    for (int k = 0; k < 32; ++k) {
        double proj = fabs(dx * c_tab.nrm_c[k] + dy * c_tab.nrm_s[k]);
        double lim = 5.0 * (fabs(c_tab.nrm_c[k]) + fabs(c_tab.nrm_s[k])) + pb * c_tab.apothem;
        if (proj > lim + EXACT_BAND) return false;
        unsure |= proj > lim - EXACT_BAND;
    }
    if (!unsure) return true;
    const int m = COLD ? gon_square_meet_call(px, py, pb, cx - 5.0, cx + 5.0, cy - 5.0, cy + 5.0)
                       : gon_square_meet(px, py, pb, cx - 5.0, cx + 5.0, cy - 5.0, cy + 5.0);
    if (m >= 0) return m == 1;
    // undecidable: the closed form
    if (fabs(dx) > 5.0 + pb || fabs(dy) > 5.0 + pb) return false;
#pragma unroll 1
    for (int k = 0; k < 32; ++k) {
        double proj = fabs(dx * c_tab.nrm_c[k] + dy * c_tab.nrm_s[k]);
        double lim = 5.0 * (fabs(c_tab.nrm_c[k]) + fabs(c_tab.nrm_s[k])) + pb * c_tab.apothem;
        if (proj > lim) return false;
    }
    return true;
}

// occupied cells that can meet the segment c -> e (a bit per cell of the bounding box, bit
// (i - i0) * 8 + (j - j0)), then the exact entry into each.  Collecting first keeps the wave's
// lanes together: the per-cell loop ran the slab test whenever any lane of the wave had a
// candidate in that cell slot, the candidate loop runs it max-popcount times.  The minimum does
// not depend on the order (OM/env:1089-1141 takes the nearest intersection).
template <int EX>
__device__ __attribute__((always_inline)) double radar_obstacles(const Args &A, const uint8_t *occ, const unsigned long long *rows, double cx,
                                  double cy, double ex, double ey, double len, bool &band, int mode) {
    double mind = len, d;
    // only cells whose square meets the segment's bounding box can meet the segment (index range
    // by a product with 0.1: it rounds within an ulp of the quotient, and floor / ceil of it still
    // bracket the cells ceil((lo - 5) / 10) .. floor((hi + 5) / 10) that can touch the box)
    int i0 = (int)floor((fmin(cx, ex) - 5.0 - A.gx0) * 0.1), i1 = (int)ceil((fmax(cx, ex) + 5.0 - A.gx0) * 0.1);
    int j0 = (int)floor((fmin(cy, ey) - 5.0 - A.gy0) * 0.1), j1 = (int)ceil((fmax(cy, ey) + 5.0 - A.gy0) * 0.1);
    i0 = i0 < 0 ? 0 : i0;
    j0 = j0 < 0 ? 0 : j0;
    i1 = i1 > A.gw - 1 ? A.gw - 1 : i1;
    j1 = j1 > A.gh - 1 ? A.gh - 1 : j1;
    // a square of half-size 5 centred at q meets the segment only if q lies within its support
    // half-width 5 (|ux| + |uy|) of the segment's line and of its extent along the line (u the
    // unit direction; everything below is scaled by L: no division).  A conservative pre-filter
    // (relative margin 1e-9, far above the rounding of these few products): the slab test decides.
    const double ddx = ex - cx, ddy = ey - cy;
    const double L2 = ddx * ddx + ddy * ddy;
    const double reach = 5.0 * (fabs(ddx) + fabs(ddy)) * (1.0 + 1e-9) + 1e-12;
    if (i1 < i0 || j1 < j0) {
        // the box lies off the grid: no cell
    } else if (rows && i1 - i0 < 8 && j1 - j0 < 8) {
        // the box's occupied cells from the row masks (one 8-B LDS read per row, all issued
        // up front), the line filter on those only
        const unsigned long long span = (2ull << (j1 - j0)) - 1;
        unsigned long long rb[8];
#pragma unroll
        for (int di = 0; di < 8; ++di) rb[di] = rows[i0 + di <= i1 ? i0 + di : 0];
        unsigned long long cand = 0;
        double almin = INFINITY;
        int bmin = 0;
#pragma unroll
        for (int di = 0; di < 8; ++di) {
            unsigned long long row = i0 + di <= i1 ? (rb[di] >> j0) & span : 0ull;
            const double wx = A.gx0 + 10.0 * (i0 + di) - cx;
            while (row) {
                const int b = __builtin_ctzll(row);
                row &= row - 1;
                const double wy = A.gy0 + 10.0 * (j0 + b) - cy;
                const double cr = wx * ddy - wy * ddx, al = wx * ddx + wy * ddy;
                if (fabs(cr) <= reach && al >= -reach && al <= L2 + reach) {
                    cand |= 1ull << (di * 8 + b);
                    if (al < almin) {
                        almin = al;
                        bmin = di * 8 + b;
                    }
                }
            }
        }
#ifdef AAC_DBG_NO_SQUARE      // timing experiments only
        mind -= (double)__popcll(cand) * 1e-30;
        cand = 0;
#endif
        // the candidate nearest along the ray first; then a square whose every point projects past
        // the current minimum cannot lower it: its hit distance is at least (al - 5(|dx| + |dy|)) / L
        // (al, reach scaled by L), so it is skipped when (al - reach)^2 > mind^2 L^2 (1 + 1e-8) -- the
        // relative margin far above the rounding of d, so the minimum is the one the full loop finds
        if (cand) {
            const double qx = A.gx0 + 10.0 * (i0 + (bmin >> 3)), qy = A.gy0 + 10.0 * (j0 + (bmin & 7));
            if (ray_square<EX>(cx, cy, ex, ey, qx - 5.0, qx + 5.0, qy - 5.0, qy + 5.0, d, band, mode) && d <= mind) mind = d;
            cand &= ~(1ull << bmin);
        }
        while (cand) {
            const int b = __builtin_ctzll(cand);
            cand &= cand - 1;
            const double qx = A.gx0 + 10.0 * (i0 + (b >> 3)), qy = A.gy0 + 10.0 * (j0 + (b & 7));
            const double lb = (qx - cx) * ddx + (qy - cy) * ddy - reach;
            if (lb > 0.0 && lb * lb > mind * mind * L2 * (1.0 + 1e-8)) continue;
            if (ray_square<EX>(cx, cy, ex, ey, qx - 5.0, qx + 5.0, qy - 5.0, qy + 5.0, d, band, mode) && d <= mind) mind = d;
        }
    } else {      // a radar longer than the 8 x 8-cell mask covers, or maps taller than 64 cells
        for (int i = i0; i <= i1; ++i)
            for (int j = j0; j <= j1; ++j) {
                if (!occ[i * A.gh + j]) continue;
                const double qx = A.gx0 + 10.0 * i, qy = A.gy0 + 10.0 * j;
                const double wx = qx - cx, wy = qy - cy;
                const double cr = wx * ddy - wy * ddx, al = wx * ddx + wy * ddy;
                if (fabs(cr) > reach || al < -reach || al > L2 + reach) continue;
                if (ray_square<EX>(cx, cy, ex, ey, qx - 5.0, qx + 5.0, qy - 5.0, qy + 5.0, d, band, mode) && d <= mind) mind = d;
            }
    }
#ifdef AAC_DBG_NO_LINES
    return mind;
#endif
    if (ray_vline(cx, cy, ex, ey, A.bound[0], d) && d < mind) mind = d;
    if (ray_vline(cx, cy, ex, ey, A.bound[1], d) && d < mind) mind = d;
    if (ray_hline(cx, cy, ex, ey, A.bound[2], d) && d < mind) mind = d;
    if (ray_hline(cx, cy, ex, ey, A.bound[3], d) && d < mind) mind = d;
    return mind;
}

// LDS image of one workgroup's envs (A = epb * N agents, <= BLOCK)
struct Lds {
    double2 pos[BLOCK], vel[BLOCK], ppos[BLOCK], pvel[BLOCK], goal[BLOCK];
    double rew[BLOCK];
    uint8_t flags[BLOCK];   // bit0 done, bit1 check_goal, bit2 reach, bit3 bound, bit4 drone, bit5 last==nearest
    uint8_t active[BLOCK];  // per local env (reset kernel)
    int32_t idx[BLOCK];
    unsigned long long rmin[BLOCK];   // variant 1: per agent, the smallest radar distance (float64 bits)
    alignas(16) float obs[OBS_STAGE_FLOATS];   // the workgroup's own | nei rows (step kernel, when they fit)
};
// the occupancy maps follow the static LDS image as dynamic LDS: n_maps * gw * gh bytes, then
// (8-B aligned) the n_maps * gw row masks when the handle has them
extern __shared__ uint8_t s_maps[];

__device__ inline int rows_off(const Args &A) { return (A.n_maps * A.gw * A.gh + 7) & ~7; }

// variant 1: after the maps (and row masks), 16-B aligned, the first WPC waypoints of each of the
// workgroup's agents (wp_cache_bytes on the host side)
__device__ inline double2 *wp_cache(const Args &A) {
    const int end = A.occ_rows ? rows_off(A) + 8 * A.n_maps * A.gw : A.n_maps * A.gw * A.gh;
    return reinterpret_cast<double2 *>(s_maps + ((end + 15) & ~15));
}

__device__ inline const unsigned long long *map_rows(const Args &A, int m) {
    return A.occ_rows ? reinterpret_cast<const unsigned long long *>(s_maps + rows_off(A)) + m * A.gw : nullptr;
}

// own + neighbour observation and tdCPA of agent i of env e (ATT/env:1285-1469)
__device__ __attribute__((always_inline)) void observe_agent(const Args &A, const Lds &S, int e, int i, int base, float *own = nullptr,
                              float *nei = nullptr) {
    const int N = A.N, K = A.K;
    const size_t ai = (size_t)e * N + i;
    const double *b = A.bound;
    const double pb = A.pb, vmax = A.vmax;
    const double2 p = S.pos[base + i], v = S.vel[base + i];
    const double px = p.x, py = p.y;
    if (!own) own = A.own + ai * A.D0;          // rows in global memory, or staged in LDS
    if (!nei) nei = A.nei + ai * K * 6;
    double npx = -1 + (px - b[0]) * A.xs, npy = -1 + (py - b[2]) * A.ys;
    const double2 g = S.goal[base + i];
    double ngx = 2 * ((g.x - b[0]) / (b[1] - b[0])) - 1, ngy = 2 * ((g.y - b[2]) / (b[3] - b[2])) - 1;
    own[0] = (float)npx;
    own[1] = (float)npy;
    if (A.variant) {      // scale_vel (WGRU/env:971)
        own[2] = (float)(A.xs * v.x);
        own[3] = (float)(A.ys * v.y);
    } else {
        own[2] = (float)(v.x / vmax);
        own[3] = (float)(v.y / vmax);
    }
    own[4] = (float)(ngx - npx);
    own[5] = (float)(ngy - npy);
    const double dxm = b[0] - b[1], dxM = b[1] - b[0], dym = b[2] - b[3], dyM = b[3] - b[2];
    int kk = 0, cc = 0, cp = 0;
    const double2 hp = S.ppos[base + i], hv = S.pvel[base + i];
    for (int j = 0; j < N; ++j) {
        if (j == i) continue;
        const double2 q = S.pos[base + j], w = S.vel[base + j];
        double dx = q.x - px, dy = q.y - py;
        if (!A.variant) {     // the own row's neighbour part (ATT only; WGRU own rows are 6 wide)
            if (A.compat) {
                own[6 + 4 * kk] = (float)(-1 + (dx - b[0]) * A.xs);
                own[7 + 4 * kk] = (float)(-1 + (dy - b[2]) * A.ys);
            } else {
                own[6 + 4 * kk] = (float)(A.xs * dx);
                own[7 + 4 * kk] = (float)(A.ys * dy);
            }
            own[8 + 4 * kk] = (float)(w.x / vmax);
            own[9 + 4 * kk] = (float)(w.y / vmax);
        }
        float *nb = nei + kk * 6;
        nb[0] = (float)(2 * ((dx - dxm) / (dxM - dxm)) - 1);
        nb[1] = (float)(2 * ((dy - dym) / (dyM - dym)) - 1);
        double g0, g1;
        if (A.compat) {
            g0 = w.y - q.x;
            g1 = pb - q.y;
        } else {
            g0 = S.goal[base + j].x - q.x;
            g1 = S.goal[base + j].y - q.y;
        }
        nb[2] = (float)(2 * ((g0 - dxm) / (dxM - dxm)) - 1);
        nb[3] = (float)(2 * ((g1 - dym) / (dyM - dym)) - 1);
        nb[4] = (float)(w.x / vmax);
        nb[5] = (float)(w.y / vmax);
        if (A.tcpa || A.conf_cur) {
            double t, d, t2, d2;
            tdcpa(q.x, q.y, px, py, w.x, w.y, v.x, v.y, pb, t, d, cc);
            const double2 qp = S.ppos[base + j], wp = S.pvel[base + j];
            tdcpa(qp.x, qp.y, hp.x, hp.y, wp.x, wp.y, hv.x, hv.y, pb, t2, d2, cp);
            if (A.tcpa) {
                A.tcpa[ai * K + kk] = t;
                A.dcpa[ai * K + kk] = d;
            }
        }
        ++kk;
    }
    if (A.conf_cur) {
        A.conf_cur[ai] = cc;
        A.conf_pre[ai] = cp;
    }
}

// one radar ray r of agent i (ATT/env:1089-1164 drones, OM/env:1089-1141 obstacles)
// EX = 1: the threshold bands (ray_poly_entry_full): mode 1 flags a ray with a band case in band and
// returns the float answer, mode 2 decides its band cases exactly
template <int EX>
__device__ __attribute__((always_inline)) double radar_ray(const Args &A, const Lds &S, int i, int r, int base, const uint8_t *occ,
                            const unsigned long long *rows, bool &band, int mode) {
    const int N = A.N;
    const double pb = A.pb;
    const double2 p = S.pos[base + i];
    const double px = p.x, py = p.y;
    const double ex = px + A.radar_len * c_tab.ray_c[r], ey = py + A.radar_len * c_tab.ray_s[r];
    const double len = gdist(ex, ey, px, py);
    double dd = len, dob = len;
    if (A.radar_mode != AAC_RADAR_OBSTACLES) {
        // neighbours whose 64-gon can meet the segment (closest point within pb: the GEOS 64-gon
        // lies inside the circle of radius pb (+1e-15)), collected per 64 as a mask, then the
        // exact entry for each candidate (same lane-compaction argument as radar_obstacles)
        const double reach2 = (pb + 1e-6) * (pb + 1e-6);
        const double ddx = ex - px, ddy = ey - py;
        const double inv = 1.0 / (ddx * ddx + ddy * ddy);
        double shortest = INFINITY;       // the nearest hit replaces len (even a rounding above it)
        for (int j0 = 0; j0 < N; j0 += 64) {
            const int jn = N - j0 < 64 ? N - j0 : 64;
            unsigned long long cand = 0;
            for (int jj = 0; jj < jn; ++jj) {
                const double2 q = S.pos[base + j0 + jj];
                const double wx = q.x - px, wy = q.y - py;
                double tt = (wx * ddx + wy * ddy) * inv;
                tt = tt < 0.0 ? 0.0 : (tt > 1.0 ? 1.0 : tt);
                const double qx = tt * ddx - wx, qy = tt * ddy - wy;
                if (j0 + jj != i && qx * qx + qy * qy <= reach2) cand |= 1ull << jj;
            }
            while (cand) {
                const int j = j0 + __builtin_ctzll(cand);
                cand &= cand - 1;
                const double2 q = S.pos[base + j];
                double t;
                if (!ray_poly_entry<EX>(px, py, ex, ey, q.x, q.y, pb, t, band, mode)) continue;
                const double ix = px + t * (ex - px), iy = py + t * (ey - py);
                const double d = gdist(ix, iy, px, py);
                shortest = d < shortest ? d : shortest;
            }
        }
        if (shortest < INFINITY) dd = shortest;
    }
    if (A.radar_mode != AAC_RADAR_DRONES) dob = radar_obstacles<EX>(A, occ, rows, px, py, ex, ey, len, band, mode);
    return A.radar_mode == AAC_RADAR_DRONES ? dd : (A.radar_mode == AAC_RADAR_OBSTACLES ? dob : (dd < dob ? dd : dob));
}

__device__ inline void load_maps(const Args &A) {
    const int bytes = A.n_maps * A.gw * A.gh;
    for (int k = threadIdx.x; k < bytes; k += BLOCK) s_maps[k] = A.occ[k];
    if (A.occ_rows) {
        unsigned long long *r = reinterpret_cast<unsigned long long *>(s_maps + rows_off(A));
        for (int k = threadIdx.x; k < A.n_maps * A.gw; k += BLOCK) r[k] = A.occ_rows[k];
    }
}

// all radar rays of the workgroup's (active) agents: one work item per (agent, ray); rmin (variant
// 1 step): each agent's smallest float64 distance, as an LDS atomic min on the (non-negative) bits
// the fused step tail's late radar column (RingOut.ring null = none): ring row of env e, column col
struct RingOut {
    float *ring;
    int64_t pos, cap;
    int rw, col;
};

__device__ inline void radar_out(const Args &A, Lds &S, int e, int i, int r, int la, bool rmin, const RingOut &ro,
                                 double d) {
    A.radar[((size_t)e * A.N + i) * NRAY + r] = (float)d;
    if (ro.ring) {
        int64_t row = ro.pos + e;
        if (row >= ro.cap) row -= ro.cap;
        ro.ring[row * ro.rw + ro.col + i * NRAY + r] = (float)d;
    }
    if (rmin) atomicMin(&S.rmin[la], (unsigned long long)__double_as_longlong(d));
}

// Exact radar (threshold bands, ray_poly_entry_full): the radar code here only flags a ray with a band
// case -- within ~1e-9 of touching a 64-gon or a cell corner away from the segment's end, rare -- and
// writes its float value; the ray (with its env's positions) goes to the band list, and
// band_fix_kernel, launched right after this kernel, re-runs it exactly and rewrites the outputs.
// Resolved in this kernel, the exact code slowed the step kernels' hot phases by ~10 us (inlined:
// register allocation and scheduling; as calls from the radar loop: scratch spills).  kind: 0 step
// (row: the ring row of the env's transition, or -1), 1 reset.
__device__ __attribute__((always_inline)) void radar_phase(const Args &A, Lds &S, int e0, int nagents,
                                                           bool check_active, const int32_t *emap = nullptr,
                                                           bool rmin = false, RingOut ro = RingOut{}, int kind = 0) {
    static_assert(NRAY <= 32 && BLOCK == 256, "a thread's work items (nagents <= BLOCK: k < NRAY) index a 32-bit mask");
    uint32_t flagged = 0;     // this thread's work items w = threadIdx.x + k BLOCK with a band case
    for (int w = threadIdx.x; w < nagents * NRAY; w += BLOCK) {
        const int la = w / NRAY, r = w - la * NRAY;
        const int le = la / A.N, i = la - le * A.N;
        const int e = emap ? emap[le] : e0 + le;
        if (e >= A.E) continue;
        if (check_active && !S.active[le]) continue;
        const int mi = A.map_idx ? A.map_idx[e] : 0;
        bool band = false;
        const double d = radar_ray<1>(A, S, i, r, le * A.N, s_maps + mi * A.gw * A.gh, map_rows(A, mi), band, 1);
        radar_out(A, S, e, i, r, la, rmin, ro, d);
        if (band) flagged |= 1u << (w >> 8);
    }
    // the flagged rays (with their env's positions) into the band list, outside the loop's registers
    while (flagged && A.band_cnt) {
        const int w = threadIdx.x + __builtin_ctz(flagged) * BLOCK;
        flagged &= flagged - 1;
        const int la = w / NRAY, r = w - la * NRAY;
        const int le = la / A.N, i = la - le * A.N;
        const int e = emap ? emap[le] : e0 + le;
        const int slot = atomicAdd(A.band_cnt, 1);
        if (slot >= A.band_cap) continue;
        // variant 1 step: the agent's reward uses its radar minimum -- mark it for the fix-up (S.flags
        // bit 7, zeroed before the radar phase; the agent phase reads it after the barrier)
        if (rmin) atomicOr(reinterpret_cast<unsigned *>(&S.flags[la & ~3]), 0x80u << (8 * (la & 3)));
        int64_t row = -1;
        if (ro.ring) {
            row = ro.pos + e;
            if (row >= ro.cap) row -= ro.cap;
        }
        A.band_hdr[slot] = BandHdr{e, i, r, kind, A.map_idx ? A.map_idx[e] : 0, 0, row};
        for (int j = 0; j < A.N; ++j) A.band_pos[(size_t)slot * A.N + j] = S.pos[le * A.N + j];
    }
}

#ifndef AAC_ENV_AGENT_STAMPS
#define ASTAMP(k) \
    do {          \
    } while (0)
#endif
#ifdef AAC_ENV_STAMPS
// diagnostic build only (tools/env_stamps.py): per-workgroup s_memtime at entry, after kinematics,
// after the radar, after the agent phase and at exit, plus s_memrealtime at entry / exit
constexpr int ESTAMP_WG = 65536;
__device__ unsigned long long g_env_st[ESTAMP_WG][7];
#define ESTAMP(k, v)                                                                                    \
    do {                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < ESTAMP_WG) g_env_st[blockIdx.x][k] = (v);                \
    } while (0)
// reset_kernel: [s_memrealtime at entry, s_memtime at entry / after the OD draw / after the state
// writes / after the radar / after the observation, s_memrealtime at exit]; zero = workgroup idle
__device__ unsigned long long g_reset_st[ESTAMP_WG][7];
#define RSTAMP(k, v)                                                                                    \
    do {                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < ESTAMP_WG) g_reset_st[blockIdx.x][k] = (v);              \
    } while (0)
#ifdef AAC_ENV_AGENT_STAMPS      // agent-phase sub-stamps of thread 0, into the reset stamp array (step only)
#define ASTAMP(k)                                                                                       \
    do {                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < ESTAMP_WG) g_reset_st[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#endif
#else
#define ESTAMP(k, v) \
    do {             \
    } while (0)
#define RSTAMP(k, v) \
    do {             \
    } while (0)
#endif

// ------------------------------------------------------------- variant 1 (randomOD_Wgru_radar)
// GEOS algorithm::Distance::pointToSegment and LineSegment::closestPoint (oracle/geos.py)
__device__ __attribute__((always_inline)) double point_to_segment(double px, double py, double ax, double ay, double bx, double by) {
    if (ax == bx && ay == by) return gdist(px, py, ax, ay);
    const double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
    const double r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
    if (r <= 0.0) return gdist(px, py, ax, ay);
    if (r >= 1.0) return gdist(px, py, bx, by);
    const double sv = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
    return fabs(sv) * sqrt(len2);
}

__device__ __attribute__((always_inline)) double2 segment_closest_point(double px, double py, double ax, double ay, double bx, double by) {
    double f;
    if (px == ax && py == ay) f = 0.0;
    else if (px == bx && py == by) f = 1.0;
    else {
        const double dx = bx - ax, dy = by - ay;
        f = ((px - ax) * dx + (py - ay) * dy) / (dx * dx + dy * dy);
    }
    if (f > 0 && f < 1) return make_double2(ax + f * (bx - ax), ay + f * (by - ay));
    return gdist(ax, ay, px, py) < gdist(bx, by, px, py) ? make_double2(ax, ay) : make_double2(bx, by);
}

// ss_reward of one agent (WGRU/env:1666-2039): the next-waypoint search pops goal-list entries (the
// list = the waypoints whose bit in rm is clear), progress toward that waypoint, cross-track reward
// against the reference path start -> waypoints (reset_world :339-343), small-step and
// near-building penalties; per-agent reward
// waypoint k of an agent: the step kernel's LDS copy of its first WPC waypoints, else HBM (the
// searches below walk the list with a compare after every load: from HBM each step waited for its load)
struct WpView {
    const double2 *lds, *hbm;
    __device__ double2 operator[](int k) const { return k < WPC ? lds[k] : hbm[k]; }
};

// the near-building penalty of WGRU/env ss_reward from the radar minimum (bug-compatible band)
__device__ inline double wgru_nbp(double rmin, double pb) {
    return (rmin >= pb && rmin <= 5) ? 3 * (((0 - 1) / (5 - pb)) * rmin + 2) : 0;
}

// rp, rk: the reward before its penalty term and how the term enters (RewFix)
__device__ __attribute__((always_inline)) double wgru_reward(const Args &A, size_t ai, WpView wp, double2 pp, double2 p, double2 v, uint32_t rm,
                              int cnt, double rmin, int goal, int bnd, int building, int &flag, int &done, int &cg,
                              uint8_t &fl, double2 start, double &rp, int &rk) {
    const double px = p.x, py = p.y, pb = A.pb;
    int nrem = cnt - __popc(rm & (cnt >= 32 ? 0xffffffffu : ((1u << cnt) - 1u)));
    double smallest = INFINITY;
    double2 nx = make_double2(0.0, 0.0);
    const uint32_t rm0 = rm;
    // waypoints in groups of WGB loads in flight: past the first WPC (LDS) they come from HBM, and a
    // wave almost always holds an agent with a longer list
    constexpr int WGB = 2;
    bool found = false;
#pragma unroll 1
    for (int k0 = 0; k0 < cnt && !found; k0 += WGB) {
        double2 wg[WGB];
#pragma unroll
        for (int u = 0; u < WGB; ++u) wg[u] = k0 + u < cnt ? wp[k0 + u] : make_double2(0.0, 0.0);
#pragma unroll
        for (int u = 0; u < WGB; ++u) {
            const int k = k0 + u;
            if (k >= cnt || found) break;
            if ((rm >> k) & 1u) continue;
            const double2 w = wg[u];
            const double d = gdist(px, py, w.x, w.y);
            if (d < smallest) {
                smallest = d;
                nx = w;
                if (smallest < 5) {
                    flag = 1;
                    if (nrem > 1) {
                        rm |= 1u << k;
                        --nrem;
                        double best = INFINITY;
                        for (int q = 0; q < cnt; ++q) {
                            if ((rm >> q) & 1u) continue;
                            const double2 uq = wp[q];
                            const double dd = gdist(uq.x, uq.y, px, py);
                            if (dd < best) {
                                best = dd;
                                nx = uq;
                            }
                        }
                    }
                    found = true;
                }
            }
        }
    }
    if (rm != rm0) {
        A.wp_cur[ai] = (int32_t)rm;
        for (int k = cnt - 1; k >= 0; --k)      // goal[-1] after the pop
            if (!((rm >> k) & 1u)) {
                A.goal[ai] = wp[k];
                break;
            }
    }
    const double dtg = 1 * (npnorm(pp.x - nx.x, pp.y - nx.y) - npnorm(px - nx.x, py - nx.y));
    ASTAMP(6);
    // cross_track_error (WGRU/env:2621-2632): nearest point of the first segment at the smallest
    // pointToSegment distance, then the point distance to it.  A segment whose bounding box lies
    // farther than the current best (squared, 1e-8 relative margin) cannot be strictly nearer: its
    // distance is not computed (the loop keeps the first strict minimum either way)
    double cross;
    {
        double best = INFINITY;
        double2 a = start, q = a;
        bool stop = false;
#pragma unroll 1
        for (int k0 = 0; k0 < cnt && !stop; k0 += WGB) {
            double2 bg[WGB];
#pragma unroll
            for (int u = 0; u < WGB; ++u) bg[u] = k0 + u < cnt ? wp[k0 + u] : make_double2(0.0, 0.0);
#pragma unroll
            for (int u = 0; u < WGB; ++u) {
                if (k0 + u >= cnt || stop) break;
                const double2 b = bg[u];
                {
                    const double ox = fmax(fmax(fmin(a.x, b.x) - px, px - fmax(a.x, b.x)), 0.0);
                    const double oy = fmax(fmax(fmin(a.y, b.y) - py, py - fmax(a.y, b.y)), 0.0);
                    if (ox * ox + oy * oy > best * best * (1.0 + 1e-8)) {
                        a = b;
                        continue;
                    }
                }
                const double d = point_to_segment(px, py, a.x, a.y, b.x, b.y);
                if (d < best) {
                    best = d;
                    q = segment_closest_point(px, py, a.x, a.y, b.x, b.y);
                }
                if (best <= 0.0) {
                    stop = true;
                    break;
                }
                a = b;
            }
        }
        cross = gdist(px, py, q.x, q.y);
    }
    double dref;
    if (cross <= pb) dref = 3 * (((0 - 1) / (pb - 0)) * cross + 1);
    else dref = -3 * 1;
    const double thr = 2 * pb;
    const double sp = npnorm(v.x, v.y);
    const double clip = sp < 0 ? 0 : (sp > thr ? thr : sp);
    const double ssp = 3 * ((thr - clip) * (1.0 / thr));
    const double nbp = wgru_nbp(rmin, pb);
    double r;
    if (bnd) {
        rp = ((((0.0 + dref) - 5) + dtg) - ssp) + 0.0;
        r = rp - nbp;
        rk = 1;
        done = 1;
        fl |= 8;
    } else if (building) {
        done = 1;
        fl |= 16;
        rp = ((((0.0 + dref) - 5) + dtg) - ssp) + 0.0;
        r = rp - nbp;
        rk = 1;
    } else if (goal) {
        cg = 1;
        r = rp = (0.0 + 5) + 0.0;
        rk = 0;
    } else {
        r = 0.0;
        if (flag && nrem > 1) r = r + 3;
        rp = (((r + dref) + dtg) - ssp) + 0.0;
        r = (rp - nbp) + 0.0;
        rk = 2;
    }
    return r;
}


// copy n floats from LDS to global memory with 16-B stores where the destination allows
__device__ inline void store_rows(float *dst, const float *src, int n) {
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const int n4 = n >> 2;
        for (int k = threadIdx.x; k < n4; k += BLOCK)
            reinterpret_cast<float4 *>(dst)[k] = reinterpret_cast<const float4 *>(src)[k];
        for (int k = 4 * n4 + threadIdx.x; k < n; k += BLOCK) dst[k] = src[k];
    } else {
        for (int k = threadIdx.x; k < n; k += BLOCK) dst[k] = src[k];
    }
}

// ---------------------------------------------------------------------- reset / auto-reset
// env slot lq of the workgroup: its entry of the packed list (emap) or the contiguous range
__device__ inline int env_of(const int32_t *emap, int e0, int lq) { return emap ? emap[lq] : e0 + lq; }

// The fused tail's OD draws, made speculatively during the step by the waves that hold no agent
// (they idle through the agent phase): every env of the workgroup draws its next episode's N bank
// entries as reset_body would (the same keys: episode + 1, the same first-valid-attempt rule), so a
// finished env's reset starts at its waypoint copy.  Nothing global is written here: bank indices go
// to S.idx[agent], the starts to spec_starts (the radar-minimum words past the agents; ATT does not
// use them, WGRU only the first nag), episode and map per env to S.idx[nag + env], S.idx[nag + epb
// + env].  Needs nag <= SPEC_MAX_AG (spec_ok).
constexpr int SPEC_MAX_AG = 84;
__device__ inline double2 *spec_starts(Lds &S, int nag) {
    return reinterpret_cast<double2 *>(&S.rmin[(nag + 1) & ~1]);
}
__device__ inline bool spec_ok(const Args &A, const ResetArgs &R) {
    return R.mode == 1 && A.epb * A.N <= SPEC_MAX_AG && !R.list;
}
__device__ __attribute__((always_inline)) void spec_draw(const Args &A, const ResetArgs &R, Lds &S, int e0, int wv, int nw) {
    // 16 lanes per env (four envs per wave at once): the draws of different envs are independent,
    // an env's N draws are a chain of dependent loads; 16 attempts per round (the first attempt
    // almost always succeeds), the lowest valid one wins as in reset_body
    const int N = A.N, nag = A.epb * N, lane = threadIdx.x & 63, gq = lane >> 4, gl = lane & 15;
    double2 *ss = spec_starts(S, nag);
    for (int l0 = 4 * wv; l0 < A.epb; l0 += 4 * nw) {
        const int lq = l0 + gq, eq = e0 + lq;
        const bool live = lq < A.epb && eq < A.E;
        const int ep = live ? R.episode[eq] + 1 : 0;
        const int bq = lq * N;
        int mp = 0, boff = 0, bn = R.bank_n;
        if (R.bank_maps > 1 && live) {
            mp = (int)(mix64(mix64(mix64(R.seed ^ 0x6d61705f64726177ull ^ (uint64_t)eq) ^ (uint64_t)ep)) %
                       (uint64_t)R.bank_maps);
            boff = R.bank_off[mp];
            bn = R.bank_off[mp + 1] - boff;
        }
        const uint64_t ke = mix64(mix64(R.seed ^ (uint64_t)eq) ^ (uint64_t)ep);
        for (int a = 0; a < N; ++a) {
            int chosen = live ? -1 : 0, last = 0, pl = 15;
            double2 sp = make_double2(0.0, 0.0);
            for (int att0 = 0; att0 < 4096; att0 += 16) {
                const bool go = chosen < 0;                  // uniform per 16-lane group
                if (!__ballot(go)) break;
                bool ok = false;
                int idx = 0;
                if (go) {
                    const uint64_t key = mix64(ke ^ ((uint64_t)a * 65536ull + (att0 + gl)));
                    idx = boff + (int)(key % (uint64_t)bn);
                    sp = R.bank_start[idx];
                    ok = true;
                    for (int b = 0; b < a; ++b) {
                        const double2 o = ss[bq + b];
                        if (!(npnorm(sp.x - o.x, sp.y - o.y) > A.pb * 2)) ok = false;
                    }
                }
                const unsigned m = (unsigned)(__ballot(ok) >> (16 * gq)) & 0xffffu;
                const int cidx = __shfl(idx, 16 * gq + (m ? __ffs(m) - 1 : 0), 64);
                const int lidx = __shfl(idx, 16 * gq + 15, 64);
                if (go) {
                    if (m) {
                        pl = __ffs(m) - 1;
                        chosen = cidx;
                    }
                    last = lidx;
                }
            }
            const double spx = __shfl(sp.x, 16 * gq + pl, 64), spy = __shfl(sp.y, 16 * gq + pl, 64);
            if (live && gl == 0) {
                S.idx[bq + a] = chosen >= 0 ? chosen : last;
                ss[bq + a] = make_double2(spx, spy);
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        }
        if (live && gl == 0) {
            S.idx[nag + lq] = ep;
            S.idx[nag + A.epb + lq] = mp;
        }
    }
}

// The reset of the workgroup's envs with S.active[le] set (at least one): OD draw (bank mode) or the
// given OD, waypoint lists, state, radar and observation rows.  Shared by reset_kernel and the fused
// step tail (step_kernel<.., true>), which calls it after its replay push with the maps in LDS.
__device__ __attribute__((always_inline)) void reset_body(const Args &A, const ResetArgs &R, Lds &S, const int32_t *emap,
                                                          int e0, bool maps_loaded, bool predrawn = false) {
    const int N = A.N;
    const int nag = A.epb * N;
    const int t = threadIdx.x;
    const int le = t / N, i = t - le * N;
    const int e = env_of(emap, e0, le < A.epb ? le : 0);
    const bool active = (t < nag) && (e < A.E) && S.active[le];
    const int base = le * N;
    const size_t ai = (size_t)e * N + i;
    if (!maps_loaded) load_maps(A);
    if (predrawn) {
        // the draws were made during the step (spec_draw): bank indices in S.idx, starts in
        // spec_starts, episode / map per env after the indices
        if (t < A.epb && S.active[t] && e0 + t < A.E) {
            R.episode[e0 + t] = S.idx[nag + t];
            if (A.map_idx) A.map_idx[e0 + t] = S.idx[nag + A.epb + t];
        }
    } else if (R.mode == 1) {
        // draw N OD entries; starts pairwise > 2 pB apart (ATT/env:258-268).  One wave per
        // resetting env: the 64 lanes test 64 consecutive attempts of agent a at once and the
        // lowest valid attempt wins, i.e. exactly the sequential rule (first valid attempt, else
        // the last of 4096).
        const int lane = t & 63, wv = t >> 6;
        for (int lq = wv; lq < A.epb; lq += BLOCK / 64) {
            const int eq = env_of(emap, e0, lq);
            if (eq >= A.E || !S.active[lq]) continue;
            const int ep = R.episode[eq] + 1;
            const int bq = lq * N;
            // multipleMap variant: random_map_idx = random.randrange(len(world_map_2D_collection)) per
            // episode (multipleMap/ma_main:464-465), then the OD from that map's bank
            int mp = 0, boff = 0, bn = R.bank_n;
            if (R.bank_maps > 1) {
                mp = (int)(mix64(mix64(mix64(R.seed ^ 0x6d61705f64726177ull ^ (uint64_t)eq) ^ (uint64_t)ep)) %
                           (uint64_t)R.bank_maps);
                boff = R.bank_off[mp];
                bn = R.bank_off[mp + 1] - boff;
            }
            for (int a = 0; a < N; ++a) {
                int chosen = -1, last = 0, pl = 63;
                double2 sp = make_double2(0.0, 0.0);
                for (int att0 = 0; att0 < 4096 && chosen < 0; att0 += 64) {
                    const int att = att0 + lane;
                    const uint64_t key =
                        mix64(mix64(mix64(R.seed ^ (uint64_t)eq) ^ (uint64_t)ep) ^ ((uint64_t)a * 65536ull + att));
                    const int idx = boff + (int)(key % (uint64_t)bn);
                    sp = R.bank_start[idx];
                    bool ok = true;
                    for (int b = 0; b < a; ++b) {
                        const double2 o = S.ppos[bq + b];
                        if (!(npnorm(sp.x - o.x, sp.y - o.y) > A.pb * 2)) ok = false;
                    }
                    const unsigned long long m = __ballot(ok);
                    if (m) {
                        pl = __ffsll((long long)m) - 1;
                        chosen = __shfl(idx, pl, 64);
                    }
                    last = __shfl(idx, 63, 64);
                }
                const int pick = chosen >= 0 ? chosen : last;
                // the chosen start from the lane that loaded it (no second dependent load)
                const double spx = __shfl(sp.x, pl, 64), spy = __shfl(sp.y, pl, 64);
                if (lane == 0) {
                    S.idx[bq + a] = pick;
                    S.ppos[bq + a] = make_double2(spx, spy);      // the chosen starts
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            }
            if (lane == 0) {
                R.episode[eq] = ep;
                if (A.map_idx) A.map_idx[eq] = mp;
            }
        }
    }
    __syncthreads();
    RSTAMP(2, __builtin_amdgcn_s_memtime());
    // the waypoint lists, copied by all threads over (agent, waypoint) items: a thread copying its
    // agent's W waypoints in a row waited for every load before the store that might alias it.  Bank
    // mode: each item also loads its entry's waypoint count (beside the waypoint, no added latency),
    // and the item holding the last waypoint puts the goal and the count in LDS for the state writes
    // (they were two more dependent loads on the resetting workgroup's chain).
    {
        const int nw = nag * A.W;
        for (int w0 = 0; w0 < nw; w0 += 4 * BLOCK) {
            double2 v[4];
            size_t dst[4];
            bool ok[4];
            int cn[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int w = w0 + u * BLOCK + t;
                const int la = w / A.W, k = w - la * A.W, lq = la / N;
                ok[u] = w < nw && S.active[lq < A.epb ? lq : 0] && env_of(emap, e0, lq < A.epb ? lq : 0) < A.E;
                const size_t aq = ok[u] ? (size_t)env_of(emap, e0, lq) * N + (la - lq * N) : 0;
                dst[u] = aq * A.W + k;
                const int bi = (R.mode == 1 && ok[u]) ? S.idx[la] : 0;
                v[u] = !ok[u] ? make_double2(0.0, 0.0)
                              : (R.mode == 1 ? R.bank_wp[(size_t)bi * A.W + k] : R.wps[aq * A.W + k]);
                cn[u] = (R.mode == 1 && ok[u]) ? R.bank_cnt[bi] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int w = w0 + u * BLOCK + t;
                const int la = w / A.W, k = w - la * A.W;
                if (ok[u]) {
                    A.wp[dst[u]] = v[u];
                    if (k == 0) A.wp0[dst[u] / A.W] = v[u];      // the current waypoint (cur = 0)
                }
                if (R.mode == 1 && ok[u] && k == cn[u] - 1) {
                    S.goal[la] = v[u];
                    S.rmin[la] = (unsigned long long)cn[u];
                }
            }
        }
    }
    if (R.mode == 1) __syncthreads();     // goal / count of each drawn entry in LDS
    if (active) {
        double2 st, g;
        int cnt;
        if (R.mode == 1) {
            st = predrawn ? spec_starts(S, nag)[t] : S.ppos[t];        // the chosen start (draw above)
            cnt = (int)S.rmin[t];
            g = S.goal[t];
        } else {
            st = R.start[ai];
            cnt = R.cnt[ai];
            g = R.wps[ai * A.W + cnt - 1];
            if (i == 0 && A.map_idx) A.map_idx[e] = R.map_idx ? R.map_idx[e] : 0;
        }
        A.goal[ai] = g;
        const double2 z = make_double2(0.0, 0.0);
        A.pos[ai] = st;
        A.pre_pos[ai] = st;
        A.start[ai] = st;
        A.vel[ai] = z;
        A.pre_vel[ai] = z;
        A.wp_cnt[ai] = cnt;
        A.wp_cur[ai] = 0;
        A.reach[ai] = 0;
        A.wall[ai] = 0;
        if (i == 0) A.step[e] = 0;
        S.pos[t] = st;
        S.ppos[t] = st;
        S.vel[t] = z;
        S.pvel[t] = z;
        S.goal[t] = g;
    }
    __syncthreads();   // map_idx (explicit or drawn) written above is read by the radar phase below
    RSTAMP(3, __builtin_amdgcn_s_memtime());
    radar_phase(A, S, e0, nag, true, emap, false, RingOut{}, 1);
#ifdef AAC_ENV_STAMPS
    __syncthreads();
#endif
    RSTAMP(4, __builtin_amdgcn_s_memtime());
    if (active) observe_agent(A, S, e, i, base);
#ifdef AAC_ENV_STAMPS
    __syncthreads();
#endif
    RSTAMP(5, __builtin_amdgcn_s_memtime());
    RSTAMP(6, __builtin_amdgcn_s_memrealtime());
}

// Fused step tail, part 1 (aac_env_step_tail): the early fields of the workgroup's nv transitions,
// copied at kernel start.  Their descriptors and a compact-column -> field table go to LDS scratch
// (the observation staging area, free until the observation phase) once per workgroup: looked up per
// element from the kernel arguments, the descriptors were re-read with scalar loads for every element
// (0.042 -> 0.075 ms per step at 4096 x 5).  Thread t owns the compact columns t, t + BLOCK, ...;
// its items are (column, env) pairs with U loads in flight before the stores.
struct TailDesc {
    const void *src;
    int width, shift;      // width | dtype << 30; shift = ring column - compact column
};
static_assert(sizeof(TailDesc) == 16, "one ds_read_b128 per descriptor");

// the column table (descriptors, running column counts, compact column -> field), written by all
// threads at kernel start from the kernel arguments; the caller orders it with a barrier
__device__ __attribute__((always_inline)) void tail_table(const Tail &T, float *table) {
    const int t = threadIdx.x;
    TailDesc *desc = reinterpret_cast<TailDesc *>(table);
    int *cum = reinterpret_cast<int *>(desc + TAIL_MAX_FIELDS);
    uint8_t *lut = reinterpret_cast<uint8_t *>(cum + TAIL_MAX_FIELDS + 1);
    const int ne = T.cum[T.nf];
#pragma unroll
    for (int q = 0; q < TAIL_MAX_FIELDS; ++q)
        if (t == q) {
            desc[q] = TailDesc{T.src[q], T.width[q] | (T.dtype[q] << 30), T.col[q] - T.cum[q]};
            cum[q] = T.cum[q];
        }
    for (int k = t; k < ne; k += BLOCK) {
        int f = 0;
#pragma unroll
        for (int q = 1; q < TAIL_MAX_FIELDS; ++q) f += q < T.nf && k >= T.cum[q];
        lut[k] = (uint8_t)f;
    }
}

// the copy of the early fields by threads tid = 0 .. nthr - 1 (all of the workgroup at kernel start,
// or the waves without agents during the agent phase: T.late_copy)
__device__ __attribute__((always_inline)) void tail_copy(const Tail &T, int64_t rpos, int e0, int nv,
                                                          const float *table, int tid, int nthr) {
    const TailDesc *desc = reinterpret_cast<const TailDesc *>(table);
    const int *cum = reinterpret_cast<const int *>(desc + TAIL_MAX_FIELDS);
    const uint8_t *lut = reinterpret_cast<const uint8_t *>(cum + TAIL_MAX_FIELDS + 1);
    const int ne = T.cum[T.nf];
    const int ncol = tid < ne ? (ne - tid + nthr - 1) / nthr : 0;
    const int items = ncol * nv;
    constexpr int U = 8;
    for (int j0 = 0; j0 < items; j0 += U) {
        float v[U];
        float *dst[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u;
            const bool ok = j < items;
            const int sl = j / nv, r = j - sl * nv;
            const int k = ok ? tid + sl * nthr : 0;
            const int f = lut[k];
            const TailDesc d = desc[f];
            const int w = d.width & 0x3fffffff;
            dst[u] = ok ? ring_row(T, rpos, e0 + r) + k + d.shift : nullptr;
            const size_t si = (size_t)(e0 + r) * w + (k - cum[f]);
            v[u] = !ok ? 0.f
                       : ((d.width >> 30) ? (float)reinterpret_cast<const uint8_t *>(d.src)[si]
                                          : reinterpret_cast<const float *>(d.src)[si]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (dst[u]) *dst[u] = v[u];
    }
}

// --------------------------------------------------------------------------------- step
// Phases: (1) kinematics, one thread per agent; (2) radar, one work item per (agent, ray) over
// all 256 threads; (3) observation + ss_reward predicates, one thread per agent; (4) team reward
// and episode termination, one thread per env.
// One instantiation per (env variant, radar mode): the other variant's reward code and the unused
// radar path are compiled out, which keeps the kernel inside its 128-VGPR budget (the run-time
// branches cost ~66 spilled VGPRs / 240 B of scratch per lane).
// ------------------------------------------------------------------------- exact radar fix-up
// One radar ray decided exactly (the threshold bands resolved: ray_poly_entry_full / ray_square in mode
// 2, whose exact tests are the calls seg_gon_meet / seg_square_meet) from an env's positions and map
// in global memory.  No candidate pre-filter: every other agent's 64-gon gets the full clip, every
// occupied cell of the segment's box the slab test (the same decisions as the filtered radar loop
// outside the bands).
__device__ double radar_ray_exact(const double2 *pos, int N, int i, int r, double pb, double rlen, int mode,
                                  const uint8_t *occ, int gw, int gh, double gx0, double gy0, const double *b) {
    const double2 p = pos[i];
    const double px = p.x, py = p.y;
    const double ex = px + rlen * c_tab.ray_c[r], ey = py + rlen * c_tab.ray_s[r];
    const double len = gdist(ex, ey, px, py);
    bool band = false;
    double dd = len, dob = len;
    if (mode != AAC_RADAR_OBSTACLES) {
        double shortest = INFINITY;
        for (int j = 0; j < N; ++j) {
            if (j == i) continue;
            double t;
            if (!ray_poly_entry_full<1>(px, py, ex, ey, pos[j].x, pos[j].y, pb, t, band, 2)) continue;
            const double d = gdist(px + t * (ex - px), py + t * (ey - py), px, py);
            shortest = d < shortest ? d : shortest;
        }
        if (shortest < INFINITY) dd = shortest;
    }
    if (mode != AAC_RADAR_DRONES) {
        double d;
        int i0 = (int)floor((fmin(px, ex) - 5.0 - gx0) * 0.1), i1 = (int)ceil((fmax(px, ex) + 5.0 - gx0) * 0.1);
        int j0 = (int)floor((fmin(py, ey) - 5.0 - gy0) * 0.1), j1 = (int)ceil((fmax(py, ey) + 5.0 - gy0) * 0.1);
        i0 = i0 < 0 ? 0 : i0;
        j0 = j0 < 0 ? 0 : j0;
        i1 = i1 > gw - 1 ? gw - 1 : i1;
        j1 = j1 > gh - 1 ? gh - 1 : j1;
        for (int ii = i0; ii <= i1; ++ii)
            for (int jj = j0; jj <= j1; ++jj) {
                if (!occ[ii * gh + jj]) continue;
                const double qx = gx0 + 10.0 * ii, qy = gy0 + 10.0 * jj;
                if (ray_square<1>(px, py, ex, ey, qx - 5.0, qx + 5.0, qy - 5.0, qy + 5.0, d, band, 2) && d <= dob) dob = d;
            }
        if (ray_vline(px, py, ex, ey, b[0], d) && d < dob) dob = d;
        if (ray_vline(px, py, ex, ey, b[1], d) && d < dob) dob = d;
        if (ray_hline(px, py, ex, ey, b[2], d) && d < dob) dob = d;
        if (ray_hline(px, py, ex, ey, b[3], d) && d < dob) dob = d;
    }
    return mode == AAC_RADAR_DRONES ? dd : (mode == AAC_RADAR_OBSTACLES ? dob : (dd < dob ? dd : dob));
}

struct FixArgs {
    const BandHdr *hdr;
    const double2 *pos;
    int32_t *cnt;
    int cap, N, mode, gw, gh;
    double pb, rlen, gx0, gy0, bound[4];
    const uint8_t *occ;
    float *radar;
    const uint8_t *env_done;   // non-null: a step entry of an env that was auto-reset in the launch keeps
                               // the reset observation's radar (its ring row is still fixed)
    float *ring;
    int rw, col;
    const RewFix *rfix;        // variant 1 step: rewards whose radar minimum is recomputed exactly
    float *reward;
    int rcol;                  // the ring's reward column (RewFix.row >= 0)
};

// The flagged rays of the launch before it (one workgroup; nothing to do in the common case), then the
// list is emptied for the next launch.  Variant 1: the listed agents' rewards from the exact radar
// minimum (all 18 rays re-run: away from the bands the exact radar is bit-identical to the float one,
// oracle/aac_oracle.c observe_env takes the minimum over all of them).
__device__ __attribute__((always_inline)) void band_fix_body(const FixArgs &F) {
    const int n = *F.cnt;
    const int m = n < F.cap ? n : F.cap;
    for (int k = threadIdx.x; k < m; k += 256) {
        const BandHdr h = F.hdr[k];
        const double d = radar_ray_exact(F.pos + (size_t)k * F.N, F.N, h.i, h.r, F.pb, F.rlen, F.mode,
                                         F.occ + (size_t)h.map * F.gw * F.gh, F.gw, F.gh, F.gx0, F.gy0, F.bound);
        const size_t oi = ((size_t)h.e * F.N + h.i) * NRAY + h.r;
        if (h.kind == 1 || !(F.env_done && F.env_done[h.e])) F.radar[oi] = (float)d;
        if (h.kind == 0 && F.ring && F.col >= 0 && h.row >= 0) F.ring[h.row * F.rw + F.col + h.i * NRAY + h.r] = (float)d;
    }
    const int nr = F.rfix ? F.cnt[2] : 0;
    const int mr = nr < F.cap ? nr : F.cap;
    for (int k = threadIdx.x; k < mr; k += 256) {
        const RewFix x = F.rfix[k];
        double rmin = INFINITY;
        for (int r = 0; r < NRAY; ++r) {      // the obstacle radar: the agent's own position and map only
            const double d = radar_ray_exact(&x.pos, 1, 0, r, F.pb, F.rlen, AAC_RADAR_OBSTACLES,
                                             F.occ + (size_t)x.map * F.gw * F.gh, F.gw, F.gh, F.gx0, F.gy0, F.bound);
            rmin = d < rmin ? d : rmin;
        }
        const double nbp = wgru_nbp(rmin, F.pb);
        const double rew = x.kind == 0 ? x.rp : (x.kind == 1 ? x.rp - nbp : (x.rp - nbp) + 0.0);
        F.reward[(size_t)x.e * F.N + x.i] = (float)rew;
        if (F.ring && x.row >= 0) F.ring[x.row * F.rw + F.rcol + x.i] = (float)rew;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (n) {
            if (n > F.cnt[1]) F.cnt[1] = n;
            F.cnt[0] = 0;
        }
        if (nr) {
            if (nr > F.cnt[3]) F.cnt[3] = nr;
            F.cnt[2] = 0;
        }
    }
}

__global__ void __launch_bounds__(256) band_fix_kernel(FixArgs F) { band_fix_body(F); }

template <int VAR, int RM, bool TAIL>
__global__ void __launch_bounds__(BLOCK, AAC_ENV_MIN_WAVES) step_kernel(Args Ain, const float2 *__restrict__ act,
                                                                         ResetArgs R, Tail T) {
    Args A = Ain;
    A.variant = VAR;
    A.radar_mode = RM;
    __shared__ Lds S;
    const int N = A.N;
    const int nag = A.epb * N;
    const int e0 = blockIdx.x * A.epb;
    // one thread per agent slot, slots packed into the first wave(s): spreading a workgroup's 20-odd
    // agents over its four waves (slot = 4 lane + wave) measured slower, 52 -> 65 us at 4096 x 5
    const int t = threadIdx.x;
    const int le = t / N, i = t - le * N;
    const int e = e0 + le;
    const bool active = (t < nag) && (e < A.E);
    const int base = le * N;
    const size_t ai = (size_t)e * N + i;
    ESTAMP(0, __builtin_amdgcn_s_memrealtime());
    ESTAMP(1, __builtin_amdgcn_s_memtime());
    const int nv = e0 + A.epb <= A.E ? A.epb : A.E - e0;     // envs of this workgroup
    if (TAIL && t < A.epb) S.active[t] = 0;      // env_done of the workgroup's envs (set below)
    RingOut ro{};
    // the kinematics' own state, loaded first: in flight across the push's early copy and the map
    // load (the agent phase's state stays in flight across the radar)
    int cur = 0, wcnt = 0;
    uint8_t reach = 0;
    double2 pp = make_double2(0.0, 0.0), pv = pp, gl = pp, st0 = pp;
    float2 a = make_float2(0.0f, 0.0f);
    if (active) {
        cur = A.wp_cur[ai];
        wcnt = A.wp_cnt[ai];
        reach = A.reach[ai];
        pp = A.pos[ai];
        pv = A.vel[ai];
        a = act[ai];
        gl = A.goal[ai];
        if (VAR) st0 = A.start[ai];       // the cross-track reference start (variant 1)
    }
    // the ring position of this push: the host's mirror, or (graph replays) a device word
    const int64_t rpos = TAIL && T.ring ? (T.pos_in ? *T.pos_in : T.pos) : 0;
    if constexpr (TAIL) {
        if (T.ring) {
            // replay push, early fields (sources of earlier launches); this step's outputs are written
            // into the ring where they are produced (radar phase, staged rows, final phase)
            if (blockIdx.x == 0 && t == 0) {
                if (T.pos_in) {      // device-side position (graph replays): advance it here
                    const int64_t np = rpos + A.E >= T.cap ? rpos + A.E - T.cap : rpos + A.E;
                    const int64_t ns = T.meta[1] + A.E;
                    *T.pos_out = np;
                    T.meta[0] = np;
                    T.meta[1] = ns < T.cap ? ns : T.cap;
                } else {
                    T.meta[0] = T.new_pos;
                    T.meta[1] = T.new_size;
                }
            }
            tail_table(T, S.obs + T.tab_off);
            __syncthreads();
            if (!T.late_copy) tail_copy(T, rpos, e0, nv, S.obs + T.tab_off, t, BLOCK);
            if (T.late[LATE_RADAR] >= 0) ro = RingOut{T.ring, rpos, T.cap, T.rw, T.late[LATE_RADAR]};
        }
    }
    load_maps(A);

    // ---- a1: kinematics (ATT/env:2639-2713)
    double2 np = make_double2(0.0, 0.0), w0 = np;
    if (active) {
        double2 nv;
        double ax = (double)a.x * A.acc_max, ay = (double)a.y * A.acc_max;
        double cvx = pv.x + ax * A.dt, cvy = pv.y + ay * A.dt;
        if (npnorm(cvx, cvy) >= A.vmax) {
            double h = atan2(cvy, cvx);
            nv = make_double2(A.vmax * cos(h), A.vmax * sin(h));
        } else {
            nv = make_double2(cvx, cvy);
        }
        np = make_double2(pp.x + nv.x * A.dt, pp.y + nv.y * A.dt);
        A.pre_pos[ai] = pp;
        A.pre_vel[ai] = pv;
        A.pos[ai] = np;
        A.vel[ai] = nv;
        S.pos[t] = np;
        S.vel[t] = nv;
        S.ppos[t] = pp;
        S.pvel[t] = pv;
        S.goal[t] = gl;
        if (!A.variant) w0 = A.wp0[ai];     // = wp[cur]; variant 1: cur is a bit mask
    }
    if (A.variant) {
        S.rmin[t] = 0x7ff0000000000000ull;       // +inf
        S.flags[t] = 0;                          // bit 7: a ray of this agent is in the band list
    }
    // variant 1: the first WPC waypoints of every agent of the workgroup, loaded now by all threads
    // (one load each, in flight across the radar phase) and put in LDS after it
    constexpr int WPI = 2;           // items per thread held across the radar (nag <= 64); the rest after it
    double2 wpv[WPI];
    const int wpn = A.variant ? nag * (A.W < WPC ? A.W : WPC) : 0;
    if (A.variant) {
#pragma unroll
        for (int u = 0; u < WPI; ++u) {
            const int w = t + u * BLOCK;
            const int kmax = A.W < WPC ? A.W : WPC;
            const int la = w / kmax, k = w - la * kmax;
            const int eq = e0 + la / N;
            wpv[u] = (w < wpn && eq < A.E) ? A.wp[((size_t)eq * N + la % N) * A.W + k] : make_double2(0.0, 0.0);
        }
    }
    aacw::lds_barrier();
    ESTAMP(2, __builtin_amdgcn_s_memtime());
#ifndef AAC_DBG_SKIP_RADAR      // timing experiments only (a round-3 probe script, in the git history)
    radar_phase(A, S, e0, nag, false, nullptr, A.variant != 0, ro);
#endif
    if (A.variant) {
        double2 *wc = wp_cache(A);
        const int kmax = A.W < WPC ? A.W : WPC;
#pragma unroll
        for (int u = 0; u < WPI; ++u) {
            const int w = t + u * BLOCK;
            if (w < wpn) wc[(w / kmax) * WPC + w % kmax] = wpv[u];
        }
        for (int w = t + WPI * BLOCK; w < wpn; w += BLOCK) {
            const int la = w / kmax, k = w - la * kmax, eq = e0 + la / N;
            if (eq < A.E) wc[la * WPC + k] = A.wp[((size_t)eq * N + la % N) * A.W + k];
        }
    }
#ifdef AAC_ENV_STAMPS
    aacw::lds_barrier();
#else
    if (A.variant) aacw::lds_barrier();     // the agent phase reads the radar minima and the waypoint cache
#endif
    ESTAMP(3, __builtin_amdgcn_s_memtime());
    const int D0 = A.D0, K6 = A.K * 6;
    const bool stage = nag * (D0 + K6) <= OBS_STAGE_FLOATS;     // uniform
    bool spec = false;
    if constexpr (TAIL) {
        // the next episodes' OD draws on the waves without agents, beside the agent phase
        const int wfirst = (nag + 63) >> 6;
        spec = T.reset && spec_ok(A, R) && wfirst < BLOCK / 64 && T.spec;
        if (spec && (t >> 6) >= wfirst) spec_draw(A, R, S, e0, (t >> 6) - wfirst, BLOCK / 64 - wfirst);
        // the push's early fields on the waves after those (all agent-free waves when no draw runs; at
        // kernel start when there are none)
        if (T.ring && T.late_copy) {
            const int wc = wfirst + (spec ? 1 : 0) < BLOCK / 64 ? wfirst + (spec ? 1 : 0) : wfirst;
            if (wc < BLOCK / 64 && (t >> 6) >= wc) tail_copy(T, rpos, e0, nv, S.obs + T.tab_off, t - 64 * wc, BLOCK - 64 * wc);
        }
    }
#ifdef AAC_DBG_SKIP_AGENT
    if (false) {
#else
    if (active) {
#endif
        ASTAMP(0);
        const uint8_t *occ = s_maps + (A.map_idx ? A.map_idx[e] : 0) * A.gw * A.gh;
        if (stage) observe_agent(A, S, e, i, base, S.obs + t * D0, S.obs + nag * D0 + t * K6);
        else observe_agent(A, S, e, i, base);
        ASTAMP(1);

        // ---- ss_reward (ATT/env:2133-2603)
        const double px = np.x, py = np.y, pb = A.pb;
        int ncoll = 0, last_coll = -1, nearest = -1;
        double shortest = INFINITY;
        for (int j = 0; j < N; ++j) {
            if (j == i) continue;
            const double2 q = S.pos[base + j];
            double d = npnorm(px - q.x, py - q.y);
            if (d < shortest) {
                shortest = d;
                nearest = j;
            }
            if (d <= pb * 2) {
                ++ncoll;
                last_coll = j;
            }
        }
        const double c_drone = 1 + (2.5 / (10 - 2.5)), m_drone = (0 - 1) / (10 - 2.5);
        double pen = 0;
        for (int j = 0; j < N && !A.variant; ++j) {
            if (j == i) continue;
            const double2 q = S.pos[base + j];
            double d = npnorm(px - q.x, py - q.y);
            if (d >= 2.5 && d <= 10) pen = pen + (1 * (m_drone * shortest + c_drone));
            else pen = pen + 0;
        }
        ASTAMP(2);
        int building = 0;
        {
            int ci = (int)floor((px - A.gx0) / 10.0 + 0.5), cj = (int)floor((py - A.gy0) / 10.0 + 0.5);
            for (int ii = ci - 1; ii <= ci + 1 && !building; ++ii)
                for (int jj = cj - 1; jj <= cj + 1; ++jj) {
                    if (ii < 0 || jj < 0 || ii >= A.gw || jj >= A.gh) continue;
                    if (!occ[ii * A.gh + jj]) continue;
                    if (building_hit<EXACT_COLD(VAR)>(px, py, A.gx0 + 10.0 * ii, A.gy0 + 10.0 * jj, pb)) {
                        building = 1;
                        break;
                    }
                }
        }
        if (building) A.wall[ai] += 1;
        ASTAMP(3);
        const double2 g = S.goal[t];
        const int goal = goal_reached<EXACT_COLD(VAR)>(px, py, g.x, g.y, pb);
        const int bnd = bound_crash(A, pp.x, pp.y, px, py);
        ASTAMP(4);
        int done = 0, cg = 0, wpf = 0;
        uint8_t fl = 0;
        double r;
        if (A.variant) {
            const WpView wv{wp_cache(A) + t * WPC, A.wp + ai * A.W};
            const bool fixr = (S.flags[t] & 0x80) != 0;      // read before the flags are rewritten below
            double rp;
            int rk;
            r = wgru_reward(A, ai, wv, pp, np, S.vel[t], (uint32_t)cur, wcnt,
                            __longlong_as_double((long long)S.rmin[t]), goal, bnd, building, wpf, done, cg, fl, st0,
                            rp, rk);
            if (cg) {
                reach = 1;
                A.reach[ai] = 1;
            }
            if (fixr && A.rfix) {      // a ray of this agent is decided exactly after the launch: so is rmin
                const int slot = atomicAdd(A.band_cnt + 2, 1);
                if (slot < A.band_cap) {
                    int64_t row = -1;
                    if (TAIL && T.ring && T.late[LATE_REW] >= 0) {
                        row = rpos + e;
                        if (row >= T.cap) row -= T.cap;
                    }
                    A.rfix[slot] = RewFix{e, i, A.map_idx ? A.map_idx[e] : 0, rk, rp, np, row};
                }
            }
        } else {
            // ATT/env:2266-2603: next waypoint in range, progress toward goal[-1]
            wpf = gdist(px, py, w0.x, w0.y) < 5;
            const double before = npnorm(pp.x - g.x, pp.y - g.y);
            const double after = npnorm(px - g.x, py - g.y);
            const double dtg = (1 * (before - after)) / A.vmax;
            if (bnd) {
                r = ((0.0 - 20) - 0.0) - 0;
                done = 1;
                fl |= 8;
            } else if (ncoll > 0) {
                r = ((0.0 - 20) - 0.0) - pen;
                done = 1;
                fl |= 16;
                if (last_coll == nearest) fl |= 32;
            } else if (goal) {
                r = (0.0 + 20) + 0.0;
                cg = 1;
                reach = 1;
                A.reach[ai] = 1;
            } else {
                if (wpf && wcnt - cur > 1) {
                    A.wp_cur[ai] = cur + 1;
                    A.wp0[ai] = A.wp[ai * A.W + cur + 1];
                }
                r = dtg - pen;
            }
        }
        uint8_t m = (uint8_t)(bnd | ((ncoll > 0) << 1) | (goal << 2) | (building << 3) | (wpf << 4));
        if (cg) m |= 32;
        fl |= (uint8_t)(done | (cg << 1) | (reach << 2));
        S.rew[t] = r;
        S.flags[t] = fl;
        A.done[ai] = (uint8_t)done;
        A.mask[ai] = m;
        ASTAMP(5);
    }
    aacw::lds_barrier();
    ESTAMP(4, __builtin_amdgcn_s_memtime());
    if (stage) {      // the workgroup's rows are contiguous in own / nei: whole 16-B stores
        store_rows(A.own + (size_t)e0 * N * D0, S.obs, nv * N * D0);
        store_rows(A.nei + (size_t)e0 * N * K6, S.obs + nag * D0, nv * N * K6);
        if constexpr (TAIL) {     // the same rows into the replay ring (next own / nei fields)
            if (T.ring) {
                const int wo = N * D0, wn = N * K6;
                if (T.late[LATE_OWN] >= 0)
                    for (int j = t; j < nv * wo; j += BLOCK) {
                        const int r = j / wo;
                        ring_row(T, rpos, e0 + r)[T.late[LATE_OWN] + (j - r * wo)] = S.obs[j];
                    }
                if (T.late[LATE_NEI] >= 0)
                    for (int j = t; j < nv * wn; j += BLOCK) {
                        const int r = j / wn;
                        ring_row(T, rpos, e0 + r)[T.late[LATE_NEI] + (j - r * wn)] = S.obs[nag * D0 + j];
                    }
            }
        }
    }
    if (active) {
        double team = A.team_reward ? pairwise_sum(&S.rew[base], N) : S.rew[t];
        A.reward[ai] = (float)team;
        if constexpr (TAIL) {
            if (T.ring) {
                float *rr = ring_row(T, rpos, e);
                if (T.late[LATE_REW] >= 0) rr[T.late[LATE_REW] + i] = (float)team;
                if (T.late[LATE_DONE] >= 0) rr[T.late[LATE_DONE] + i] = (float)(S.flags[t] & 1);
            }
        }
        if (i == 0) {
            int any_done = 0, all_goal = 1, all_reach = 1, b0 = 0, b2 = 0, b3 = 0;
            for (int j = 0; j < N; ++j) {
                uint8_t f = S.flags[base + j];
                any_done |= f & 1;
                all_goal &= (f >> 1) & 1;
                all_reach &= (f >> 2) & 1;
                b0 |= (f >> 3) & 1;
                b2 |= (f >> 4) & 1;
                b3 |= (f >> 5) & 1;
            }
            // ATT: [bound, 0, drone, last contact == nearest]; variant 1: bound_building_check
            // [bound, building] (WGRU/env:1956, :1963)
            A.bbc[4 * e + 0] = (uint8_t)b0;
            A.bbc[4 * e + 1] = (uint8_t)(A.variant ? b2 : 0);
            A.bbc[4 * e + 2] = (uint8_t)(A.variant ? 0 : b2);
            A.bbc[4 * e + 3] = (uint8_t)(A.variant ? 0 : b3);
            int st = A.step[e] + 1;
            A.step[e] = st;
            const uint8_t ed = (uint8_t)((A.episode_length < st) || any_done || all_goal || all_reach);
            A.env_done[e] = ed;
            if (TAIL) S.active[le] = ed;
        }
    }
    if constexpr (TAIL) {
        // after the step (whose transitions are in the ring already): zero the given rows of the
        // finished envs and reset them (aac_env_step_tail = step + replay push + row zeroing +
        // auto-reset, in that order)
        __syncthreads();      // env_done flags; the staged rows' ring copies have read S.obs
        int any = 0;
        for (int k = 0; k < A.epb; ++k) any |= S.active[k];
        if (any) {
            if (T.zero_rows) {
                const int n = nv * T.zero_w;
                for (int j = t; j < n; j += BLOCK) {
                    const int r = j / T.zero_w;
                    if (S.active[r]) T.zero_rows[(size_t)e0 * T.zero_w + j] = 0.f;
                }
            }
            if (T.reset) reset_body(A, R, S, nullptr, e0, true, spec);
        }
    }
    ESTAMP(5, __builtin_amdgcn_s_memtime());
    ESTAMP(6, __builtin_amdgcn_s_memrealtime());
}

// wp0 = wp[cur] after the host set wp / wp_cur (aac_env_set_state); cur clamped into the list
__global__ void __launch_bounds__(256) wp0_refresh_kernel(double2 *wp0, const double2 *wp, const int32_t *cur,
                                                          int64_t EN, int W) {
    const int64_t ai = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (ai >= EN) return;
    int c = cur[ai];
    c = c < 0 ? 0 : (c >= W ? W - 1 : c);
    wp0[ai] = wp[ai * W + c];
}

__global__ void __launch_bounds__(BLOCK) reset_kernel(Args A, ResetArgs R) {
    __shared__ Lds S;
    const int N = A.N;
    const int nag = A.epb * N;
    const int e0 = blockIdx.x * A.epb;
    const int t = threadIdx.x;
    // which envs this workgroup resets (contiguous range, or its slots of the packed list of the
    // done envs); skip the whole workgroup if none (the common case)
    __shared__ int32_t emap[BLOCK];
    if (t < A.epb) {
        if (R.list) {
            const int q = e0 + t;
            const bool on = q < R.list[0];
            emap[t] = on ? R.list[1 + q] : 0;
            S.active[t] = on;
        } else {
            const int e = e0 + t;
            emap[t] = e;
            S.active[t] = (e < A.E) && (R.mask == nullptr || R.mask[e] != 0);
        }
    }
    __syncthreads();
    int any = 0;
    for (int k = 0; k < A.epb; ++k) any |= S.active[k];
    if (!any) {
        RSTAMP(1, 0ull);      // stamp builds: mark the workgroup idle in this launch
        return;
    }
    RSTAMP(0, __builtin_amdgcn_s_memrealtime());
    RSTAMP(1, __builtin_amdgcn_s_memtime());
    reset_body(A, R, S, emap, e0, false);
}

// ordered list of the done envs for the packed auto-reset (aacw::compact_flags)
__global__ void __launch_bounds__(1024) env_compact_kernel(const uint8_t *__restrict__ mask, int E, int32_t *rlist) {
    aacw::compact_flags(mask, E, rlist);
}

// ------------------------------------------------------------------------------ host side
thread_local std::string g_err;
// Auto-reset over the packed list of done envs: -1 (default) per variant -- off for the ATT env, where
// few envs end per step at config 3, so the reset is one workgroup's latency either way and the
// packing launch only adds to it (kernel trace: reset 36.4 us -> 37.7 us + 4.8 us packing); on for
// the WGRU variant, where ~38 % of the envs end per step at config 4 and the contiguous ranges keep
// ~1 000 workgroups busy (two rounds) for what fits in one.  AAC_ENV_RESET_PACKED=0 / 1 or
// aac_env_set_reset_compact force it.
int g_env_compact = [] {
    const char *v = getenv("AAC_ENV_RESET_PACKED");
    return v ? (v[0] == '1' ? 1 : 0) : -1;
}();

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                                           \
    do {                                                                                                    \
        hipError_t _e = (x);                                                                                \
        if (_e != hipSuccess) return fail(AAC_E_HIP, std::string(#x) + ": " + hipGetErrorString(_e));      \
    } while (0)

}  // namespace

struct aac_env {
    aac_env_cfg cfg;
    int device;
    int K, D0, W, epb, blocks;
    double2 *pos, *vel, *pre_pos, *pre_vel, *goal, *wp, *start, *wp0;
    int32_t *wp_cur, *wp_cnt, *wall, *step, *map_idx, *episode;
    int32_t *episode_own;     // the handle's own counter buffer (episode may be a caller's buffer)
    uint8_t *reach, *occ;
    unsigned long long *occ_rows;    // row bit masks of occ (grid_h <= 64), else null
    double2 *bank_start, *bank_wp;
    int32_t *bank_cnt, *bank_off;
    int32_t bank_n, bank_maps;
    uint64_t bank_seed;
    int32_t *rlist;           // [1 + E]: packed resetting envs of the last auto-reset
    BandHdr *band_hdr;        // radar threshold-band list (radar_phase, band_fix_kernel)
    double2 *band_pos;
    int32_t *band_cnt;
    RewFix *rfix;             // variant 1: rewards recomputed from the exact radar minimum
};

constexpr int BAND_CAP = 16384;   // flagged rays per launch: never more than a few in practice; the
                                  // threshold tests flag hundreds.  More are counted (aac_env_band_max)

// dynamic LDS of the step / reset kernels: the handle's occupancy maps and their row masks
static size_t map_bytes(const aac_env *h) {
    const size_t b = (size_t)h->cfg.n_maps * h->cfg.grid_w * h->cfg.grid_h;
    return h->occ_rows ? ((b + 7) & ~(size_t)7) + 8 * (size_t)h->cfg.n_maps * h->cfg.grid_w : b;
}

static Args make_args(const aac_env *h, const aac_step_out *o) {
    Args A;
    const aac_env_cfg &c = h->cfg;
    A.E = c.E;
    A.N = c.N;
    A.K = h->K;
    A.D0 = h->D0;
    A.W = h->W;
    A.radar_mode = c.radar_mode;
    A.compat = c.compat;
    A.team_reward = c.team_reward;
    A.episode_length = c.episode_length;
    A.gw = c.grid_w;
    A.gh = c.grid_h;
    A.n_maps = c.n_maps;
    A.epb = h->epb;
    A.variant = c.variant;
    for (int k = 0; k < 4; ++k) A.bound[k] = c.bound[k];
    A.gx0 = std::ceil(c.bound[0] / c.cell) * c.cell;
    A.gy0 = std::ceil(c.bound[2] / c.cell) * c.cell;
    A.xs = (1.0 - (-1.0)) / (c.bound[1] - c.bound[0]);
    A.ys = (1.0 - (-1.0)) / (c.bound[3] - c.bound[2]);
    A.dt = c.dt;
    A.acc_max = c.acc_max;
    A.vmax = c.vmax;
    A.pb = c.pB;
    A.radar_len = c.radar_len;
    A.pos = h->pos;
    A.vel = h->vel;
    A.pre_pos = h->pre_pos;
    A.pre_vel = h->pre_vel;
    A.goal = h->goal;
    A.wp = h->wp;
    A.wp0 = h->wp0;
    A.start = h->start;
    A.wp_cur = h->wp_cur;
    A.wp_cnt = h->wp_cnt;
    A.wall = h->wall;
    A.step = h->step;
    A.map_idx = h->map_idx;
    A.reach = h->reach;
    A.occ = h->occ;
    A.occ_rows = h->occ_rows;
    A.own = o->own;
    A.radar = o->radar;
    A.nei = o->nei;
    A.reward = o->reward;
    A.done = o->done;
    A.mask = o->mask;
    A.env_done = o->env_done;
    A.bbc = o->bbc;
    A.tcpa = o->tcpa;
    A.dcpa = o->dcpa;
    A.conf_cur = o->conf_cur;
    A.conf_pre = o->conf_pre;
    A.band_hdr = h->band_hdr;
    A.band_pos = h->band_pos;
    A.band_cnt = h->band_cnt;
    A.band_cap = BAND_CAP;
    A.rfix = c.variant ? h->rfix : nullptr;
    return A;
}

// band_fix_kernel after a step / reset launch on the same stream (ring: the step tail's ring and its
// late radar column, env_done: skip the radar output of envs the launch reset)
static FixArgs fix_args(const aac_env *h, const Args &A, const uint8_t *env_done = nullptr, float *ring = nullptr,
                        int rw = 0, int col = -1, int rcol = -1) {
    FixArgs F;
    F.hdr = h->band_hdr;
    F.pos = h->band_pos;
    F.cnt = h->band_cnt;
    F.cap = BAND_CAP;
    F.N = A.N;
    F.mode = A.radar_mode;
    F.gw = A.gw;
    F.gh = A.gh;
    F.pb = A.pb;
    F.rlen = A.radar_len;
    F.gx0 = A.gx0;
    F.gy0 = A.gy0;
    for (int k = 0; k < 4; ++k) F.bound[k] = A.bound[k];
    F.occ = A.occ;
    F.radar = A.radar;
    F.env_done = env_done;
    F.ring = col >= 0 || rcol >= 0 ? ring : nullptr;
    F.rw = rw;
    F.col = col;
    F.rfix = A.rfix;
    F.reward = A.reward;
    F.rcol = rcol;
    return F;
}

static void launch_band_fix(const aac_env *h, const Args &A, hipStream_t st, const uint8_t *env_done = nullptr,
                            float *ring = nullptr, int rw = 0, int col = -1, int rcol = -1) {
    hipLaunchKernelGGL(band_fix_kernel, dim3(1), dim3(256), 0, st, fix_args(h, A, env_done, ring, rw, col, rcol));
}

static ResetArgs bank_reset_args(const aac_env *h) {
    ResetArgs R{};
    R.mode = 1;
    R.bank_start = h->bank_start;
    R.bank_wp = h->bank_wp;
    R.bank_cnt = h->bank_cnt;
    R.bank_n = h->bank_n;
    R.bank_off = h->bank_off;
    R.bank_maps = h->bank_maps;
    R.seed = h->bank_seed;
    R.episode = h->episode;
    return R;
}

extern "C" {

const char *aac_last_error(void) { return g_err.c_str(); }

int aac_env_create(const aac_env_cfg *cfg, int device, aac_env **out) {
    if (!cfg || !out) return fail(AAC_E_INVALID, "null argument");
    const aac_env_cfg &c = *cfg;
    if (c.E <= 0 || c.N < 2 || c.N > BLOCK) return fail(AAC_E_INVALID, "need E > 0 and 2 <= N <= 256");
    if (c.R != NRAY) return fail(AAC_E_INVALID, "R must be 18 (range(0, 360, 20))");
    if (c.radar_mode < 0 || c.radar_mode > 2) return fail(AAC_E_INVALID, "bad radar_mode");
    if (c.max_wp < 1) return fail(AAC_E_INVALID, "max_wp must be >= 1");
    if (c.n_maps < 1 || !c.occ || c.grid_w < 1 || c.grid_h < 1) return fail(AAC_E_INVALID, "bad occupancy maps");
    if ((size_t)c.n_maps * c.grid_w * (c.grid_h + 8) + 8 > MAX_MAP_BYTES)
        return fail(AAC_E_INVALID, "maps exceed LDS budget");
    if (c.cell != 10.0) return fail(AAC_E_INVALID, "cell must be 10 m (grid geometry of ATT/grid:138)");
    if (c.variant < 0 || c.variant > 1) return fail(AAC_E_INVALID, "variant: 0 one_model_att, 1 randomOD_Wgru_radar");
    if (c.variant == 1 && (c.radar_mode != AAC_RADAR_OBSTACLES || c.team_reward || c.max_wp > 32))
        return fail(AAC_E_INVALID, "variant 1 (WGRU): obstacle radar, per-agent reward, max_wp <= 32");
    HIPCHK(hipSetDevice(device));
    aac_env *h = new aac_env();
    std::memset(h, 0, sizeof(*h));
    h->cfg = c;
    h->cfg.occ = nullptr;
    h->device = device;
    h->K = c.N - 1;
    h->D0 = c.variant ? 6 : 6 + 4 * h->K;
    h->W = c.max_wp;
    // agents per 256-thread workgroup: ~24 (x 18 rays of radar work) while that leaves fewer than
    // 1024 workgroups (4 per CU, all resident: 46 vs 51-58 us per step at 4096 x 5 for 35 / 50 / 15
    // agents); ~50 once the grid stays >= 1024 workgroups with them (262 144 x 5: 1.66 -> 1.16 ms).
    // AAC_ENV_AGENTS_PER_WG forces a value (tuning).
    static const int apw_env = [] {
        const char *v = getenv("AAC_ENV_AGENTS_PER_WG");
        const int k = v ? atoi(v) : 0;
        return k < 0 ? 0 : (k > BLOCK ? BLOCK : k);
    }();
    auto epb_for = [&](int apw) { return c.N > apw ? 1 : apw / c.N; };
    if (apw_env) {
        h->epb = epb_for(apw_env);
    } else if (c.E / epb_for(50) >= 1024) {
        h->epb = epb_for(50);
    } else {
        // ~24 agents per workgroup, raised (up to ~50) until the grid fits one round of 1024
        // workgroups: at 4096 x 8 (config 4) 3 envs per workgroup made 1366 workgroups, two rounds;
        // 4 envs: 0.070 -> 0.055 ms per step launch
        h->epb = epb_for(24);
        while (h->epb < epb_for(50) && (c.E + h->epb - 1) / h->epb > 1024) ++h->epb;
    }
    h->blocks = (c.E + h->epb - 1) / h->epb;
    const size_t EN = (size_t)c.E * c.N;
    hipError_t st = hipSuccess;
#define ALLOC(p, n)                                                       \
    if (st == hipSuccess) st = hipMalloc((void **)&h->p, (n) * sizeof(*h->p)); \
    if (st == hipSuccess) st = hipMemset(h->p, 0, (n) * sizeof(*h->p));
    ALLOC(pos, EN) ALLOC(vel, EN) ALLOC(pre_pos, EN) ALLOC(pre_vel, EN) ALLOC(goal, EN) ALLOC(start, EN)
    ALLOC(wp, EN * h->W) ALLOC(wp0, EN) ALLOC(wp_cur, EN) ALLOC(wp_cnt, EN) ALLOC(wall, EN) ALLOC(reach, EN)
    ALLOC(step, (size_t)c.E) ALLOC(map_idx, (size_t)c.E) ALLOC(episode, (size_t)c.E)
    ALLOC(rlist, (size_t)c.E + 1)
    ALLOC(band_hdr, (size_t)BAND_CAP) ALLOC(band_pos, (size_t)BAND_CAP * c.N) ALLOC(band_cnt, 4) ALLOC(rfix, (size_t)BAND_CAP)
    h->episode_own = h->episode;
    ALLOC(occ, (size_t)c.n_maps * c.grid_w * c.grid_h)
#undef ALLOC
    if (st == hipSuccess) st = hipMemcpy(h->occ, c.occ, (size_t)c.n_maps * c.grid_w * c.grid_h, hipMemcpyHostToDevice);
    if (st == hipSuccess && c.grid_h <= 64) {      // row masks for the radar's cell enumeration
        std::vector<unsigned long long> rows((size_t)c.n_maps * c.grid_w, 0ull);
        for (size_t r = 0; r < rows.size(); ++r)
            for (int j = 0; j < c.grid_h; ++j)
                if (c.occ[r * c.grid_h + j]) rows[r] |= 1ull << j;
        st = hipMalloc((void **)&h->occ_rows, rows.size() * sizeof(unsigned long long));
        if (st == hipSuccess)
            st = hipMemcpy(h->occ_rows, rows.data(), rows.size() * sizeof(unsigned long long), hipMemcpyHostToDevice);
    }
    if (st == hipSuccess) {
        Tab t;
        fill_tables(t);
        st = hipMemcpyToSymbol(HIP_SYMBOL(c_tab), &t, sizeof(Tab));
    }
    if (st != hipSuccess) {
        aac_env_destroy(h);
        return fail(AAC_E_HIP, std::string("aac_env_create: ") + hipGetErrorString(st));
    }
    *out = h;
    return AAC_OK;
}

void aac_env_destroy(aac_env *h) {
    if (!h) return;
    void *ptrs[] = {h->pos, h->vel, h->pre_pos, h->pre_vel, h->goal, h->start, h->wp, h->wp0, h->wp_cur, h->wp_cnt, h->wall,
                    h->reach, h->step, h->map_idx, h->episode_own, h->occ, h->bank_start, h->bank_wp, h->bank_cnt,
                    h->bank_off, h->rlist, h->occ_rows, h->band_hdr, h->band_pos, h->band_cnt, h->rfix};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete h;
}

static int check_out(const aac_step_out *o) {
    if (!o || !o->own || !o->radar || !o->nei) return fail(AAC_E_INVALID, "observation outputs required");
    if ((o->tcpa == nullptr) != (o->dcpa == nullptr)) return fail(AAC_E_INVALID, "tcpa/dcpa must be both set");
    if ((o->conf_cur == nullptr) != (o->conf_pre == nullptr)) return fail(AAC_E_INVALID, "conf_cur/pre both");
    return AAC_OK;
}

static int launch_step(aac_env *h, const float *actions, const aac_step_out *o, const ResetArgs &R, const Tail &T,
                       bool tail, void *stream) {
    if (!h || !actions) return fail(AAC_E_INVALID, "null argument");
    int rc = check_out(o);
    if (rc) return rc;
    if (!o->reward || !o->done || !o->mask || !o->env_done || !o->bbc) return fail(AAC_E_INVALID, "step outputs");
    Args A = make_args(h, o);
    const dim3 grid(h->blocks), block(BLOCK);
    size_t lds = map_bytes(h);
    if (A.variant) lds = ((lds + 15) & ~(size_t)15) + sizeof(double2) * WPC * (size_t)h->epb * h->cfg.N;
    const hipStream_t st = (hipStream_t)stream;
    const float2 *a2 = reinterpret_cast<const float2 *>(actions);
    FixArgs F = tail ? fix_args(h, A, T.reset ? o->env_done : nullptr, T.ring, T.rw, T.late[LATE_RADAR], T.late[LATE_REW])
                     : fix_args(h, A);
#define STEP_LAUNCH(V, M)                                                                                        \
    do {                                                                                                         \
        if (tail) hipLaunchKernelGGL((step_kernel<V, M, true>), grid, block, lds, st, A, a2, R, T);              \
        else hipLaunchKernelGGL((step_kernel<V, M, false>), grid, block, lds, st, A, a2, R, T);                  \
    } while (0)
    if (A.variant) STEP_LAUNCH(1, AAC_RADAR_OBSTACLES);
    else if (A.radar_mode == AAC_RADAR_DRONES) STEP_LAUNCH(0, AAC_RADAR_DRONES);
    else if (A.radar_mode == AAC_RADAR_OBSTACLES) STEP_LAUNCH(0, AAC_RADAR_OBSTACLES);
    else STEP_LAUNCH(0, AAC_RADAR_COMBINED);
#undef STEP_LAUNCH
    hipLaunchKernelGGL(band_fix_kernel, dim3(1), dim3(256), 0, st, F);
    HIPCHK(hipGetLastError());
    return AAC_OK;
}

int aac_env_step(aac_env *h, const float *actions, const aac_step_out *o, void *stream) {
    return launch_step(h, actions, o, ResetArgs{}, Tail{}, false, stream);
}

int aac_env_step_tail(aac_env *h, const float *actions, const aac_step_out *o, const aac_step_tail *t,
                      void *stream) {
    if (!h || !t) return fail(AAC_E_INVALID, "null argument");
    Tail T{};
    ResetArgs R{};
    if (t->ring) {
        const int n = t->n_fields;
        if (n < 1 || n > TAIL_MAX_FIELDS || !t->srcs || !t->widths) return fail(AAC_E_INVALID, "step tail: 1..12 push fields");
        if (t->capacity < h->cfg.E || t->row_width < 1 || !t->meta)
            return fail(AAC_E_INVALID, "step tail: need E <= capacity, row_width >= 1 and meta");
        if (t->pos < 0 || t->pos >= t->capacity || t->size < 0 || t->size > t->capacity)
            return fail(AAC_E_INVALID, "step tail: need 0 <= pos < capacity, size <= capacity");
        if (!o) return fail(AAC_E_INVALID, "null argument");
        T.ring = t->ring;
        T.rw = t->row_width;
        T.cap = t->capacity;
        T.pos = t->pos;
        T.meta = t->meta;
        if ((t->pos_in == nullptr) != (t->pos_out == nullptr) || (t->pos_in && t->pos_in == t->pos_out))
            return fail(AAC_E_INVALID, "step tail: pos_in and pos_out both set (two distinct words) or both NULL");
        T.pos_in = t->pos_in;
        T.pos_out = t->pos_out;
        T.new_pos = (t->pos + h->cfg.E) % t->capacity;
        T.new_size = std::min<int64_t>(t->size + h->cfg.E, t->capacity);
        for (int k = 0; k < LATE_N; ++k) T.late[k] = -1;
        // a field whose source is one of this step's outputs is written where the step computes it
        const int N = h->cfg.N, K = h->K;
        const void *outs[LATE_N] = {o->own, o->radar, o->nei, o->reward, o->done};
        const int ow[LATE_N] = {N * h->D0, N * NRAY, N * K * 6, N, N};
        const int odt[LATE_N] = {0, 0, 0, 0, 1};
        int col = 0, ne = 0;
        T.cum[0] = 0;
        for (int f = 0; f < n; ++f) {
            const int w = t->widths[f], dt = t->dtypes ? t->dtypes[f] : 0;
            if (!t->srcs[f] || w < 1) return fail(AAC_E_INVALID, "step tail: null source or width < 1");
            if (dt != 0 && dt != 1) return fail(AAC_E_INVALID, "step tail: dtype 0 (f32) or 1 (u8)");
            int role = -1;
            for (int k = 0; k < LATE_N; ++k)
                if (t->srcs[f] == outs[k]) role = k;
            if (role >= 0) {
                if (w != ow[role] || dt != odt[role] || T.late[role] >= 0)
                    return fail(AAC_E_INVALID, "step tail: a step-output field must have its output's width and dtype");
                T.late[role] = col;
            } else {
                T.src[T.nf] = t->srcs[f];
                T.width[T.nf] = w;
                T.dtype[T.nf] = dt;
                T.col[T.nf] = col;
                ne += w;
                T.cum[++T.nf] = ne;
            }
            col += w;
        }
        if (col > T.rw) return fail(AAC_E_INVALID, "step tail: field widths exceed row_width (the ring's row stride)");
        for (int q = T.nf; q < TAIL_MAX_FIELDS; ++q) {     // unused descriptor slots: harmless values
            T.src[q] = t->srcs[0];
            T.width[q] = 1;
            T.dtype[q] = 0;
            T.col[q] = 0;
            T.cum[q + 1] = ne;
        }
        const size_t tab = sizeof(TailDesc) * TAIL_MAX_FIELDS + sizeof(int) * (TAIL_MAX_FIELDS + 1) + ne;
        if (tab > sizeof(float) * OBS_STAGE_FLOATS)
            return fail(AAC_E_INVALID, "step tail: too many early columns for the column table");
        // the table at the end of the staging area; the early copy moves into the agent phase when the
        // staged observation rows leave it alone and some wave holds no agent
        T.tab_off = (int)((sizeof(float) * OBS_STAGE_FLOATS - tab) / sizeof(float)) & ~3;
        const int nag = h->epb * N, stage = nag * (h->D0 + 6 * K);
        const int staged = stage <= OBS_STAGE_FLOATS ? stage : 0;
        static const int late_env = [] {
            const char *v = getenv("AAC_ENV_LATE_COPY");
            return v ? atoi(v) : 1;
        }();
        T.late_copy = late_env && staged <= T.tab_off && (nag + 63) / 64 < BLOCK / 64;
        if ((T.late[LATE_OWN] >= 0 || T.late[LATE_NEI] >= 0) &&
            h->epb * h->cfg.N * (h->D0 + 6 * K) > OBS_STAGE_FLOATS)
            return fail(AAC_E_INVALID, "step tail: observation rows too wide to push from the staging area");
    }
    if (t->zero_rows) {
        if (t->zero_width < 1) return fail(AAC_E_INVALID, "step tail: zero_width >= 1");
        T.zero_rows = t->zero_rows;
        T.zero_w = t->zero_width;
    }
    if (t->auto_reset) {
        if (!h->bank_n) return fail(AAC_E_STATE, "no OD bank installed (aac_env_set_od_bank)");
        R = bank_reset_args(h);
        T.reset = 1;
        // AAC_ENV_SPEC_DRAW=0: draw after the step, as reset_kernel does (A/B switch; same results)
        static const int spec = [] {
            const char *v = getenv("AAC_ENV_SPEC_DRAW");
            return v ? atoi(v) : 1;
        }();
        T.spec = spec;
    }
    return launch_step(h, actions, o, R, T, true, stream);
}

int aac_env_reset(aac_env *h, const uint8_t *mask, const double *start, const double *wps, const int32_t *cnt,
                  const int32_t *map_idx, const aac_step_out *o, void *stream) {
    if (!h || !start || !wps || !cnt) return fail(AAC_E_INVALID, "null argument");
    int rc = check_out(o);
    if (rc) return rc;
    Args A = make_args(h, o);
    ResetArgs R{};
    R.mode = 0;
    R.mask = mask;
    R.start = reinterpret_cast<const double2 *>(start);
    R.wps = reinterpret_cast<const double2 *>(wps);
    R.cnt = cnt;
    R.map_idx = map_idx;
    R.episode = h->episode;
    hipLaunchKernelGGL(reset_kernel, dim3(h->blocks), dim3(BLOCK), map_bytes(h), (hipStream_t)stream, A, R);
    launch_band_fix(h, A, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return AAC_OK;
}

int aac_env_set_od_banks(aac_env *h, int32_t n_maps, const double *start, const double *wps, const int32_t *cnt,
                         const int32_t *n_per_map, uint64_t seed) {
    if (!h || !start || !wps || !cnt || !n_per_map || n_maps < 1) return fail(AAC_E_INVALID, "bad OD banks");
    if (n_maps != h->cfg.n_maps) return fail(AAC_E_INVALID, "one OD bank per map (n_maps of the handle)");
    std::vector<int32_t> off(n_maps + 1, 0);
    for (int m = 0; m < n_maps; ++m) {
        if (n_per_map[m] <= 0) return fail(AAC_E_INVALID, "empty OD bank");
        off[m + 1] = off[m] + n_per_map[m];
    }
    const int32_t n = off[n_maps];
    for (int32_t k = 0; k < n; ++k)
        if (cnt[k] < 1 || cnt[k] > h->W) return fail(AAC_E_INVALID, "OD bank waypoint count out of [1, W]");
    HIPCHK(hipSetDevice(h->device));
    if (h->bank_start) {
        (void)hipFree(h->bank_start); (void)hipFree(h->bank_wp); (void)hipFree(h->bank_cnt); (void)hipFree(h->bank_off);
    }
    h->bank_start = nullptr; h->bank_wp = nullptr; h->bank_cnt = nullptr; h->bank_off = nullptr;
    HIPCHK(hipMalloc((void **)&h->bank_start, sizeof(double2) * n));
    HIPCHK(hipMalloc((void **)&h->bank_wp, sizeof(double2) * (size_t)n * h->W));
    HIPCHK(hipMalloc((void **)&h->bank_cnt, sizeof(int32_t) * n));
    HIPCHK(hipMalloc((void **)&h->bank_off, sizeof(int32_t) * (n_maps + 1)));
    HIPCHK(hipMemcpy(h->bank_start, start, sizeof(double2) * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->bank_wp, wps, sizeof(double2) * (size_t)n * h->W, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->bank_cnt, cnt, sizeof(int32_t) * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->bank_off, off.data(), sizeof(int32_t) * (n_maps + 1), hipMemcpyHostToDevice));
    h->bank_n = n;
    h->bank_maps = n_maps;
    h->bank_seed = seed;
    return AAC_OK;
}

int aac_env_set_od_bank(aac_env *h, const double *start, const double *wps, const int32_t *cnt, int32_t n,
                        uint64_t seed) {
    if (!h || !start || !wps || !cnt || n <= 0) return fail(AAC_E_INVALID, "bad OD bank");
    if (h->cfg.n_maps != 1) return fail(AAC_E_INVALID, "n_maps > 1: install one OD bank per map (aac_env_set_od_banks)");
    return aac_env_set_od_banks(h, 1, start, wps, cnt, &n, seed);
}

int aac_env_auto_reset(aac_env *h, const uint8_t *env_done, const aac_step_out *o, void *stream) {
    if (!h) return fail(AAC_E_INVALID, "null handle");
    if (!h->bank_n) return fail(AAC_E_STATE, "no OD bank installed (aac_env_set_od_bank)");
    int rc = check_out(o);
    if (rc) return rc;
    Args A = make_args(h, o);
    ResetArgs R = bank_reset_args(h);
    R.mask = env_done;
    const bool packed = g_env_compact < 0 ? h->cfg.variant != 0 : g_env_compact != 0;
    if (env_done && packed) {
        hipLaunchKernelGGL(env_compact_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, env_done, h->cfg.E,
                           h->rlist);
        HIPCHK(hipGetLastError());
        R.list = h->rlist;
    }
    hipLaunchKernelGGL(reset_kernel, dim3(h->blocks), dim3(BLOCK), map_bytes(h), (hipStream_t)stream, A, R);
    launch_band_fix(h, A, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return AAC_OK;
}

void aac_env_set_reset_compact(int32_t on) { g_env_compact = on < 0 ? -1 : (on != 0); }

int aac_env_stamps(unsigned long long *out, int32_t n_wg) {
#ifdef AAC_ENV_STAMPS
    const size_t n = sizeof(unsigned long long) * 7 * (size_t)std::min(n_wg, ESTAMP_WG);
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_env_st), n));
    return AAC_OK;
#else
    (void)out;
    (void)n_wg;
    return fail(AAC_E_STATE, "built without AAC_ENV_STAMPS");
#endif
}

int aac_env_reset_stamps(unsigned long long *out, int32_t n_wg) {
#ifdef AAC_ENV_STAMPS
    const size_t n = sizeof(unsigned long long) * 7 * (size_t)std::min(n_wg, ESTAMP_WG);
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_reset_st), n));
    return AAC_OK;
#else
    (void)out;
    (void)n_wg;
    return fail(AAC_E_STATE, "built without AAC_ENV_STAMPS");
#endif
}

int aac_env_band_max(aac_env *h, int32_t *out, int32_t *cap, void *stream) {
    if (!h || !out) return fail(AAC_E_INVALID, "null argument");
    int32_t c[4];
    HIPCHK(hipMemcpyAsync(c, h->band_cnt, sizeof(c), hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    *out = c[1] > c[3] ? c[1] : c[3];     // flagged rays, or (variant 1) rewards to recompute
    if (cap) *cap = BAND_CAP;
    return AAC_OK;
}

int aac_env_use_episode_buffer(aac_env *h, int32_t *episode_dev, void *stream) {
    if (!h || !episode_dev) return fail(AAC_E_INVALID, "null argument");
    HIPCHK(hipSetDevice(h->device));
    // on the caller's stream: ordered after its pending auto-resets and its fill of episode_dev
    if (episode_dev != h->episode)
        HIPCHK(hipMemcpyAsync(episode_dev, h->episode, sizeof(int32_t) * (size_t)h->cfg.E, hipMemcpyDeviceToDevice,
                              (hipStream_t)stream));
    h->episode = episode_dev;
    return AAC_OK;
}

#define CPY(dst, src, n)                                                                                  \
    if (dst && src) HIPCHK(hipMemcpyAsync((void *)(dst), (const void *)(src), (n), hipMemcpyDeviceToDevice, \
                                          (hipStream_t)stream));

int aac_env_get_state(aac_env *h, double *pos, double *vel, double *pre_pos, double *pre_vel, double *goal, double *wp,
                      int32_t *wp_cur, int32_t *wp_cnt, uint8_t *reach, int32_t *wall, int32_t *step,
                      int32_t *map_idx, double *start, void *stream) {
    if (!h) return fail(AAC_E_INVALID, "null handle");
    const size_t EN = (size_t)h->cfg.E * h->cfg.N, E = h->cfg.E;
    CPY(start, h->start, EN * 16)
    CPY(pos, h->pos, EN * 16) CPY(vel, h->vel, EN * 16) CPY(pre_pos, h->pre_pos, EN * 16)
    CPY(pre_vel, h->pre_vel, EN * 16) CPY(goal, h->goal, EN * 16) CPY(wp, h->wp, EN * h->W * 16)
    CPY(wp_cur, h->wp_cur, EN * 4) CPY(wp_cnt, h->wp_cnt, EN * 4) CPY(reach, h->reach, EN)
    CPY(wall, h->wall, EN * 4) CPY(step, h->step, E * 4) CPY(map_idx, h->map_idx, E * 4)
    return AAC_OK;
}

int aac_env_set_state(aac_env *h, const double *pos, const double *vel, const double *pre_pos, const double *pre_vel,
                      const double *goal, const double *wp, const int32_t *wp_cur, const int32_t *wp_cnt,
                      const uint8_t *reach, const int32_t *wall, const int32_t *step, const int32_t *map_idx,
                      const double *start, void *stream) {
    if (!h) return fail(AAC_E_INVALID, "null handle");
    const size_t EN = (size_t)h->cfg.E * h->cfg.N, E = h->cfg.E;
    CPY(h->start, start, EN * 16)
    CPY(h->pos, pos, EN * 16) CPY(h->vel, vel, EN * 16) CPY(h->pre_pos, pre_pos, EN * 16)
    CPY(h->pre_vel, pre_vel, EN * 16) CPY(h->goal, goal, EN * 16) CPY(h->wp, wp, EN * h->W * 16)
    CPY(h->wp_cur, wp_cur, EN * 4) CPY(h->wp_cnt, wp_cnt, EN * 4) CPY(h->reach, reach, EN)
    CPY(h->wall, wall, EN * 4) CPY(h->step, step, E * 4) CPY(h->map_idx, map_idx, E * 4)
    if (wp || wp_cur) {      // the compact current-waypoint copy follows wp / wp_cur
        hipLaunchKernelGGL(wp0_refresh_kernel, dim3((unsigned)((EN + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           h->wp0, h->wp, h->wp_cur, (int64_t)EN, h->W);
        HIPCHK(hipGetLastError());
    }
    return AAC_OK;
}
#undef CPY

}  // extern "C"
