// aac_uam.hip -- gfx950 kernels + C ABI of the UAM environment.
//
// Reference: UAM/env:551-771 reset_world_change_skin, :4667-4904 step, :1294-1919
// cur_state_norm_state_v3, :3892-4629 ss_reward_Mar_changeskin; UAM/util:41-51, :165-334;
// UAM/main:624-637 termination (UAM/ = MADDPG_ownENV_randomOD_radar_N_model_use_tdCPA_forV2_changeskin_UAM).
//
// A 256-thread workgroup owns floor(64 / N) whole envs (<= 64 aircraft).  Everything an aircraft
// interacts with -- the other aircraft of its env, the env's drifting cloud and go-around
// aircraft, the runway and the bound -- is in LDS or constant memory, so there is no
// inter-workgroup traffic.  Phases: (0) clouds, one thread per (env, cloud); (1) kinematics, one
// thread per aircraft; (2) neighbour order by distance rank; (3) radar, one work item per
// (aircraft, ray); (4) observation + goal touch; (5) ss_reward predicates per aircraft; (6) the
// per-env pass that applies the reward's order-dependent coefficient doubling, done flags and
// termination.  State is SoA double2 in HBM; this is fp64 branchy geometry, no MFMA.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <algorithm>
#include <vector>

#include "../../include/aac_uam.h"
#include "aac_geom.h"
#include "aac_wave.h"

#define BLOCK 256
#define MAXA 64   // aircraft per workgroup
#define KMAX (MAXA - 1)
#define NONE8 255
#define CLIP_CAP 2048   // radar clip jobs per workgroup in LDS (8 KB: four workgroups per CU still fit)

#ifndef AAC_UAM_MIN_WAVES     // waves per SIMD the step kernel is compiled for: 4 (<= 128 VGPRs) instead
#define AAC_UAM_MIN_WAVES 4   // of the 130-VGPR / 3-wave build
#endif

namespace {

// ------------------------------------------------------------------------ UAM world constants
struct World {
    double cloud_start[2][2], cloud_goal[2][2];   // cloud_a / cloud_b (UAM/env:567-568)
    double path[4][6][2];                          // go_0..go_3 (UAM/env:562-565)
    int path_first[4][6];                          // cloud_path.index(path[t]): first equal point
    double radius[2], vel[2];                      // cloud / go-around aircraft (UAM/cloud.py)
    double runway[4];                              // x0, x1, y0, y1 (UAM/env:559)
};
__constant__ World c_world;

struct UArgs {
    int E, N, K, epb, episode_length;
    double dt, acc_max, vmax, pb, radar_len;
    double bound[4];
    double2 *pos, *vel, *pre_pos, *pre_vel, *goal, *start, *clouds;
    double *heading;
    uint8_t *reach, *top2;
    int32_t *cloud_kind, *cloud_tgt, *step, *episode;
    double *own, *radar, *nei, *nei6, *reward, *tcpa, *dcpa;
    int32_t *conf_cur, *conf_pre;
    uint8_t *done, *mask, *env_done, *bbc;
};

struct UReset {
    int mode;                 // 0 explicit, 1 bank
    const uint8_t *mask;      // env mask (explicit) or env_done (bank); NULL = all
    const double2 *start, *goal;
    const int32_t *clouds;    // [E][2] explicit or [n][2] bank
    int32_t bank_n;
    uint64_t seed;
    const int32_t *list;      // [count, env...] of the resetting envs (uam_compact_kernel); NULL:
                              // workgroup b takes envs b*epb ... (mask-filtered)
};

#ifdef AAC_UAM_STAMPS
// phase timestamps of the first 64 workgroups of uam_step_kernel (probe builds only)
__device__ unsigned long long g_uam_st[64][16];
#define USTAMP(i)                                                                                     \
    do {                                                                                               \
        if (blockIdx.x < 64 && threadIdx.x == 0) g_uam_st[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define USTAMP(i) \
    do {          \
    } while (0)
#endif

struct Lds {
    double2 pos[MAXA], vel[MAXA], ppos[MAXA], pvel[MAXA], goal[MAXA];
    double heading[MAXA];
    double rad[MAXA][NRAY];
    double2 cl[MAXA][2];                  // per local env: cloud centres after this step
    uint8_t order[MAXA][KMAX];            // neighbours sorted by distance (local indices)
    uint8_t reach[MAXA];
    uint8_t active[MAXA];                 // per local env
    // ss_reward scratch per aircraft
    uint8_t kind[MAXA];                   // 0 bound, 1 cloud, 2 drone, 3 goal, 4 normal
    uint8_t flag[MAXA];                   // bit0 near-drone in band, bit1 its bearing doubles the
                                          // coefficient, bit2 collision bearing doubles the crash
                                          // penalty, bit3 previous-nearest-two collided
    double nd_val[MAXA], base[MAXA];      // m d + c of the near-drone band; dist_to_goal - near_building
    int ccnt[MAXA], pcnt[MAXA];           // tdCPA potential-conflict counts (current, previous state)
    unsigned nclip;                       // radar work list: (ray, polygon) clip jobs (radar_phase)
    uint32_t clip[CLIP_CAP];
};

__device__ inline double nmlz(double v, double lo, double hi) { return 2 * ((v - lo) / (hi - lo)) - 1; }

__device__ inline double bearing(double xh, double yh, double xi, double yi) {
    // calculate_bearing (UAM/util:321-334): math.degrees(x) = x * (180 / pi)
    const double th = atan2(yi - yh, xi - xh) * (180.0 / PI_GEOS);
    return th < 0 ? -th : 360 - th;
}

// Full Cyrus-Beck clip of segment c->e against the clockwise GEOS 64-gon(p, r): the entry if c is
// outside, the exit if c is inside (LineString.intersection(polygon.boundary), UAM/env:1429-1486)
__device__ bool ray_gon_boundary_full(double cx, double cy, double ex, double ey, double px, double py, double r,
                                      double &tout) {
    const double ddx = ex - cx, ddy = ey - cy;
    double tin = -INFINITY, tex = INFINITY;
    double vx = px + r * c_tab.circ_c[0], vy = py + r * c_tab.circ_s[0];
    for (int k = 0; k < 64; ++k) {
        const int k1 = (k + 1) & 63;
        const double wx = px + r * c_tab.circ_c[k1], wy = py + r * c_tab.circ_s[k1];
        const double exx = wx - vx, eyy = wy - vy;
        const double a = exx * (cy - vy) - eyy * (cx - vx);
        const double b = exx * ddy - eyy * ddx;
        if (b == 0.0) {
            if (a > 0.0) return false;
        } else if (b < 0.0) {
            const double t = -a / b;
            tin = t > tin ? t : tin;
        } else {
            const double t = -a / b;
            tex = t < tex ? t : tex;
        }
        vx = wx;
        vy = wy;
    }
    if (tin > tex) return false;
    if (tin >= 0.0) {
        if (tin > 1.0) return false;
        tout = tin;
        return true;
    }
    if (tex < 0.0 || tex > 1.0) return false;   // polygon behind, or the segment ends inside
    tout = tex;
    return true;
}

// The same result with fast paths (inv_l2 = 1 / |e - c|^2 of the ray):
//  * exact pre-filter: the 64-gon lies within the circle of radius r around p, so a segment that
//    passes farther than r + 1e-6 from p misses it (the reciprocal's rounding is far below 1e-6);
//  * c outside the circumscribed circle: the entry by the window clip of aac_geom.h;
//  * c inside the inscribed circle (so inside the polygon): every edge has a < 0, no entering edge
//    gives t >= 0, and the result is the exit min(-a/b) over the leaving edges.  The exit point lies
//    on the edge the ray crosses, within half an edge (pi/64) of the ray's exit angle from the
//    circumscribed circle, so the six edges around that angle hold the minimum: same vertices, same
//    arithmetic as the full clip, whose value it returns.
//  * anything else (c in the thin annulus between the circles): the full clip.
__device__ inline bool ray_gon_candidate(double cx, double cy, double ex, double ey, double px, double py, double r,
                                         double inv_l2) {
    const double ddx = ex - cx, ddy = ey - cy;
    const double wx = px - cx, wy = py - cy;
    double tt = (wx * ddx + wy * ddy) * inv_l2;
    tt = tt < 0.0 ? 0.0 : (tt > 1.0 ? 1.0 : tt);
    const double qx = tt * ddx - wx, qy = tt * ddy - wy;
    return qx * qx + qy * qy <= (r + 1e-6) * (r + 1e-6);
}

// ray_gon_boundary past its pre-filter (the caller has established ray_gon_candidate)
__device__ bool ray_gon_boundary_cand(double cx, double cy, double ex, double ey, double px, double py, double r,
                                      double &tout) {
    const double ddx = ex - cx, ddy = ey - cy;
    const double wx = px - cx, wy = py - cy;
    const double w2 = wx * wx + wy * wy;
    if (w2 > r * r * (1.0 + 1e-9)) return ray_poly_entry(cx, cy, ex, ey, px, py, r, tout);
    const double ap = r * c_tab.apothem;
    if (w2 < ap * ap * (1.0 - 1e-9)) {
        const double L = sqrt(ddx * ddx + ddy * ddy);
        const double s0 = (wx * ddx + wy * ddy) / L;
        const double h2 = w2 - s0 * s0;
        const double to = (s0 + sqrt(fmax(r * r - h2, 0.0))) / L;      // circumscribed-circle exit
        const float phi = atan2f((float)(cy + to * ddy - py), (float)(cx + to * ddx - px));
        const int i0 = (int)lrintf(-phi * (64.0f / 6.28318530717958647f));
        double tex = INFINITY;
#pragma unroll
        for (int dk = -3; dk <= 2; ++dk) {
            const int k = (i0 + dk) & 63, k1 = (k + 1) & 63;
            const double vx = px + r * c_tab.circ_c[k], vy = py + r * c_tab.circ_s[k];
            const double qx = px + r * c_tab.circ_c[k1], qy = py + r * c_tab.circ_s[k1];
            const double exx = qx - vx, eyy = qy - vy;
            const double a = exx * (cy - vy) - eyy * (cx - vx);
            const double b = exx * ddy - eyy * ddx;
            if (b > 0.0) {
                const double t = -a / b;
                tex = t < tex ? t : tex;
            }
        }
        if (tex == INFINITY) return ray_gon_boundary_full(cx, cy, ex, ey, px, py, r, tout);
        if (tex > 1.0) return false;
        tout = tex;
        return true;
    }
    return ray_gon_boundary_full(cx, cy, ex, ey, px, py, r, tout);
}

__device__ inline bool ray_gon_boundary(double cx, double cy, double ex, double ey, double px, double py, double r,
                                        double inv_l2, double &tout) {
    return ray_gon_candidate(cx, cy, ex, ey, px, py, r, inv_l2) &&
           ray_gon_boundary_cand(cx, cy, ex, ey, px, py, r, tout);
}

// segment c->e vs the finite bound segment x = lx, y in [y0, y1] (UAM/env:1413-1427)
__device__ bool ray_vseg(double cx, double cy, double ex, double ey, double lx, double y0, double y1, double &d) {
    if ((cx - lx) * (ex - lx) > 0.0 || ex == cx) return false;
    const double t = (lx - cx) / (ex - cx);
    const double y = cy + t * (ey - cy);
    if (y < y0 || y > y1) return false;
    d = gdist(lx, y, cx, cy);
    return true;
}

__device__ bool ray_hseg(double cx, double cy, double ex, double ey, double ly, double x0, double x1, double &d) {
    if ((cy - ly) * (ey - ly) > 0.0 || ey == cy) return false;
    const double t = (ly - cy) / (ey - cy);
    const double x = cx + t * (ex - cx);
    if (x < x0 || x > x1) return false;
    d = gdist(x, ly, cx, cy);
    return true;
}

// interiors of 64-gon(p, r) and the rectangle centred p + (dx, dy) with half sizes hx, hy overlap
// (polygons_single_cloud_conflict vs the runway, UAM/util:291-297, UAM/env:4095-4106)
__device__ bool gon_rect_overlap(double dx, double dy, double hx, double hy, double r) {
    if (fabs(dx) >= hx + r || fabs(dy) >= hy + r) return false;
    const double ox = fmax(fabs(dx) - hx, 0.0), oy = fmax(fabs(dy) - hy, 0.0);
    const double dist = sqrt(ox * ox + oy * oy);
    if (dist > r * (1.0 + 1e-12) + 1e-12) return false;
    if (dist < r * c_tab.apothem * (1.0 - 1e-12) - 1e-12) return true;
    for (int k = 0; k < 32; ++k) {
        const double proj = fabs(dx * c_tab.nrm_c[k] + dy * c_tab.nrm_s[k]);
        const double lim = hx * fabs(c_tab.nrm_c[k]) + hy * fabs(c_tab.nrm_s[k]) + r * c_tab.apothem;
        if (proj >= lim) return false;
    }
    return true;
}

// ------------------------------------------------------------------------------ phases
// pairwise np.linalg.norm distances of the workgroup's aircraft, row la = [d(la, base + j)]_j
// (dynamic LDS, epb * N * N doubles); npnorm is symmetric in the sign of the difference
extern __shared__ double s_dist[];

__device__ void dist_row(const UArgs &A, const Lds &S, int la, int base) {
    const double2 p = S.pos[la];
    double *row = s_dist + (size_t)la * A.N;
    for (int j = 0; j < A.N; ++j) {
        const double2 q = S.pos[base + j];
        row[j] = npnorm(q.x - p.x, q.y - p.y);
    }
}

// (2) neighbour order: get_current_agent_nei(queue=True) is a stable sort by np.linalg.norm
// distance, i.e. rank_j = #{k : d_k < d_j or (d_k == d_j and k < j)}.  One (aircraft, neighbour)
// pair per work item over the whole workgroup (one thread per aircraft left three quarters of the
// threads idle on the N^2 comparisons: ~57 k cycles per workgroup at N = 16).
// N <= 16: one 16-lane DPP row per aircraft, lane j holding d_j; the row's 15 rotations (row_ror)
// bring every d_k to lane j, which counts the ranks in registers (no LDS reads in the loop).  Lanes
// j >= N and the aircraft itself hold +inf, which ranks after every real distance: the same rank as
// the LDS loop below.
__device__ inline double dpp_ror_f64(double x, int n) {
    const long long b = __double_as_longlong(x);
    int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    switch (n) {      // the DPP control must be an immediate: row_ror:n = 0x120 + n
#define ROR(k)                                                                      \
    case k:                                                                         \
        lo = __builtin_amdgcn_update_dpp(0, lo, 0x120 + k, 0xf, 0xf, false);        \
        hi = __builtin_amdgcn_update_dpp(0, hi, 0x120 + k, 0xf, 0xf, false);        \
        break;
        ROR(1) ROR(2) ROR(3) ROR(4) ROR(5) ROR(6) ROR(7) ROR(8) ROR(9) ROR(10) ROR(11) ROR(12) ROR(13) ROR(14)
        ROR(15)
#undef ROR
    }
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ inline int dpp_ror_i32(int x, int n) {
    switch (n) {
#define ROR(k) \
    case k: return __builtin_amdgcn_update_dpp(0, x, 0x120 + k, 0xf, 0xf, false);
        ROR(1) ROR(2) ROR(3) ROR(4) ROR(5) ROR(6) ROR(7) ROR(8) ROR(9) ROR(10) ROR(11) ROR(12) ROR(13) ROR(14)
        ROR(15)
#undef ROR
    }
    return x;
}

__device__ void order_phase_rows(const UArgs &A, Lds &S, int nag) {
    const int N = A.N;
    const int j = threadIdx.x & 15;
    for (int la0 = 0; la0 < nag; la0 += BLOCK / 16) {
        const int la = la0 + (threadIdx.x >> 4);     // uniform per 16-lane row
        const int le = la / N, i = la - le * N;
        const bool on = la < nag && S.active[le < A.epb ? le : 0];
        const double dj = (on && j < N && j != i) ? s_dist[(size_t)la * N + j] : INFINITY;
        int rank = 0;
#pragma unroll
        for (int s = 1; s < 16; ++s) {
            const double dk = dpp_ror_f64(dj, s);
            const int k = dpp_ror_i32(j, s);
            rank += (dk < dj) || (dk == dj && k < j);
        }
        if (on && j < N && j != i) S.order[la][rank] = (uint8_t)j;
    }
}

__device__ void order_phase(const UArgs &A, Lds &S, int nag) {
    const int N = A.N;
    if (N <= 16) {
        order_phase_rows(A, S, nag);
        return;
    }
    for (int w = threadIdx.x; w < nag * N; w += BLOCK) {
        const int la = w / N, j = w - la * N;
        const int le = la / N, i = la - le * N;
        if (!S.active[le] || j == i) continue;
        const double *row = s_dist + (size_t)la * N;
        const double dj = row[j];
        int rank = 0;
        for (int k = 0; k < N; ++k) {
            const double dk = row[k];
            rank += (k != i && k != j) && ((dk < dj) || (dk == dj && k < j));
        }
        S.order[la][rank] = (uint8_t)j;
    }
}

// (3) radar of aircraft i (UAM/env:1360-1486): per ray the minimum over the runway boundary, the 4
// bound segments, the cloud boundaries and the other aircraft's 64-gons; default the ray's GEOS length.
// The radar as a work list (the default): (3a) per (aircraft, ray) the fixed boundaries -- ray length,
// runway, bound segments -- and the cheap exact pre-filter of the 64-gons (the env's two clouds and
// the other aircraft), whose candidates are appended to an LDS list of (ray, polygon) clip jobs;
// (3b) the clips of the list spread evenly over all 256 threads, each hit folded into its ray by an
// LDS atomic min on the (non-negative) float64 bits; (3c) the rays to HBM.  The per-ray loop of
// radar_ray ran the clips of one ray in one lane, so a wave waited for its most crowded ray (the
// crowded start zones give rays with 5-10 candidates beside rays with none): 2/3 of the step
// kernel's cycles.  The minimum does not depend on the order: bit-identical to radar_ray.
// A job is (w << 8) | j: w = local aircraft * NRAY + ray, j < 64 another aircraft, 64 + k cloud k.
// A list that would overflow CLIP_CAP leaves the lane to clip its remaining candidates itself.
__device__ inline double ray_clip_dist(const UArgs &A, const Lds &S, int le, int base, int i, int r, int j,
                                       bool &hit) {
    const double2 p = S.pos[base + i];
    const double cx = p.x, cy = p.y;
    const double ex = cx + A.radar_len * c_tab.ray_c[r], ey = cy + A.radar_len * c_tab.ray_s[r];
    double2 q;
    double rad;
    if (j >= 64) {
        q = S.cl[le][j - 64];
        rad = c_world.radius[j - 64];
    } else {
        q = S.pos[base + j];
        rad = A.pb;
    }
    double t;
    hit = ray_gon_boundary_cand(cx, cy, ex, ey, q.x, q.y, rad, t);
    return hit ? gdist(cx + t * (ex - cx), cy + t * (ey - cy), cx, cy) : 0.0;
}

// overflow clips of the pair pass land after every ray's base value (phase 3a) has been written:
// fold them in with the same LDS atomic min as the list's clips (non-negative float64 bits)
__device__ inline void pending_min(Lds &S, int la, int r, double d) {
    atomicMin(reinterpret_cast<unsigned long long *>(&S.rad[la][r]), (unsigned long long)__double_as_longlong(d));
}

// slots for a lane's cnt jobs: inclusive wave scan of the counts, one LDS atomic per wave (every
// lane of the wave calls it)
__device__ inline int clip_slots(Lds &S, int cnt) {
    const int lane = threadIdx.x & 63;
    int incl = cnt;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const int v = __shfl_up(incl, dd, 64);
        if (lane >= dd) incl += v;
    }
    int wbase = 0;
    if (lane == 63 && incl > 0) wbase = (int)atomicAdd(&S.nclip, (unsigned)incl);
    wbase = __shfl(wbase, 63, 64);
    return wbase + incl - cnt;
}

__device__ void radar_phase(const UArgs &A, Lds &S, int e0, int nag, const int32_t *emap = nullptr) {
    const int total = nag * NRAY;
    if (threadIdx.x == 0) S.nclip = 0;
    __syncthreads();
    // (3a) per (aircraft, ray): the fixed boundaries and the clouds' pre-filter; uniform trip count
    // so that every lane joins the wave scan
    for (int w0 = 0; w0 < total; w0 += BLOCK) {
        const int w = w0 + threadIdx.x;
        const int la = w / NRAY, r = w - la * NRAY;
        const int le = la / A.N, i = la - le * A.N;
        const bool on = w < total && S.active[le < A.epb ? le : 0] && (emap ? emap[le] : e0 + le) < A.E;
        double best = 0.0;
        int ccl = 0;                      // clouds (bits 0, 1)
        if (on) {
            const int base = le * A.N;
            const double2 p = S.pos[base + i];
            const double cx = p.x, cy = p.y;
            const double ex = cx + A.radar_len * c_tab.ray_c[r], ey = cy + A.radar_len * c_tab.ray_s[r];
            best = gdist(ex, ey, cx, cy);
            double d;
            // the runway's slab test (four divisions) only for segments whose bounding box comes
            // within 1e-9 of the rectangle: farther, the exact test cannot report a hit
            const double *rw = c_world.runway;
            if (fmax(cx, ex) >= rw[0] - 1e-9 && fmin(cx, ex) <= rw[1] + 1e-9 && fmax(cy, ey) >= rw[2] - 1e-9 &&
                fmin(cy, ey) <= rw[3] + 1e-9 && ray_square(cx, cy, ex, ey, rw[0], rw[1], rw[2], rw[3], d) && d < best)
                best = d;
            const double *b = A.bound;
            if (ray_vseg(cx, cy, ex, ey, b[0], b[2], b[3], d) && d < best) best = d;
            if (ray_vseg(cx, cy, ex, ey, b[1], b[2], b[3], d) && d < best) best = d;
            if (ray_hseg(cx, cy, ex, ey, b[3], b[0], b[1], d) && d < best) best = d;
            if (ray_hseg(cx, cy, ex, ey, b[2], b[0], b[1], d) && d < best) best = d;
            const double inv_l2 = 1.0 / ((ex - cx) * (ex - cx) + (ey - cy) * (ey - cy));
            for (int k = 0; k < 2; ++k) {
                const double2 c = S.cl[le][k];
                if (ray_gon_candidate(cx, cy, ex, ey, c.x, c.y, c_world.radius[k], inv_l2)) ccl |= 1 << k;
            }
        }
        int slot = clip_slots(S, __popc(ccl));
        if (on) {
            while (ccl) {
                const int j = 64 + __builtin_ctz(ccl);
                ccl &= ccl - 1;
                if (slot < CLIP_CAP) {
                    S.clip[slot] = ((uint32_t)w << 8) | (uint32_t)j;
                } else {          // list full: clip it here (same arithmetic, same minimum)
                    bool hit;
                    const double d = ray_clip_dist(A, S, le, le * A.N, i, r, j, hit);
                    if (hit && d < best) best = d;
                }
                ++slot;
            }
            S.rad[la][r] = best;
        }
    }
    __syncthreads();     // every ray's base value is in S.rad before 3a' may fold overflow clips into it
    // (3a') per (aircraft, other aircraft): which of the 18 rays can meet the other's 64-gon.  A
    // float32 superset of ray_gon_candidate's test (segment-to-centre distance <= pB + 1e-6): the
    // centre within pB + 1e-6 + 1e-3 of the ray's line and of its extent; the 1e-3 margin is far
    // above float32 rounding at these coordinates (~1e-5), and a pair outside the exact test that
    // gets through only costs a clip that reports no hit (the clips are exact for any segment).
    // Per pair instead of per ray: 18 float32 tests replace 18 float64 ones, the candidates'
    // distances come out of one subtraction.
    const int npair = nag * A.N;
    const float lim = (float)A.pb + 1e-6f + 1e-3f, Lf = (float)A.radar_len + lim;
    for (int p0 = 0; p0 < npair; p0 += BLOCK) {
        const int pr = p0 + threadIdx.x;
        const int la = pr / A.N, j = pr - la * A.N;
        const int le = la / A.N, i = la - le * A.N;
        const bool on = pr < npair && j != i && S.active[le < A.epb ? le : 0] &&
                        (emap ? emap[le] : e0 + le) < A.E;
        unsigned rays = 0;
        if (on) {
            const int base = le * A.N;
            const double2 p = S.pos[base + i], q = S.pos[base + j];
            const float dx = (float)(q.x - p.x), dy = (float)(q.y - p.y);
#pragma unroll
            for (int r = 0; r < NRAY; ++r) {
                const float c = (float)c_tab.ray_c[r], sn = (float)c_tab.ray_s[r];
                const float perp = dx * sn - dy * c, along = dx * c + dy * sn;
                if (fabsf(perp) <= lim && along >= -lim && along <= Lf) rays |= 1u << r;
            }
        }
        int slot = clip_slots(S, __popc(rays));
        if (on && rays) {
            const int base = le * A.N;
            while (rays) {
                const int r = __builtin_ctz(rays);
                rays &= rays - 1;
                const int w = la * NRAY + r;
                if (slot < CLIP_CAP) {
                    S.clip[slot] = ((uint32_t)w << 8) | (uint32_t)j;
                } else {          // list full: clip it now; the ray's minimum through the LDS atomic
                    bool hit;
                    const double d = ray_clip_dist(A, S, le, base, i, r, j, hit);
                    if (hit) pending_min(S, la, r, d);
                }
                ++slot;
            }
        }
    }
    __syncthreads();
    USTAMP(7);
    // (3b) the clip jobs, evenly over the workgroup
    const int nj = S.nclip < (unsigned)CLIP_CAP ? (int)S.nclip : CLIP_CAP;
    for (int q = threadIdx.x; q < nj; q += BLOCK) {
        const uint32_t job = S.clip[q];
        const int w = (int)(job >> 8), j = (int)(job & 255u);
        const int la = w / NRAY, r = w - la * NRAY;
        const int le = la / A.N, i = la - le * A.N;
        bool hit;
        const double d = ray_clip_dist(A, S, le, le * A.N, i, r, j, hit);
        if (hit) atomicMin(reinterpret_cast<unsigned long long *>(&S.rad[la][r]), (unsigned long long)__double_as_longlong(d));
    }
    __syncthreads();
    USTAMP(8);
    // (3c) the rays to HBM
    for (int w = threadIdx.x; w < total; w += BLOCK) {
        const int la = w / NRAY, r = w - la * NRAY;
        const int le = la / A.N, i = la - le * A.N;
        const int e = emap ? emap[le] : e0 + le;
        if (e >= A.E || !S.active[le]) continue;
        A.radar[((size_t)e * A.N + i) * NRAY + r] = S.rad[la][r];
    }
}

// (4) observation rows (UAM/env:1616-1880) + tdCPA (UAM/env:1738-1745).  The own row and the two
// nearest neighbours per aircraft; the per-neighbour rows (p2, p3, tcpa / dcpa) as work items over
// (aircraft, neighbour slot) on all 256 threads -- one thread per aircraft ran K = 15 slots in a row
// on a single wave -- with the two potential-conflict counts summed by LDS atomics (integer sums:
// the order does not matter).
__device__ void observe_own(const UArgs &A, Lds &S, int e, int la, int i) {
    const size_t ai = (size_t)e * A.N + i;
    const double *b = A.bound;
    const double2 p = S.pos[la], v = S.vel[la], g = S.goal[la];
    const double npx = nmlz(p.x, b[0], b[1]), npy = nmlz(p.y, b[2], b[3]);
    double *own = A.own + ai * 7;
    own[0] = npx;
    own[1] = npy;
    own[2] = v.x / A.vmax;
    own[3] = v.y / A.vmax;
    own[4] = nmlz(g.x, b[0], b[1]) - npx;
    own[5] = nmlz(g.y, b[2], b[3]) - npy;
    own[6] = S.heading[la];
    A.top2[ai * 2 + 0] = A.K > 0 ? S.order[la][0] : NONE8;
    A.top2[ai * 2 + 1] = A.K > 1 ? S.order[la][1] : NONE8;
    S.ccnt[la] = 0;
    S.pcnt[la] = 0;
}

__device__ void observe_slot(const UArgs &A, Lds &S, int e, int la, int base, int i, int k) {
    const int N = A.N, K = A.K;
    const size_t ai = (size_t)e * N + i;
    const double *b = A.bound;
    const double2 p = S.pos[la], v = S.vel[la];
    const int j = S.order[la][k];
    const double2 q = S.pos[base + j], w = S.vel[base + j];
    if (A.nei) {
        const double npx = nmlz(p.x, b[0], b[1]), npy = nmlz(p.y, b[2], b[3]);
        double *nb = A.nei + (ai * K + k) * 5;
        nb[0] = npx - nmlz(q.x, b[0], b[1]);
        nb[1] = npy - nmlz(q.y, b[2], b[3]);
        nb[2] = w.x / A.vmax;
        nb[3] = w.y / A.vmax;
        nb[4] = S.heading[la];
    }
    if (A.nei6) {
        const double dxm = b[0] - b[1], dxM = b[1] - b[0], dym = b[2] - b[3], dyM = b[3] - b[2];
        double *n6 = A.nei6 + (ai * K + k) * 6;
        n6[0] = 2 * (((q.x - p.x) - dxm) / (dxM - dxm)) - 1;
        n6[1] = 2 * (((q.y - p.y) - dym) / (dyM - dym)) - 1;
        n6[2] = 2 * (((w.y - q.x) - dxm) / (dxM - dxm)) - 1;     // other_agent[-2] - other_agent[0]
        n6[3] = 2 * (((A.pb - q.y) - dym) / (dyM - dym)) - 1;    // other_agent[-1] - other_agent[1]
        n6[4] = w.x / A.vmax;
        n6[5] = w.y / A.vmax;
    }
    if (A.tcpa || A.conf_cur) {
        double tc, dc, t2, d2;
        int cc = 0, cp = 0;
        tdcpa(q.x, q.y, p.x, p.y, w.x, w.y, v.x, v.y, A.pb, tc, dc, cc);
        const double2 hp = S.ppos[la], hv = S.pvel[la];
        const double2 qp = S.ppos[base + j], wp = S.pvel[base + j];
        tdcpa(qp.x, qp.y, hp.x, hp.y, wp.x, wp.y, hv.x, hv.y, A.pb, t2, d2, cp);
        if (A.tcpa) {
            A.tcpa[ai * K + k] = tc;
            A.dcpa[ai * K + k] = dc;
        }
        if (cc) atomicAdd(&S.ccnt[la], cc);
        if (cp) atomicAdd(&S.pcnt[la], cp);
    }
}

// the whole phase for the workgroup's aircraft (step and reset); ends with a barrier
__device__ void observe_phase(const UArgs &A, Lds &S, int e0, int nag, const int32_t *emap) {
    const int N = A.N, K = A.K;
    for (int la = threadIdx.x; la < nag; la += BLOCK) {
        const int le = la / N, i = la - le * N;
        const int e = emap ? emap[le] : e0 + le;
        if (e < A.E && S.active[le]) observe_own(A, S, e, la, i);
    }
    __syncthreads();
    for (int w = threadIdx.x; w < nag * K; w += BLOCK) {
        const int la = w / K, k = w - la * K;
        const int le = la / N, i = la - le * N;
        const int e = emap ? emap[le] : e0 + le;
        if (e < A.E && S.active[le]) observe_slot(A, S, e, la, le * N, i, k);
    }
    __syncthreads();
    if (A.conf_cur)
        for (int la = threadIdx.x; la < nag; la += BLOCK) {
            const int le = la / N, i = la - le * N;
            const int e = emap ? emap[le] : e0 + le;
            if (e < A.E && S.active[le]) {
                A.conf_cur[(size_t)e * N + i] = S.ccnt[la];
                A.conf_pre[(size_t)e * N + i] = S.pcnt[la];
            }
        }
}

__device__ inline void lds_agent(Lds &S, int la, double2 pos, double2 vel, double2 pp, double2 pv, double2 g,
                                 double hd) {
    S.pos[la] = pos;
    S.vel[la] = vel;
    S.ppos[la] = pp;
    S.pvel[la] = pv;
    S.goal[la] = g;
    S.heading[la] = hd;
}

// the reset of the workgroup's envs with S.active set (local slot -> env: emap, or e0 + slot):
// episode draw, clouds, aircraft, then the observation (UAM/env:551-771); the step tail and the reset
// kernel share it.  src: an LDS array of MAXA ints.
__device__ __attribute__((always_inline)) void reset_envs(const UArgs &A, const UReset &R, Lds &S, int e0, const int32_t *emap,
                                                     int32_t *src) {
    const int N = A.N;
    const int nag = A.epb * N;
    const int t = threadIdx.x;
    const auto env_of = [&](int q) { return emap ? emap[q] : e0 + q; };
    const int le = t / N, i = t - le * N;
    const int e = env_of(le < A.epb ? le : 0);
    const bool active = (t < nag) && (e < A.E) && S.active[le];
    const int base = le * N;
    const size_t ai = (size_t)e * N + i;
    // which episode each resetting env takes (bank: a fresh draw per reset)
    if (t < A.epb && S.active[t]) {
        const int eq = env_of(t);
        if (R.mode == 1) {
            const int ep = A.episode[eq] + 1;
            A.episode[eq] = ep;
            src[t] = (int)(mix64(mix64(R.seed ^ (uint64_t)eq) ^ (uint64_t)ep) % (uint64_t)R.bank_n);
        } else {
            src[t] = eq;
        }
    }
    __syncthreads();
    // clouds (UAM/env:576-703)
    if (t < 2 * A.epb && S.active[t >> 1]) {
        const int lq = t >> 1, k = t & 1, eq = env_of(lq);
        const int kind = R.clouds[src[lq] * 2 + k];
        const double2 c = k == 0 ? make_double2(c_world.cloud_start[kind][0], c_world.cloud_start[kind][1])
                                 : make_double2(c_world.path[kind][0][0], c_world.path[kind][0][1]);
        A.clouds[eq * 2 + k] = c;
        A.cloud_kind[eq * 2 + k] = kind;
        if (k == 1) A.cloud_tgt[eq] = 1;
        if (k == 0) A.step[eq] = 0;
        S.cl[lq][k] = c;
    }
    // aircraft (UAM/env:733-771)
    if (active) {
        const size_t si = (size_t)src[le] * N + i;
        const double2 st = R.start[si], g = R.goal[si];
        const double hd = atan2(g.y - st.y, g.x - st.x);
        const double2 v = make_double2(0 * cos(hd), 0 * sin(hd));
        A.pos[ai] = st;
        A.pre_pos[ai] = st;
        A.start[ai] = st;
        A.goal[ai] = g;
        A.vel[ai] = v;
        A.pre_vel[ai] = v;
        A.heading[ai] = hd;
        A.reach[ai] = 0;
        lds_agent(S, t, st, v, st, v, g, hd);
    }
    __syncthreads();
    if (active) dist_row(A, S, t, base);
    __syncthreads();
    order_phase(A, S, nag);
    __syncthreads();
    radar_phase(A, S, e0, nag, emap);
    __syncthreads();
    observe_phase(A, S, e0, nag, emap);
}

// ------------------------------------------------------------------------------- step
// (the replay push inside this launch was built, bit-exact, and measured slower: the launch grew 188 ->
// 234 us against the 23-us push launch it replaced; so was the bank reset of the finished envs in it,
// config 5 226 vs 238 M agent-env-steps/s; round 5, removed in round 6)
__global__ void __launch_bounds__(BLOCK, AAC_UAM_MIN_WAVES) uam_step_kernel(UArgs A, const double2 *__restrict__ act) {
    __shared__ Lds S;

    const int N = A.N, K = A.K;
    const int nag = A.epb * N;
    const int e0 = blockIdx.x * A.epb;
    const int t = threadIdx.x; USTAMP(0);
    const int le = t / N, i = t - le * N;
    const int e = e0 + le;
    const bool active = (t < nag) && (e < A.E);
    const int base = le * N;
    const size_t ai = (size_t)e * N + i;
    if (t < A.epb) S.active[t] = (e0 + t) < A.E;

    // ---- (0) clouds: drifting cloud -> its goal, go-around aircraft along its loop (UAM/env:4681-4697)
    if (t < 2 * A.epb) {
        const int lq = t >> 1, k = t & 1, eq = e0 + lq;
        if (eq < A.E) {
            const double2 c = A.clouds[eq * 2 + k];
            const int kind = A.cloud_kind[eq * 2 + k];
            double tx, ty;
            if (k == 1) {
                // corridor = LineString([pre_pos, pos]).buffer(1) with pre_pos == pos is the 64-gon
                // at pos; it meets target.buffer(0.5) -> next preset point (UAM/util:41-51)
                int tg = A.cloud_tgt[eq];
                const double *pt = c_world.path[kind][tg];
                if (gons_meet(pt[0] - c.x, pt[1] - c.y, c_world.radius[1] + 0.5, false)) {
                    tg = (c_world.path_first[kind][tg] + 1) % 6;
                    A.cloud_tgt[eq] = tg;
                }
                tx = c_world.path[kind][tg][0];
                ty = c_world.path[kind][tg][1];
            } else {
                tx = c_world.cloud_goal[kind][0];
                ty = c_world.cloud_goal[kind][1];
            }
            // calculate_next_position (UAM/util:300-318)
            const double dx = tx - c.x, dy = ty - c.y;
            const double dist = npnorm(dx, dy);
            const double ux = dist < 1 ? 0.0 : dx / dist, uy = dist < 1 ? 0.0 : dy / dist;
            const double step = c_world.vel[k] * A.dt;
            const double2 nc = make_double2(c.x + ux * step, c.y + uy * step);
            A.clouds[eq * 2 + k] = nc;
            S.cl[lq][k] = nc;
        }
    }

    // ---- (1) kinematics (UAM/env:4716-4797)
    uint8_t old0 = NONE8, old1 = NONE8, reach = 0;
    double2 np = make_double2(0.0, 0.0), pp = np;
    if (active) {
        pp = A.pos[ai];
        const double2 pv = A.vel[ai];
        const double2 a = act[ai];
        reach = A.reach[ai];
        old0 = A.top2[ai * 2 + 0];
        old1 = A.top2[ai * 2 + 1];
        double hd = A.heading[ai];
        const double ax = a.x * A.acc_max, ay = a.y * A.acc_max;
        const double cvx = pv.x + ax * A.dt, cvy = pv.y + ay * A.dt;
        const double nh = atan2(cvy, cvx);
        double2 nv;
        if (npnorm(cvx, cvy) >= A.vmax) nv = make_double2(A.vmax * cos(nh), A.vmax * sin(nh));
        else nv = make_double2(cvx, cvy);
        double dx = 0.0, dy = 0.0;
        if (!reach) {
            dx = nv.x * A.dt;
            dy = nv.y * A.dt;
            hd = atan2(dy, dx);
        }
        np = make_double2(pp.x + dx, pp.y + dy);
        A.pre_pos[ai] = pp;
        A.pre_vel[ai] = pv;
        A.pos[ai] = np;
        A.vel[ai] = nv;
        A.heading[ai] = hd;
        lds_agent(S, t, np, nv, pp, pv, A.goal[ai], hd);
        S.reach[t] = reach;
    }
    __syncthreads(); USTAMP(1);
    if (active) dist_row(A, S, t, base);
    __syncthreads(); USTAMP(2);
    order_phase(A, S, nag);
    __syncthreads(); USTAMP(3);
    radar_phase(A, S, e0, nag);
    __syncthreads(); USTAMP(4);

    // ---- (4) observation; the goal touch of every aircraft first (UAM/env:3929-3936)
    observe_phase(A, S, e0, nag, nullptr);
    if (active) {
        const double2 g = S.goal[t];
        if (gons_meet(g.x - np.x, g.y - np.y, A.pb + 1.0, false)) S.reach[t] = 1;
    }
    __syncthreads(); USTAMP(5);

    // ---- (5) ss_reward_Mar_changeskin predicates of aircraft i (UAM/env:3937-4486)
    if (active) {
        const double px = np.x, py = np.y, pb = A.pb;
        const int me = S.reach[t];
        int ncoll = 0, nearest = -1, last = -1, prev_two = 0;
        double shortest = INFINITY;
        const double *drow = s_dist + (size_t)t * N;
        for (int k = 0; k < K; ++k) {
            const int j = S.order[t][k];
            const double d = drow[j];
            if (d < shortest) {
                shortest = d;
                nearest = j;
            }
            if (d <= pb * 2 && !(S.reach[base + j] || me)) {
                ++ncoll;
                last = j;
                prev_two |= (j == old0) || (j == old1);
            }
        }
        int cloud = 0;
        if (!me) {
            const double *rw = c_world.runway;
            cloud = gon_rect_overlap((rw[0] + rw[1]) / 2 - px, (rw[2] + rw[3]) / 2 - py, (rw[1] - rw[0]) / 2,
                                     (rw[3] - rw[2]) / 2, pb);
            for (int k = 0; k < 2 && !cloud; ++k) {
                const double2 c = S.cl[le][k];
                cloud = gons_meet(c.x - px, c.y - py, pb + c_world.radius[k], true);
            }
        }
        const double2 g = S.goal[t];
        const int goal = gons_meet(g.x - px, g.y - py, pb + 1.0, false);
        // dist_to_goal = 5 (1 - total_length_to_end_of_line(pos, ref_line) / L)  (UAM/env:4202-4208)
        const double2 s = A.start[ai];
        const double L = gdist(g.x, g.y, s.x, s.y);
        const double rdx = g.x - s.x, rdy = g.y - s.y;
        double fr = ((px - s.x) * rdx + (py - s.y) * rdy) / (rdx * rdx + rdy * rdy);
        fr = fr < 0.0 ? 0.0 : (fr > 1.0 ? 1.0 : fr);
        const double left = gdist(px, py, s.x + fr * rdx, s.y + fr * rdy) + (L - fr * L);
        const double dtg = 5.0 * (1 - (left / L));
        // near-drone band (UAM/env:4305-4327); near-building penalty (UAM/env:4466-4481)
        uint8_t fl = 0;
        double ndv = 0.0;
        if (nearest >= 0 && shortest >= 2.0 && shortest <= 5.0) {
            const double2 q = S.pos[base + nearest];
            const double br = bearing(px, py, q.x, q.y);
            fl |= 1 | ((br >= 90.0 && br <= 180) << 1);
            ndv = ((0 - 1) / (5.0 - 2.0)) * shortest + (1 + (2.0 / (5.0 - 2.0)));
        }
        double mn = S.rad[t][0];
        for (int r = 1; r < NRAY; ++r) mn = S.rad[t][r] < mn ? S.rad[t][r] : mn;
        const double nbp = (mn >= pb && mn <= 5.0) ? 2.0 * (((0 - 1) / (5.0 - pb)) * mn + 2) : 0.0;
        const int bnd = capsule_crash(pb, A.bound, pp.x, pp.y, px, py);
        uint8_t kind;
        if (bnd) kind = 0;
        else if (cloud) kind = 1;
        else if (ncoll > 0) {
            kind = 2;
            const double2 q = S.pos[base + last];
            const double br = bearing(px, py, q.x, q.y);
            fl |= ((br >= 90.0 && br <= 180) << 2) | (prev_two << 3);
        } else if (goal) kind = 3;
        else kind = 4;
        S.kind[t] = kind;
        S.flag[t] = fl;
        S.nd_val[t] = ndv;
        S.base[t] = (0 + dtg) - nbp;
        A.mask[ai] = (uint8_t)(bnd | (cloud << 1) | ((ncoll > 0) << 2) | (goal << 3) | ((kind == 3) << 4) |
                               ((kind == 2 && prev_two) << 5));
        if (kind == 3) S.reach[t] = 1;
        A.reach[ai] = S.reach[t];
    }
    __syncthreads(); USTAMP(6);

    // ---- (6) per env, aircraft in order: the coefficient doubling persists over later aircraft
    //      of the same call (UAM/env:4320, :4546); done, bbc, termination (UAM/main:624-637).
    // N <= 16: one 16-lane row per env, lane j = aircraft j.  Each doubling multiplies by 2, which is
    // exact, so aircraft j's coefficients are 2.0 and 50.0 times 2^(doublings among aircraft 0..j):
    // an inclusive prefix count over the row (ballot + popcount) instead of the sequential walk.
    if (N <= 16) {
        const int q = t >> 4, j = t & 15;
        const int eq = e0 + q;
        const bool on = q < A.epb && eq < A.E && j < N;     // q uniform per row
        const int la = q * N + j;
        uint8_t fl = 0, kind = 4, rch = 1;
        if (on) {
            fl = S.flag[la];
            kind = S.kind[la];
            rch = S.reach[la];
        }
        const unsigned long long dbl_nd = __ballot(on && (fl & 1) && (fl & 2));
        const unsigned long long dbl_cr = __ballot(on && kind == 2 && (fl & 4));
        const int sh = 16 * ((t >> 4) & 3);
        const unsigned long long upto = ((2ull << j) - 1) << sh, row = 0xffffull << sh;
        const double ndc = ldexp(2.0, __popcll(dbl_nd & upto));
        const double crash = ldexp(50.0, __popcll(dbl_cr & upto));
        int dn = 0;
        if (on) {
            const double nd = (fl & 1) ? ndc * S.nd_val[la] : ndc * 0;
            double rew;
            dn = 1;
            if (kind == 0 || kind == 1 || kind == 2) {
                rew = 0 - crash;
            } else if (kind == 3) {
                rew = 0 + 50.0 + 0;
                dn = 0;
            } else {
                rew = S.base[la] - nd;
                dn = 0;
            }
            const size_t aj = (size_t)eq * N + j;
            A.reward[aj] = rew;
            A.done[aj] = (uint8_t)dn;
        }
        const unsigned long long m_done = __ballot(on && dn), m_nreach = __ballot(on && !rch);
        const unsigned long long m_k0 = __ballot(on && kind == 0), m_k1 = __ballot(on && kind == 1);
        const unsigned long long m_k2 = __ballot(on && kind == 2), m_k3 = __ballot(on && kind == 2 && (fl & 8));
        if (on && j == 0) {
            A.bbc[4 * eq + 0] = (m_k0 & row) != 0;
            A.bbc[4 * eq + 1] = (m_k1 & row) != 0;
            A.bbc[4 * eq + 2] = (m_k2 & row) != 0;
            A.bbc[4 * eq + 3] = (m_k3 & row) != 0;
            const int st = A.step[eq] + 1;
            A.step[eq] = st;
            A.env_done[eq] = (uint8_t)((A.episode_length < st) || (m_done & row) != 0 || (m_nreach & row) == 0);
        }
    } else if (t < A.epb && e0 + t < A.E) {
        const int eq = e0 + t, bq = t * N;
        double crash = 50.0, ndc = 2.0;
        int any_done = 0, all_reach = 1;
        uint8_t bb[4] = {0, 0, 0, 0};
        for (int j = 0; j < N; ++j) {
            const int la = bq + j;
            const uint8_t fl = S.flag[la], kind = S.kind[la];
            double nd;
            if (fl & 1) {
                if (fl & 2) ndc = ndc * 2;
                nd = ndc * S.nd_val[la];
            } else {
                nd = ndc * 0;
            }
            double rew;
            int dn = 1;
            if (kind == 0) {
                rew = 0 - crash;
                bb[0] = 1;
            } else if (kind == 1) {
                rew = 0 - crash;
                bb[1] = 1;
            } else if (kind == 2) {
                if (fl & 4) crash = crash * 2;
                rew = 0 - crash;
                bb[2] = 1;
                if (fl & 8) bb[3] = 1;
            } else if (kind == 3) {
                rew = 0 + 50.0 + 0;
                dn = 0;
            } else {
                rew = S.base[la] - nd;
                dn = 0;
            }
            const size_t aj = (size_t)eq * N + j;
            A.reward[aj] = rew;
            A.done[aj] = (uint8_t)dn;
            any_done |= dn;
            all_reach &= S.reach[la];
        }
        for (int q = 0; q < 4; ++q) A.bbc[4 * eq + q] = bb[q];
        const int st = A.step[eq] + 1;
        A.step[eq] = st;
        A.env_done[eq] = (uint8_t)((A.episode_length < st) || any_done || all_reach);
    }
    USTAMP(15);
}

// ------------------------------------------------------------------------------ reset
__global__ void __launch_bounds__(BLOCK) uam_reset_kernel(UArgs A, UReset R) {
    __shared__ Lds S;
    const int e0 = blockIdx.x * A.epb;
    const int t = threadIdx.x;
    // local env slot -> env: contiguous, or the compacted list of resetting envs (so that every
    // workgroup that runs has epb envs to reset instead of the few of its contiguous range)
    __shared__ int32_t emap[MAXA];
    __shared__ int32_t src[MAXA];
    if (t < A.epb) {
        if (R.list) {
            const int q = e0 + t;
            const bool on = q < R.list[0];
            emap[t] = on ? R.list[1 + q] : 0;
            S.active[t] = on;
        } else {
            const int eq = e0 + t;
            emap[t] = eq;
            S.active[t] = (eq < A.E) && (R.mask == nullptr || R.mask[eq] != 0);
        }
    }
    __syncthreads();
    int any = 0;
    for (int k = 0; k < A.epb; ++k) any |= S.active[k];
    if (!any) return;
    reset_envs(A, R, S, e0, emap, src);
}

// ordered list of the done envs for the packed auto-reset (aacw::compact_flags)
__global__ void __launch_bounds__(1024) uam_compact_kernel(const uint8_t *__restrict__ mask, int E, int32_t *rlist) {
    aacw::compact_flags(mask, E, rlist);
}

// exactness check of ray_gon_boundary's fast paths against the full clip (aac_uam_ray_gon_check):
// random segments of radar length from points around a 64-gon, focused on the inside / annulus /
// near-tangent cases; counts results that differ in the hit flag or any bit of t
__global__ void ray_gon_check_kernel(int64_t n, uint64_t seed, double r, double len, unsigned long long *bad) {
    unsigned long long nb = 0;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h1 = mix64(seed ^ (uint64_t)q), h2 = mix64(h1), h3 = mix64(h2);
        const double u1 = (double)(h1 >> 11) * (1.0 / 9007199254740992.0);
        const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
        const double u3 = (double)(h3 >> 11) * (1.0 / 9007199254740992.0);
        // origin radius: half the cases inside the polygon, the rest up to 3 r (entry / miss / annulus)
        const double rad = (q & 1) ? r * u1 : r * 3.0 * u1;
        const double ang = 6.283185307179586 * u2, dir = 6.283185307179586 * u3;
        const double px = 1.25, py = -0.75;
        const double cx = px + rad * cos(ang), cy = py + rad * sin(ang);
        const double ex = cx + len * cos(dir), ey = cy + len * sin(dir);
        const double inv_l2 = 1.0 / ((ex - cx) * (ex - cx) + (ey - cy) * (ey - cy));
        double t1 = -7.0, t2 = -7.0;
        const bool a = ray_gon_boundary(cx, cy, ex, ey, px, py, r, inv_l2, t1);
        const bool b = ray_gon_boundary_full(cx, cy, ex, ey, px, py, r, t2);
        if (a != b || (a && __double_as_longlong(t1) != __double_as_longlong(t2))) ++nb;
    }
    if (nb) atomicAdd(bad, nb);
}

// ------------------------------------------------------------------------------ host side
thread_local std::string g_uerr;
// AAC_UAM_RESET_CONTIGUOUS=1: auto-reset over contiguous env ranges (no compaction; A/B and tests)
bool g_no_compact = [] {
    const char *v = getenv("AAC_UAM_RESET_CONTIGUOUS");
    return v && v[0] == '1';
}();

int ufail(int code, const std::string &msg) {
    g_uerr = msg;
    return code;
}

#define UCHK(x)                                                                                             \
    do {                                                                                                    \
        hipError_t _e = (x);                                                                                \
        if (_e != hipSuccess) return ufail(AAC_E_HIP, std::string(#x) + ": " + hipGetErrorString(_e));     \
    } while (0)

const int GO_AC[4][12] = {{20, 20, 20, 35, 5, 35, 5, 5, 20, 5, 20, 20},
                          {20, 20, 20, 5, 5, 5, 5, 35, 20, 35, 20, 20},
                          {20, 20, 20, 35, 35, 35, 35, 5, 20, 5, 20, 20},
                          {20, 20, 20, 5, 35, 5, 35, 35, 20, 35, 20, 20}};
const int CLOUD_SET[2][4] = {{8, 30, 10, 10}, {30, 10, 35, 30}};

void fill_world(World &w) {
    for (int k = 0; k < 2; ++k) {
        w.cloud_start[k][0] = CLOUD_SET[k][0];
        w.cloud_start[k][1] = CLOUD_SET[k][1];
        w.cloud_goal[k][0] = CLOUD_SET[k][2];
        w.cloud_goal[k][1] = CLOUD_SET[k][3];
    }
    for (int p = 0; p < 4; ++p)
        for (int q = 0; q < 6; ++q) {
            w.path[p][q][0] = GO_AC[p][2 * q];
            w.path[p][q][1] = GO_AC[p][2 * q + 1];
            int first = q;
            for (int r = 0; r < q; ++r)
                if (GO_AC[p][2 * r] == GO_AC[p][2 * q] && GO_AC[p][2 * r + 1] == GO_AC[p][2 * q + 1]) {
                    first = r;
                    break;
                }
            w.path_first[p][q] = first;
        }
    w.radius[0] = 3.0;   // cloud contour_range (UAM/cloud.py:18)
    w.radius[1] = 1.0;   // go-around aircraft separation radius (UAM/cloud.py:46)
    w.vel[0] = 0.4;
    w.vel[1] = 2.0;
    w.runway[0] = 18.0;
    w.runway[1] = 22.0;
    w.runway[2] = 10.0;
    w.runway[3] = 30.0;
}

// ----- episode sampling rules (UAM/env:575-747, UAM/util:165-237) with a splitmix stream
struct Rng {
    uint64_t s;
    uint64_t next() { return mix64(s++); }
    double uniform(double a, double b) { return a + (b - a) * ((double)(next() >> 11) * (1.0 / 9007199254740992.0)); }
    int below(int n) { return (int)(next() % (uint64_t)n); }
};

struct Rect {
    double x0, x1, y0, y1;
};

std::vector<Rect> end_regions(int cloud0, double x_start, const double *b) {
    std::vector<Rect> nofly;
    const int sx[2] = {CLOUD_SET[cloud0][0], GO_AC[0][0]}, sy[2] = {CLOUD_SET[cloud0][1], GO_AC[0][1]};
    for (int k = 0; k < 2; ++k) nofly.push_back({sx[k] - 5.0, sx[k] + 5.0, sy[k] - 5.0, sy[k] + 5.0});
    nofly.push_back({b[0], b[1], b[2], b[2] + 5});
    nofly.push_back({b[0], b[1], b[3] - 5, b[3]});
    nofly.push_back({b[0], b[0] + 5, b[2], b[3]});
    nofly.push_back({b[1] - 5, b[1], b[2], b[3]});
    std::vector<Rect> reg = {{b[0], b[1], b[2], b[3]}};
    for (const Rect &z : nofly) {
        std::vector<Rect> nw;
        for (const Rect &r : reg) {
            if (r.x0 < z.x1 && r.x1 > z.x0 && r.y0 < z.y1 && r.y1 > z.y0) {
                if (r.x0 < z.x0) nw.push_back({r.x0, z.x0, r.y0, r.y1});
                if (r.x1 > z.x1) nw.push_back({z.x1, r.x1, r.y0, r.y1});
                if (r.y0 < z.y0) nw.push_back({std::max(r.x0, z.x0), std::min(r.x1, z.x1), r.y0, z.y0});
                if (r.y1 > z.y1) nw.push_back({std::max(r.x0, z.x0), std::min(r.x1, z.x1), z.y1, r.y1});
            } else {
                nw.push_back(r);
            }
        }
        reg = nw;
    }
    std::vector<Rect> out;
    for (const Rect &r : reg)
        if ((x_start < 18.0 && r.x1 <= 18.0) || (x_start > 22.0 && r.x0 >= 22.0)) out.push_back(r);
    return out;
}

}  // namespace

struct aac_uam {
    aac_uam_cfg cfg;
    int device, K, epb, blocks;
    double2 *pos, *vel, *pre_pos, *pre_vel, *goal, *start, *clouds;
    double *heading;
    uint8_t *reach, *top2;
    int32_t *cloud_kind, *cloud_tgt, *step, *episode;
    double2 *bank_start, *bank_goal;
    int32_t *bank_clouds;
    int32_t bank_n;
    uint64_t bank_seed;
    int32_t *rlist;           // [1 + E]: compacted resetting envs of the last auto-reset
    int32_t *episode_own;     // the handle's own counter buffer (episode may be a caller's buffer)
};

static size_t dist_bytes(const aac_uam *h) { return sizeof(double) * (size_t)h->epb * h->cfg.N * h->cfg.N; }

static UArgs make_uargs(const aac_uam *h, const aac_uam_out *o) {
    UArgs A;
    std::memset(&A, 0, sizeof(A));
    const aac_uam_cfg &c = h->cfg;
    A.E = c.E;
    A.N = c.N;
    A.K = h->K;
    A.epb = h->epb;
    A.episode_length = c.episode_length;
    A.dt = c.dt;
    A.acc_max = c.acc_max;
    A.vmax = c.vmax;
    A.pb = c.pB;
    A.radar_len = c.radar_len;
    for (int k = 0; k < 4; ++k) A.bound[k] = c.bound[k];
    A.pos = h->pos;
    A.vel = h->vel;
    A.pre_pos = h->pre_pos;
    A.pre_vel = h->pre_vel;
    A.goal = h->goal;
    A.start = h->start;
    A.clouds = h->clouds;
    A.heading = h->heading;
    A.reach = h->reach;
    A.top2 = h->top2;
    A.cloud_kind = h->cloud_kind;
    A.cloud_tgt = h->cloud_tgt;
    A.step = h->step;
    A.episode = h->episode;
    A.own = o->own;
    A.radar = o->radar;
    A.nei = o->nei;
    A.nei6 = o->nei6;
    A.reward = o->reward;
    A.tcpa = o->tcpa;
    A.dcpa = o->dcpa;
    A.conf_cur = o->conf_cur;
    A.conf_pre = o->conf_pre;
    A.done = o->done;
    A.mask = o->mask;
    A.env_done = o->env_done;
    A.bbc = o->bbc;
    return A;
}

static int check_uout(const aac_uam_out *o) {
    if (!o || !o->own || !o->radar) return ufail(AAC_E_INVALID, "own and radar outputs required");
    if ((o->tcpa == nullptr) != (o->dcpa == nullptr)) return ufail(AAC_E_INVALID, "tcpa/dcpa must be both set");
    if ((o->conf_cur == nullptr) != (o->conf_pre == nullptr)) return ufail(AAC_E_INVALID, "conf_cur/pre both");
    return AAC_OK;
}

extern "C" {

int aac_uam_ray_gon_check(int64_t n, uint64_t seed, double r, double len, uint64_t *bad) {
    if (n <= 0 || !bad || r <= 0.0 || len <= 0.0) return ufail(AAC_E_INVALID, "ray_gon_check: bad argument");
    unsigned long long *d = nullptr;
    UCHK(hipMalloc((void **)&d, sizeof(unsigned long long)));
    UCHK(hipMemset(d, 0, sizeof(unsigned long long)));
    hipLaunchKernelGGL(ray_gon_check_kernel, dim3(2048), dim3(256), 0, 0, n, seed, r, len, d);
    UCHK(hipGetLastError());
    unsigned long long hcount = 0;
    UCHK(hipMemcpy(&hcount, d, sizeof(hcount), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    *bad = hcount;
    return AAC_OK;
}

#ifdef AAC_UAM_STAMPS
int aac_uam_stamps(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_uam_st), sizeof(g_uam_st)) == hipSuccess ? 0 : -1;
}
#endif

const char *aac_uam_last_error(void) { return g_uerr.c_str(); }

int aac_uam_create(const aac_uam_cfg *cfg, int device, aac_uam **out) {
    if (!cfg || !out) return ufail(AAC_E_INVALID, "null argument");
    const aac_uam_cfg &c = *cfg;
    if (c.E <= 0 || c.N < 2 || c.N > MAXA) return ufail(AAC_E_INVALID, "need E > 0 and 2 <= N <= 64");
    if (!(c.radar_len > 0) || !(c.pB > 0) || !(c.vmax > 0) || !(c.bound[1] > c.bound[0]) || !(c.bound[3] > c.bound[2]))
        return ufail(AAC_E_INVALID, "bad geometry");
    UCHK(hipSetDevice(device));
    aac_uam *h = new aac_uam();
    std::memset(h, 0, sizeof(*h));
    h->cfg = c;
    h->device = device;
    h->K = c.N - 1;
    h->epb = MAXA / c.N;
    h->blocks = (c.E + h->epb - 1) / h->epb;
    const size_t EN = (size_t)c.E * c.N, E = c.E;
    hipError_t st = hipSuccess;
#define ALLOC(p, n)                                                              \
    if (st == hipSuccess) st = hipMalloc((void **)&h->p, (n) * sizeof(*h->p));   \
    if (st == hipSuccess) st = hipMemset(h->p, 0, (n) * sizeof(*h->p));
    ALLOC(pos, EN) ALLOC(vel, EN) ALLOC(pre_pos, EN) ALLOC(pre_vel, EN) ALLOC(goal, EN) ALLOC(start, EN)
    ALLOC(heading, EN) ALLOC(reach, EN) ALLOC(top2, EN * 2) ALLOC(clouds, E * 2) ALLOC(cloud_kind, E * 2)
    ALLOC(cloud_tgt, E) ALLOC(step, E) ALLOC(episode, E) ALLOC(rlist, E + 1)
    h->episode_own = h->episode;
#undef ALLOC
    if (st == hipSuccess) {
        Tab t;
        fill_tables(t);
        st = hipMemcpyToSymbol(HIP_SYMBOL(c_tab), &t, sizeof(Tab));
    }
    if (st == hipSuccess) {
        World w;
        fill_world(w);
        st = hipMemcpyToSymbol(HIP_SYMBOL(c_world), &w, sizeof(World));
    }
    if (st != hipSuccess) {
        aac_uam_destroy(h);
        return ufail(AAC_E_HIP, std::string("aac_uam_create: ") + hipGetErrorString(st));
    }
    *out = h;
    return AAC_OK;
}

void aac_uam_destroy(aac_uam *h) {
    if (!h) return;
    void *ptrs[] = {h->pos,   h->vel,        h->pre_pos,   h->pre_vel, h->goal,    h->start,      h->clouds,
                    h->heading, h->reach,    h->top2,      h->cloud_kind, h->cloud_tgt, h->step, h->episode_own,
                    h->bank_start, h->bank_goal, h->bank_clouds, h->rlist};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete h;
}

int aac_uam_step(aac_uam *h, const double *actions, const aac_uam_out *o, void *stream) {
    if (!h || !actions) return ufail(AAC_E_INVALID, "null argument");
    int rc = check_uout(o);
    if (rc) return rc;
    if (!o->reward || !o->done || !o->mask || !o->env_done || !o->bbc) return ufail(AAC_E_INVALID, "step outputs");
    UArgs A = make_uargs(h, o);
    hipLaunchKernelGGL(uam_step_kernel, dim3(h->blocks), dim3(BLOCK), dist_bytes(h), (hipStream_t)stream, A,
                       reinterpret_cast<const double2 *>(actions));
    UCHK(hipGetLastError());
    return AAC_OK;
}

static int launch_reset(aac_uam *h, const UReset &R, const aac_uam_out *o, void *stream) {
    int rc = check_uout(o);
    if (rc) return rc;
    UArgs A = make_uargs(h, o);
    hipLaunchKernelGGL(uam_reset_kernel, dim3(h->blocks), dim3(BLOCK), dist_bytes(h), (hipStream_t)stream, A, R);
    UCHK(hipGetLastError());
    return AAC_OK;
}

int aac_uam_reset(aac_uam *h, const uint8_t *mask, const double *start, const double *goal, const int32_t *clouds,
                  const aac_uam_out *o, void *stream) {
    if (!h || !start || !goal || !clouds) return ufail(AAC_E_INVALID, "null argument");
    UReset R{};
    R.mode = 0;
    R.mask = mask;
    R.start = reinterpret_cast<const double2 *>(start);
    R.goal = reinterpret_cast<const double2 *>(goal);
    R.clouds = clouds;
    return launch_reset(h, R, o, stream);
}

int aac_uam_set_bank(aac_uam *h, const double *start, const double *goal, const int32_t *clouds, int32_t n,
                     uint64_t seed) {
    if (!h || !start || !goal || !clouds || n <= 0) return ufail(AAC_E_INVALID, "bad episode bank");
    for (int32_t k = 0; k < n; ++k)
        if (clouds[2 * k] < 0 || clouds[2 * k] > 1 || clouds[2 * k + 1] < 0 || clouds[2 * k + 1] > 3)
            return ufail(AAC_E_INVALID, "episode bank cloud choice out of range");
    UCHK(hipSetDevice(h->device));
    if (h->bank_start) { (void)hipFree(h->bank_start); (void)hipFree(h->bank_goal); (void)hipFree(h->bank_clouds); }
    h->bank_start = h->bank_goal = nullptr;
    h->bank_clouds = nullptr;
    const size_t nN = (size_t)n * h->cfg.N;
    UCHK(hipMalloc((void **)&h->bank_start, sizeof(double2) * nN));
    UCHK(hipMalloc((void **)&h->bank_goal, sizeof(double2) * nN));
    UCHK(hipMalloc((void **)&h->bank_clouds, sizeof(int32_t) * 2 * n));
    UCHK(hipMemcpy(h->bank_start, start, sizeof(double2) * nN, hipMemcpyHostToDevice));
    UCHK(hipMemcpy(h->bank_goal, goal, sizeof(double2) * nN, hipMemcpyHostToDevice));
    UCHK(hipMemcpy(h->bank_clouds, clouds, sizeof(int32_t) * 2 * n, hipMemcpyHostToDevice));
    h->bank_n = n;
    h->bank_seed = seed;
    return AAC_OK;
}

void aac_uam_set_reset_compact(int32_t on) { g_no_compact = on == 0; }

int aac_uam_use_episode_buffer(aac_uam *h, int32_t *episode_dev, void *stream) {
    if (!h || !episode_dev) return ufail(AAC_E_INVALID, "null argument");
    UCHK(hipSetDevice(h->device));
    // on the caller's stream: ordered after its pending auto-resets and its fill of episode_dev
    if (episode_dev != h->episode)
        UCHK(hipMemcpyAsync(episode_dev, h->episode, sizeof(int32_t) * (size_t)h->cfg.E, hipMemcpyDeviceToDevice,
                            (hipStream_t)stream));
    h->episode = episode_dev;
    return AAC_OK;
}

int aac_uam_auto_reset(aac_uam *h, const uint8_t *env_done, const aac_uam_out *o, void *stream) {
    if (!h) return ufail(AAC_E_INVALID, "null handle");
    if (!h->bank_n) return ufail(AAC_E_STATE, "no episode bank installed (aac_uam_set_bank)");
    UReset R{};
    R.mode = 1;
    R.mask = env_done;
    R.start = h->bank_start;
    R.goal = h->bank_goal;
    R.clouds = h->bank_clouds;
    R.bank_n = h->bank_n;
    R.seed = h->bank_seed;
    if (env_done && !g_no_compact) {
        hipLaunchKernelGGL(uam_compact_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, env_done, h->cfg.E,
                           h->rlist);
        UCHK(hipGetLastError());
        R.list = h->rlist;
    }
    return launch_reset(h, R, o, stream);
}

int aac_uam_bank_build(int32_t n, int32_t N, uint64_t seed, double *start, double *goal, int32_t *clouds) {
    if (n <= 0 || N < 2 || N > MAXA || !start || !goal || !clouds) return ufail(AAC_E_INVALID, "bad bank request");
    const double b[4] = {0.0, 40.0, 0.0, 40.0};
    const double zones[2][4] = {{15, 17, 15, 25}, {23, 25, 15, 25}};
    const double sep = 0.5 * 3;
    Rng rng{mix64(seed) ^ 0x5bd1e995ull};
    std::vector<Rect> regs[2][2];   // [cloud_0][side]
    for (int c0 = 0; c0 < 2; ++c0) {
        regs[c0][0] = end_regions(c0, 16.0, b);
        regs[c0][1] = end_regions(c0, 24.0, b);
    }
    for (int32_t k = 0; k < n; ++k) {
        const int c0 = rng.below(2), c1 = rng.below(4);
        clouds[2 * k] = c0;
        clouds[2 * k + 1] = c1;
        double *S = start + (size_t)k * N * 2, *G = goal + (size_t)k * N * 2;
        for (int a = 0; a < N; ++a) {
            double sx = 0, sy = 0;
            for (int tries = 0; tries < 100000; ++tries) {
                const double *z = zones[rng.below(2)];
                sx = rng.uniform(z[0], z[1]);
                sy = rng.uniform(z[2], z[3]);
                bool ok = true;
                for (int q = 0; q < a && ok; ++q) {
                    const double dx = sx - S[2 * q], dy = sy - S[2 * q + 1];
                    ok = std::sqrt(std::fma(dy, dy, dx * dx)) > sep;
                }
                if (ok) break;
            }
            const std::vector<Rect> &R = regs[c0][sx < 18.0 ? 0 : 1];
            if (R.empty()) return ufail(AAC_E_STATE, "no end region on the start's side of the runway");
            const Rect &r = R[rng.below((int)R.size())];
            S[2 * a] = sx;
            S[2 * a + 1] = sy;
            G[2 * a] = rng.uniform(r.x0, r.x1);
            G[2 * a + 1] = rng.uniform(r.y0, r.y1);
        }
    }
    return AAC_OK;
}

#define UCPY(dst, src, n)                                                                                   \
    if (dst && src) UCHK(hipMemcpyAsync((void *)(dst), (const void *)(src), (n), hipMemcpyDeviceToDevice,   \
                                        (hipStream_t)stream));

int aac_uam_get_state(aac_uam *h, double *pos, double *vel, double *pre_pos, double *pre_vel, double *goal,
                      double *start, double *heading, uint8_t *reach, double *clouds, int32_t *cloud_kind,
                      int32_t *cloud_tgt, int32_t *step, uint8_t *top2, void *stream) {
    if (!h) return ufail(AAC_E_INVALID, "null handle");
    const size_t EN = (size_t)h->cfg.E * h->cfg.N, E = h->cfg.E;
    UCPY(pos, h->pos, EN * 16) UCPY(vel, h->vel, EN * 16) UCPY(pre_pos, h->pre_pos, EN * 16)
    UCPY(pre_vel, h->pre_vel, EN * 16) UCPY(goal, h->goal, EN * 16) UCPY(start, h->start, EN * 16)
    UCPY(heading, h->heading, EN * 8) UCPY(reach, h->reach, EN) UCPY(clouds, h->clouds, E * 32)
    UCPY(cloud_kind, h->cloud_kind, E * 8) UCPY(cloud_tgt, h->cloud_tgt, E * 4) UCPY(step, h->step, E * 4)
    UCPY(top2, h->top2, EN * 2)
    return AAC_OK;
}

int aac_uam_set_state(aac_uam *h, const double *pos, const double *vel, const double *pre_pos, const double *pre_vel,
                      const double *goal, const double *start, const double *heading, const uint8_t *reach,
                      const double *clouds, const int32_t *cloud_kind, const int32_t *cloud_tgt, const int32_t *step,
                      const uint8_t *top2, void *stream) {
    if (!h) return ufail(AAC_E_INVALID, "null handle");
    const size_t EN = (size_t)h->cfg.E * h->cfg.N, E = h->cfg.E;
    UCPY(h->pos, pos, EN * 16) UCPY(h->vel, vel, EN * 16) UCPY(h->pre_pos, pre_pos, EN * 16)
    UCPY(h->pre_vel, pre_vel, EN * 16) UCPY(h->goal, goal, EN * 16) UCPY(h->start, start, EN * 16)
    UCPY(h->heading, heading, EN * 8) UCPY(h->reach, reach, EN) UCPY(h->clouds, clouds, E * 32)
    UCPY(h->cloud_kind, cloud_kind, E * 8) UCPY(h->cloud_tgt, cloud_tgt, E * 4) UCPY(h->step, step, E * 4)
    UCPY(h->top2, top2, EN * 2)
    return AAC_OK;
}
#undef UCPY

}  // extern "C"
