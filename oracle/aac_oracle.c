/* aac_oracle.c -- batched CPU restatement of the one_model_att environment step.
 *
 * TEST INFRASTRUCTURE ONLY: built by oracle/Makefile into oracle/_build/libaac_oracle.so and
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker or
 * the timed CPU baseline.  Never linked into the product.
 *
 * It is the same algorithm as oracle/env_ref.py (which follows the reference line by line) and
 * is tested bit-identical to it; it exists because env_ref is per-agent Python and too slow to
 * check the GPU at full sizes.  Arithmetic contract (compile with -ffp-contract=off -O2):
 *   np.linalg.norm([x, y])  == sqrt(fma(y, y, x*x))   (cblas_ddot FMA tail; verified on numpy 2.2)
 *   np.dot(a, b)            == fma(a1, b1, a0*b0)
 *   GEOS Coordinate distance == sqrt(dx*dx + dy*dy)   (no FMA)
 *   np.sum over N agents    == numpy pairwise_sum (sequential below 8, 8 accumulators above)
 * Reference lines: ATT/env:2627-2713 (kinematics), :758-773 (neighbours), :1051-1170 + OM/env:
 * 1049-1148 (radar), :1285-1469 (obs), ATT/util:308-329 (tdCPA), ATT/env:2105-2618 (ss_reward),
 * ATT/main:448-462 (termination).
 * variant = 1: the randomOD_Wgru_radar env of config 4 (oracle/wgru_env_ref.py, WGRU/env:824-1054,
 * :1666-2039, :2048-2131, WGRU/ma_main:653-661): obstacle radar, 6-wide own rows with scale_vel,
 * per-agent reward against the next waypoint and the reference path.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PI_GEOS 3.14159265358979323846
#define NRAY 18

typedef struct {
    int32_t E, N, W;            /* envs, agents, waypoint capacity */
    int32_t radar_mode;         /* 0 drones, 1 obstacles, 2 combined */
    int32_t compat;             /* 1: bug-compatible observation quirks */
    int32_t team_reward;        /* 1: full_observable_critic_flag team sum (ATT/env:2602-2603) */
    int32_t episode_length;
    int32_t gw, gh;             /* occupancy grid (x-major [i*gh + j]) */
    double bound[4];
    const uint8_t *occ;         /* n_maps stacked grids [m][i*gh + j] */
    int32_t n_maps;             /* multipleMap variant: env e reads map map_idx[e] */
    int32_t variant;            /* 0 one_model_att, 1 randomOD_Wgru_radar */
    double vmax;                /* max_spd: 5 (ATT/main:150), 10 (WGRU/ma_main:409) */
} oc_cfg;

typedef struct {
    double *pos, *vel, *pre_pos, *pre_vel;   /* E*N*2 */
    double *goal;                            /* E*N*2 : goal[-1] */
    double *wp;                              /* E*N*W*2 */
    int32_t *wp_cur, *wp_cnt;                /* E*N */
    uint8_t *reach;                          /* E*N reach_target latch */
    int32_t *wall;                           /* E*N collide_wall_count */
    int32_t *step;                           /* E */
    int32_t *map_idx;                        /* E (NULL: every env on map 0) */
    double *start;                           /* E*N*2 episode start (variant 1: reference path) */
} oc_state;

/* the occupancy grid of env e (MADDPG_ownENV_randomOD_radar_multipleMap: one map per episode) */
static const uint8_t *env_occ(const oc_cfg *c, const oc_state *s, int e) {
    const int m = s->map_idx ? s->map_idx[e] : 0;
    return c->occ + (size_t)(m >= 0 && m < (c->n_maps > 0 ? c->n_maps : 1) ? m : 0) * c->gw * c->gh;
}

typedef struct {
    float *own, *radar, *nei, *reward;       /* E*N*D0, E*N*18, E*N*K*6, E*N */
    uint8_t *done, *mask, *env_done, *bbc;   /* E*N, E*N, E, E*4 */
    double *tcpa, *dcpa;                     /* optional E*N*K (current state) */
    int32_t *conf_cur, *conf_pre;            /* optional E*N */
} oc_out;

/* ------------------------------------------------------------------ tables */
static double circ_c[64], circ_s[64], nrm_c[64], nrm_s[64], ray_c[NRAY], ray_s[NRAY];
static double apothem;
static int tables_ready = 0;

static void init_tables(void) {
    if (tables_ready) return;
    double quantum = PI_GEOS / 2.0 / 16;
    double total = fabs(0.0 - 2.0 * PI_GEOS);
    int nseg = (int)(total / quantum + 0.5);
    double inc = total / nseg;
    for (int i = 0; i < 64; ++i) {
        double a = 0.0 + (double)(-1 * i) * inc;
        circ_c[i] = cos(a);
        circ_s[i] = sin(a);
        nrm_c[i] = cos((i + 0.5) * PI_GEOS / 32.0);
        nrm_s[i] = sin((i + 0.5) * PI_GEOS / 32.0);
    }
    for (int r = 0; r < NRAY; ++r) {
        double rad = (double)(20 * r) * (PI_GEOS / 180.0);   /* math.radians */
        ray_c[r] = cos(rad);
        ray_s[r] = sin(rad);
    }
    apothem = cos(PI_GEOS / 64.0);
    tables_ready = 1;
}

static inline double npnorm(double x, double y) { return sqrt(fma(y, y, x * x)); }
static inline double gdist(double ax, double ay, double bx, double by) {
    double dx = ax - bx, dy = ay - by;
    return sqrt(dx * dx + dy * dy);
}

/* ----------------------------------------------------------- GEOS shapes */
/* min/max over the vertices of LineString([p0,p1]).buffer(r) (see oracle/geos.py) */
static void fillet_ext(double px, double py, double start, double end, double r, int skip_first,
                       double *mnx, double *mxx, double *mny, double *mxy) {
    double quantum = PI_GEOS / 2.0 / 16;
    double total = fabs(start - end);
    int nseg = (int)(total / quantum + 0.5);
    double inc = total / nseg;
    for (int i = skip_first; i < nseg; ++i) {
        double a = start + (double)(-1 * i) * inc;
        double x = px + r * cos(a), y = py + r * sin(a);
        if (x < *mnx) *mnx = x;
        if (x > *mxx) *mxx = x;
        if (y < *mny) *mny = y;
        if (y > *mxy) *mxy = y;
    }
}

static void upd(double x, double y, double *mnx, double *mxx, double *mny, double *mxy) {
    if (x < *mnx) *mnx = x;
    if (x > *mxx) *mxx = x;
    if (y < *mny) *mny = y;
    if (y > *mxy) *mxy = y;
}

static int bound_crash(double x0, double y0, double x1, double y1, double r, const double *b) {
    double mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY;
    if (x0 == x1 && y0 == y1) {
        for (int i = 0; i < 64; ++i) upd(x0 + r * circ_c[i], y0 + r * circ_s[i], &mnx, &mxx, &mny, &mxy);
        /* vertex 0 is (x + r, y) exactly; circ_c[0] == 1, circ_s[0] == 0 give the same */
    } else {
        double dx = x1 - x0, dy = y1 - y0;
        double len = sqrt(dx * dx + dy * dy);
        double ux = 1 * r * dx / len, uy = 1 * r * dy / len;
        /* left offset (p0 - uy, p0 + ux) (p1 - uy, p1 + ux); right = negated u */
        upd(x1 - uy, y1 + ux, &mnx, &mxx, &mny, &mxy);      /* L.p1 */
        upd(x1 + uy, y1 - ux, &mnx, &mxx, &mny, &mxy);      /* R.p1 */
        upd(x0 + uy, y0 - ux, &mnx, &mxx, &mny, &mxy);      /* R.p0 */
        upd(x0 - uy, y0 + ux, &mnx, &mxx, &mny, &mxy);      /* L.p0 */
        double a1 = atan2(dy, dx);
        fillet_ext(x1, y1, a1 + PI_GEOS / 2.0, a1 - PI_GEOS / 2.0, r, 1, &mnx, &mxx, &mny, &mxy);
        double a0 = atan2(y0 - y1, x0 - x1);
        fillet_ext(x0, y0, a0 + PI_GEOS / 2.0, a0 - PI_GEOS / 2.0, r, 1, &mnx, &mxx, &mny, &mxy);
    }
    return (mnx <= b[0] && b[0] <= mxx) || (mnx <= b[1] && b[1] <= mxx) ||
           (mny <= b[2] && b[2] <= mxy) || (mny <= b[3] && b[3] <= mxy);
}


/* ------------------------------------------------ exact predicates (threshold bands)
 * The closed forms above use the ideal polygons (exact edge normals, apothem); GEOS decides
 * intersects / intersection exactly (DD orientation) on the ROUNDED float vertices.  Within BAND of
 * a threshold the exact formulation on those vertices decides (oracle/geos.py BAND, BAND_T; the
 * kernel does the same with floating-point expansions, csrc/aac_geom.h).  This restatement is
 * independent of the kernel's: every coordinate is scaled to an integer (x * 2^52 is one for
 * 1 <= |x| < 1024, which holds for every coordinate of the ATT / OM world) and the separating-axis
 * projections are evaluated in 128-bit integers. */
#define BAND 1e-9
#define BAND_T 1e-9

typedef __int128 i128;

static i128 iscale(double x) {
    const double a = fabs(x);
    if (!(x == 0.0 || (a >= 1.0 && a < 1024.0))) abort();      /* outside the exact domain */
    return (i128)(int64_t)ldexp(x, 52);
}

/* closed convex polygons P (np points) and Q (nq points) meet (touching counts): no edge of either
 * (nq == 2: a segment, its one axis) separates them; projections onto the edge normal in i128 */
static int convex_meet_exact(const double *px, const double *py, int np, const double *qx, const double *qy, int nq) {
    i128 PX[64], PY[64], QX[64], QY[64];
    for (int i = 0; i < np; ++i) { PX[i] = iscale(px[i]); PY[i] = iscale(py[i]); }
    for (int i = 0; i < nq; ++i) { QX[i] = iscale(qx[i]); QY[i] = iscale(qy[i]); }
    for (int side = 0; side < 2; ++side) {
        const i128 *EX = side ? QX : PX, *EY = side ? QY : PY;
        const int ne = side ? nq : np;
        for (int k = 0; k < ne; ++k) {
            const i128 vx = EX[k], vy = EY[k], wx = EX[(k + 1) % ne], wy = EY[(k + 1) % ne];
            const i128 nx = wy - vy, ny = -(wx - vx);
            i128 amin = 0, amax = 0, bmin = 0, bmax = 0;
            for (int i = 0; i < np; ++i) {
                const i128 v = nx * (PX[i] - vx) + ny * (PY[i] - vy);
                if (i == 0 || v < amin) amin = v;
                if (i == 0 || v > amax) amax = v;
            }
            for (int i = 0; i < nq; ++i) {
                const i128 v = nx * (QX[i] - vx) + ny * (QY[i] - vy);
                if (i == 0 || v < bmin) bmin = v;
                if (i == 0 || v > bmax) bmax = v;
            }
            if (amax < bmin || bmax < amin) return 0;
        }
    }
    return 1;
}

static void gon(double px, double py, double r, double *x, double *y) {
    for (int i = 0; i < 64; ++i) { x[i] = px + r * circ_c[i]; y[i] = py + r * circ_s[i]; }
}

static int goal_reached(double px, double py, double gx, double gy, double pb) {
    double dx = gx - px, dy = gy - py;
    double thr = (pb + 1.0) * apothem;
    double m = -INFINITY;
    for (int k = 0; k < 64; ++k) {
        double v = dx * nrm_c[k] + dy * nrm_s[k];
        if (v > m) m = v;
    }
    if (m > thr + BAND) return 0;
    if (m < thr - BAND) return 1;
    double ax[64], ay[64], bx[64], by[64];
    gon(px, py, pb, ax, ay);
    gon(gx, gy, 1.0, bx, by);
    return convex_meet_exact(ax, ay, 64, bx, by, 64);
}

static int building_hit(double px, double py, double cx, double cy, double pb) {
    double dx = cx - px, dy = cy - py;
    int unsure = 0;
    const double v2[2] = {fabs(dx), fabs(dy)};
    for (int q = 0; q < 2; ++q) {
        if (v2[q] > 5.0 + pb + BAND) return 0;
        if (v2[q] > 5.0 + pb - BAND) unsure = 1;
    }
    for (int k = 0; k < 32; ++k) {
        double proj = fabs(dx * nrm_c[k] + dy * nrm_s[k]);
        double lim = 5.0 * (fabs(nrm_c[k]) + fabs(nrm_s[k])) + pb * apothem;
        if (proj > lim + BAND) return 0;
        if (proj > lim - BAND) unsure = 1;
    }
    if (!unsure) return 1;
    double ax[64], ay[64];
    gon(px, py, pb, ax, ay);
    const double sx[4] = {cx - 5.0, cx - 5.0, cx + 5.0, cx + 5.0}, sy[4] = {cy - 5.0, cy + 5.0, cy + 5.0, cy - 5.0};
    return convex_meet_exact(ax, ay, 64, sx, sy, 4);
}

/* Cyrus-Beck entry of segment c->e into the clockwise 64-gon of circumradius r at (px,py); an
 * interval [tlo, thi] within BAND_T of empty (touching) is decided by the exact test */
static int ray_poly_entry(double cx, double cy, double ex, double ey, double px, double py, double r, double *tout) {
    double ddx = ex - cx, ddy = ey - cy;
    double tlo = 0.0, thi = 1.0;
    for (int k = 0; k < 64; ++k) {
        int k1 = (k + 1) & 63;
        double vx = px + r * circ_c[k], vy = py + r * circ_s[k];
        double wx = px + r * circ_c[k1], wy = py + r * circ_s[k1];
        double exx = wx - vx, eyy = wy - vy;
        double a = exx * (cy - vy) - eyy * (cx - vx);
        double b = exx * ddy - eyy * ddx;
        if (b == 0.0) {
            if (a > 0.0) return 0;
        } else if (b < 0.0) {
            double t = -a / b;
            if (t > tlo) tlo = t;
        } else {
            double t = -a / b;
            if (t < thi) thi = t;
        }
    }
    if (tlo - thi > BAND_T) return 0;
    if (tlo - thi >= -BAND_T && tlo < 1.0 - BAND_T) {      /* (a touch at t ~ 1: distance L either way) */
        double gx[64], gy[64];
        const double sx[2] = {cx, ex}, sy[2] = {cy, ey};
        gon(px, py, r, gx, gy);
        if (!convex_meet_exact(gx, gy, 64, sx, sy, 2)) return 0;
        tlo = tlo < 0.0 ? 0.0 : (tlo > 1.0 ? 1.0 : tlo);
    } else if (tlo > thi) {
        return 0;
    }
    *tout = tlo;
    return 1;
}

static int ray_square(double cx, double cy, double ex, double ey, double x0, double x1, double y0, double y1, double *dout) {
    double ddx = ex - cx, ddy = ey - cy;
    double tx0, tx1, ty0, ty1;
    /* a ray along an edge from a start point on that edge: distance 0 (OM/env:1105-1116) */
    if ((ddx == 0.0 && (cx == x0 || cx == x1) && cy >= y0 && cy <= y1) ||
        (ddy == 0.0 && (cy == y0 || cy == y1) && cx >= x0 && cx <= x1)) {
        *dout = 0.0;
        return 1;
    }
    if (ddx == 0.0) {
        if (cx < x0 || cx > x1) return 0;
        tx0 = -INFINITY; tx1 = INFINITY;
    } else {
        double ta = (x0 - cx) / ddx, tb = (x1 - cx) / ddx;
        if (ta < tb) { tx0 = ta; tx1 = tb; } else { tx0 = tb; tx1 = ta; }
    }
    if (ddy == 0.0) {
        if (cy < y0 || cy > y1) return 0;
        ty0 = -INFINITY; ty1 = INFINITY;
    } else {
        double ta = (y0 - cy) / ddy, tb = (y1 - cy) / ddy;
        if (ta < tb) { ty0 = ta; ty1 = tb; } else { ty0 = tb; ty1 = ta; }
    }
    double tin = tx0 > ty0 ? tx0 : ty0;
    double tout = tx1 < ty1 ? tx1 : ty1;
    if (fabs(tin - tout) <= BAND_T && tin < 1.0 - BAND_T) {
        /* the rounded slab quotients tie (a ray through a corner; near t = 1 the distance is L either
         * way): the segment meets the boundary iff it meets the closed square and not only the open one */
        const double qx[4] = {x0, x0, x1, x1}, qy[4] = {y0, y1, y1, y0}, sx[2] = {cx, ex}, sy[2] = {cy, ey};
        const int inside = x0 < cx && cx < x1 && y0 < cy && cy < y1 && x0 < ex && ex < x1 && y0 < ey && ey < y1;
        if (inside || !convex_meet_exact(qx, qy, 4, sx, sy, 2)) return 0;
        double t = tin >= 0.0 ? tin : tout;
        t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
        *dout = gdist(cx + t * ddx, cy + t * ddy, cx, cy);
        return 1;
    }
    if (tin > tout || tout < 0.0 || tin > 1.0) return 0;
    double t = tin >= 0.0 ? tin : tout;
    if (t > 1.0) return 0;
    *dout = gdist(cx + t * ddx, cy + t * ddy, cx, cy);
    return 1;
}

static int ray_vline(double cx, double cy, double ex, double ey, double lx, double *dout) {
    if (cx == lx && ex == lx) { *dout = 0.0; return 1; }
    if ((cx - lx) * (ex - lx) > 0.0) return 0;
    double t = (lx - cx) / (ex - cx);
    *dout = gdist(lx, cy + t * (ey - cy), cx, cy);
    return 1;
}

static int ray_hline(double cx, double cy, double ex, double ey, double ly, double *dout) {
    if (cy == ly && ey == ly) { *dout = 0.0; return 1; }
    if ((cy - ly) * (ey - ly) > 0.0) return 0;
    double t = (ly - cy) / (ey - cy);
    *dout = gdist(cx + t * (ex - cx), ly, cx, cy);
    return 1;
}

static double radar_obstacles(const oc_cfg *c, const uint8_t *occ, double cx, double cy, double ex, double ey,
                              double len) {
    double mind = len, d;
    const double *b = c->bound;
    double gx0 = ceil(b[0] / 10.0) * 10.0, gy0 = ceil(b[2] / 10.0) * 10.0;
    /* occupied cells whose square can touch the ray: centre within 15 + 5 of c (box) */
    int i0 = (int)floor((cx - 20.0 - gx0) / 10.0), i1 = (int)ceil((cx + 20.0 - gx0) / 10.0);
    int j0 = (int)floor((cy - 20.0 - gy0) / 10.0), j1 = (int)ceil((cy + 20.0 - gy0) / 10.0);
    if (i0 < 0) i0 = 0;
    if (j0 < 0) j0 = 0;
    if (i1 > c->gw - 1) i1 = c->gw - 1;
    if (j1 > c->gh - 1) j1 = c->gh - 1;
    for (int i = i0; i <= i1; ++i)
        for (int j = j0; j <= j1; ++j) {
            if (!occ[i * c->gh + j]) continue;
            double qx = gx0 + 10.0 * i, qy = gy0 + 10.0 * j;
            if (ray_square(cx, cy, ex, ey, qx - 5.0, qx + 5.0, qy - 5.0, qy + 5.0, &d) && d <= mind) mind = d;
        }
    if (ray_vline(cx, cy, ex, ey, b[0], &d) && d < mind) mind = d;
    if (ray_vline(cx, cy, ex, ey, b[1], &d) && d < mind) mind = d;
    if (ray_hline(cx, cy, ex, ey, b[2], &d) && d < mind) mind = d;
    if (ray_hline(cx, cy, ex, ey, b[3], &d) && d < mind) mind = d;
    return mind;
}

static double pairwise_sum(const double *a, int n) {
    if (n < 8) {
        double s = a[0];
        for (int i = 1; i < n; ++i) s += a[i];
        return s;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

/* ------------------------------------------------------------ tdCPA (util:308-329) */
static void tdcpa(double ox, double oy, double hx, double hy, double ovx, double ovy, double hvx, double hvy,
                  double pb, double *tcpa, double *dcpa, int *total) {
    double rx = -1 * (ox - hx), ry = -1 * (oy - hy);
    double wx = ovx - hvx, wy = ovy - hvy;
    double nw = npnorm(wx, wy);
    double sq = nw * nw;
    double t, d;
    if (sq == 0) {
        t = -10;
        double nnx = ox + ovx * 1, nny = oy + ovy * 1;
        double nhx = hx + hvx * 1, nhy = hy + hvy * 1;
        d = npnorm(nhx - nnx, nhy - nny);
        if (d < pb + pb) *total += 1;
    } else {
        t = fma(ry, wy, rx * wx) / sq;
        d = npnorm((rx * -1) + (wx * t), (ry * -1) + (wy * t));
    }
    if (t <= 1 && t >= 0 && d < pb + pb) *total += 1;
    *tcpa = t;
    *dcpa = d;
}

/* ------------------------------------------------------------ observation (env:837-1493) */
/* rmin (variant 1, may be NULL): per agent, the smallest radar distance in float64 */
static void observe_env(const oc_cfg *c, oc_state *s, oc_out *o, int e, double *rmin) {
    const int N = c->N, K = N - 1, D0 = c->variant ? 6 : 6 + 4 * K;
    const double *b = c->bound;
    const double XS = (1.0 - (-1.0)) / (b[1] - b[0]), YS = (1.0 - (-1.0)) / (b[3] - b[2]);
    const double pb = 2.5, vmax = c->vmax;
    for (int i = 0; i < N; ++i) {
        size_t ai = (size_t)e * N + i;
        double px = s->pos[2 * ai], py = s->pos[2 * ai + 1];
        double vx = s->vel[2 * ai], vy = s->vel[2 * ai + 1];
        float *own = o->own + ai * D0;
        double npx = -1 + (px - b[0]) * XS, npy = -1 + (py - b[2]) * YS;
        double gx = s->goal[2 * ai], gy = s->goal[2 * ai + 1];
        double ngx = 2 * ((gx - b[0]) / (b[1] - b[0])) - 1, ngy = 2 * ((gy - b[2]) / (b[3] - b[2])) - 1;
        own[0] = (float)npx; own[1] = (float)npy;
        if (c->variant) { own[2] = (float)(XS * vx); own[3] = (float)(YS * vy); }   /* scale_vel */
        else { own[2] = (float)(vx / vmax); own[3] = (float)(vy / vmax); }
        own[4] = (float)(ngx - npx); own[5] = (float)(ngy - npy);
        int kk = 0, cc = 0, cp = 0;
        for (int j = 0; j < N; ++j) {
            if (j == i) continue;
            size_t aj = (size_t)e * N + j;
            double qx = s->pos[2 * aj], qy = s->pos[2 * aj + 1];
            double wx = s->vel[2 * aj], wy = s->vel[2 * aj + 1];
            double dx = qx - px, dy = qy - py;
            if (!c->variant) {
                if (c->compat) {
                    own[6 + 4 * kk] = (float)(-1 + (dx - b[0]) * XS);
                    own[7 + 4 * kk] = (float)(-1 + (dy - b[2]) * YS);
                } else {
                    own[6 + 4 * kk] = (float)(XS * dx);
                    own[7 + 4 * kk] = (float)(YS * dy);
                }
                own[8 + 4 * kk] = (float)(wx / vmax);
                own[9 + 4 * kk] = (float)(wy / vmax);
            }
            float *nb = o->nei + (ai * K + kk) * 6;
            double dxm = b[0] - b[1], dxM = b[1] - b[0], dym = b[2] - b[3], dyM = b[3] - b[2];
            nb[0] = (float)(2 * ((dx - dxm) / (dxM - dxm)) - 1);
            nb[1] = (float)(2 * ((dy - dym) / (dyM - dym)) - 1);
            double g0, g1;
            if (c->compat) { g0 = wy - qx; g1 = pb - qy; }
            else { g0 = s->goal[2 * aj] - qx; g1 = s->goal[2 * aj + 1] - qy; }
            nb[2] = (float)(2 * ((g0 - dxm) / (dxM - dxm)) - 1);
            nb[3] = (float)(2 * ((g1 - dym) / (dyM - dym)) - 1);
            nb[4] = (float)(wx / vmax);
            nb[5] = (float)(wy / vmax);
            double t, d;
            tdcpa(qx, qy, px, py, wx, wy, vx, vy, pb, &t, &d, &cc);
            if (o->tcpa) { o->tcpa[ai * K + kk] = t; o->dcpa[ai * K + kk] = d; }
            double t2, d2;
            tdcpa(s->pre_pos[2 * aj], s->pre_pos[2 * aj + 1], s->pre_pos[2 * ai], s->pre_pos[2 * ai + 1],
                  s->pre_vel[2 * aj], s->pre_vel[2 * aj + 1], s->pre_vel[2 * ai], s->pre_vel[2 * ai + 1], pb, &t2, &d2, &cp);
            ++kk;
        }
        if (o->conf_cur) { o->conf_cur[ai] = cc; o->conf_pre[ai] = cp; }
        /* radar */
        double rm = INFINITY;
        for (int r = 0; r < NRAY; ++r) {
            double ex = px + 15.0 * ray_c[r], ey = py + 15.0 * ray_s[r];
            double len = gdist(ex, ey, px, py);
            double dd = len, dob = len;
            if (c->radar_mode != 1) {
                double shortest = INFINITY;
                for (int j = 0; j < N; ++j) {
                    if (j == i) continue;
                    size_t aj = (size_t)e * N + j;
                    double t;
                    if (!ray_poly_entry(px, py, ex, ey, s->pos[2 * aj], s->pos[2 * aj + 1], pb, &t)) continue;
                    double ix = px + t * (ex - px), iy = py + t * (ey - py);
                    double d = gdist(ix, iy, px, py);
                    if (d < shortest) { shortest = d; dd = d; }
                }
            }
            if (c->radar_mode != 0) dob = radar_obstacles(c, env_occ(c, s, e), px, py, ex, ey, len);
            double v = c->radar_mode == 0 ? dd : (c->radar_mode == 1 ? dob : (dd < dob ? dd : dob));
            o->radar[ai * NRAY + r] = (float)v;
            if (v < rm) rm = v;
        }
        if (rmin) rmin[i] = rm;
    }
}

/* ------------------------------------------------ GEOS point -> LineString (oracle/geos.py) */
static double point_to_segment(double px, double py, double ax, double ay, double bx, double by) {
    if (ax == bx && ay == by) return gdist(px, py, ax, ay);
    double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
    double r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
    if (r <= 0.0) return gdist(px, py, ax, ay);
    if (r >= 1.0) return gdist(px, py, bx, by);
    double sv = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
    return fabs(sv) * sqrt(len2);
}

static void segment_closest_point(double px, double py, double ax, double ay, double bx, double by, double *qx,
                                  double *qy) {
    double f;
    if (px == ax && py == ay) f = 0.0;
    else if (px == bx && py == by) f = 1.0;
    else {
        double dx = bx - ax, dy = by - ay;
        f = ((px - ax) * dx + (py - ay) * dy) / (dx * dx + dy * dy);
    }
    if (f > 0 && f < 1) { *qx = ax + f * (bx - ax); *qy = ay + f * (by - ay); return; }
    double d0 = gdist(ax, ay, px, py), d1 = gdist(bx, by, px, py);
    if (d0 < d1) { *qx = ax; *qy = ay; } else { *qx = bx; *qy = by; }
}

/* cross_track_error(point, ref_line)[0] (WGRU/env:2621-2632); the path is start, wp[0..n) */
static double cross_track(double px, double py, const double *start, const double *wp, int n) {
    double best = INFINITY, nx = 0.0, ny = 0.0, ax = start[0], ay = start[1];
    for (int k = 0; k < n; ++k) {
        double bx = wp[2 * k], by = wp[2 * k + 1];
        double d = point_to_segment(px, py, ax, ay, bx, by);
        if (d < best) { best = d; segment_closest_point(px, py, ax, ay, bx, by, &nx, &ny); }
        if (best <= 0.0) break;
        ax = bx; ay = by;
    }
    return gdist(px, py, nx, ny);
}

/* WGRU ss_reward of agent ai (WGRU/env:1666-2039); returns the reward, sets the outputs */
static double wgru_reward(const oc_cfg *c, oc_state *s, int e, int i, double rmin, int ncoll, int building,
                          int *done_out, int *cg_out, uint8_t *mask_out, uint8_t *bbc) {
    const int N = c->N;
    const double pb = 2.5;
    size_t ai = (size_t)e * N + i;
    double px = s->pos[2 * ai], py = s->pos[2 * ai + 1];
    double gx = s->goal[2 * ai], gy = s->goal[2 * ai + 1];
    int goal = goal_reached(px, py, gx, gy, pb);
    /* the next waypoint: remaining goal list = waypoints not flagged in wp_cur (bit k) */
    const double *wp = s->wp + (size_t)ai * c->W * 2;
    const int cnt = s->wp_cnt[ai];
    uint32_t rm = (uint32_t)s->wp_cur[ai];
    int nrem = 0;
    for (int k = 0; k < cnt; ++k) nrem += !((rm >> k) & 1u);
    double smallest = INFINITY, nx = 0.0, ny = 0.0;
    int flag = 0;
    for (int k = 0; k < cnt; ++k) {
        if ((rm >> k) & 1u) continue;
        double d = gdist(px, py, wp[2 * k], wp[2 * k + 1]);
        if (d < smallest) {
            smallest = d;
            nx = wp[2 * k]; ny = wp[2 * k + 1];
            if (smallest < 5) {
                flag = 1;
                if (nrem > 1) {
                    rm |= 1u << k;
                    --nrem;
                    double best = INFINITY;
                    for (int q = 0; q < cnt; ++q) {
                        if ((rm >> q) & 1u) continue;
                        double dd = gdist(wp[2 * q], wp[2 * q + 1], px, py);
                        if (dd < best) { best = dd; nx = wp[2 * q]; ny = wp[2 * q + 1]; }
                    }
                }
                break;
            }
        }
    }
    s->wp_cur[ai] = (int32_t)rm;
    for (int k = cnt - 1; k >= 0; --k)         /* goal[-1] after the pop */
        if (!((rm >> k) & 1u)) { s->goal[2 * ai] = wp[2 * k]; s->goal[2 * ai + 1] = wp[2 * k + 1]; break; }
    double before = npnorm(s->pre_pos[2 * ai] - nx, s->pre_pos[2 * ai + 1] - ny);
    double after = npnorm(px - nx, py - ny);
    double dtg = 1 * (before - after);
    double cross = cross_track(px, py, s->start + 2 * ai, wp, cnt);
    double dref;
    if (cross <= pb) { double m = (0 - 1) / (pb - 0); dref = 3 * (m * cross + 1); }
    else dref = -3 * 1;
    double thr = 2 * pb;
    double sp = npnorm(s->vel[2 * ai], s->vel[2 * ai + 1]);
    double clip = sp < 0 ? 0 : (sp > thr ? thr : sp);
    double ssp = 3 * ((thr - clip) * (1.0 / thr));
    double m2 = (0 - 1) / (5 - pb);
    double nbp = (rmin >= pb && rmin <= 5) ? 3 * (m2 * rmin + 2) : 0;
    int bnd = bound_crash(s->pre_pos[2 * ai], s->pre_pos[2 * ai + 1], px, py, pb, c->bound);
    uint8_t m = (uint8_t)(bnd | ((ncoll > 0) << 1) | (goal << 2) | (building << 3) | (flag << 4));
    int done = 0, cg = 0;
    double r;
    if (bnd) {
        r = (((((0.0 + dref) - 5) + dtg) - ssp) + 0.0) - nbp;
        done = 1; bbc[0] = 1;
    } else if (building) {
        done = 1; bbc[1] = 1;
        r = (((((0.0 + dref) - 5) + dtg) - ssp) + 0.0) - nbp;
    } else if (goal) {
        cg = 1; s->reach[ai] = 1;
        r = (0.0 + 5) + 0.0;
    } else {
        r = 0.0;
        if (flag && nrem > 1) r = r + 3;
        r = (((((r + dref) + dtg) - ssp) + 0.0) - nbp) + 0.0;
    }
    if (cg) m |= 32;
    *done_out = done; *cg_out = cg; *mask_out = m;
    return r;
}

/* ------------------------------------------------------------ step (env:2627 + ss_reward) */
void oc_step(const oc_cfg *c, oc_state *s, const float *act, oc_out *o) {
    init_tables();
    const int N = c->N, E = c->E;
    const double *b = c->bound;
    const double pb = 2.5, vmax = c->vmax, dt = 0.5;
    double rew[64], rmin[64];
    for (int e = 0; e < E; ++e) {
        /* a1 kinematics */
        for (int i = 0; i < N; ++i) {
            size_t ai = (size_t)e * N + i;
            s->pre_pos[2 * ai] = s->pos[2 * ai];
            s->pre_pos[2 * ai + 1] = s->pos[2 * ai + 1];
            s->pre_vel[2 * ai] = s->vel[2 * ai];
            s->pre_vel[2 * ai + 1] = s->vel[2 * ai + 1];
            double ax = (double)act[2 * ai] * 8, ay = (double)act[2 * ai + 1] * 8;
            double cvx = s->vel[2 * ai] + ax * dt, cvy = s->vel[2 * ai + 1] + ay * dt;
            double nh = atan2(cvy, cvx);
            if (npnorm(cvx, cvy) >= vmax) {
                s->vel[2 * ai] = vmax * cos(nh);
                s->vel[2 * ai + 1] = vmax * sin(nh);
            } else {
                s->vel[2 * ai] = cvx;
                s->vel[2 * ai + 1] = cvy;
            }
            s->pos[2 * ai] = s->pos[2 * ai] + s->vel[2 * ai] * dt;
            s->pos[2 * ai + 1] = s->pos[2 * ai + 1] + s->vel[2 * ai + 1] * dt;
        }
        observe_env(c, s, o, e, c->variant ? rmin : NULL);
        /* ss_reward */
        uint8_t bbc[4] = {0, 0, 0, 0};
        int all_goal = 1, any_done = 0, all_reach = 1;
        const double c_drone = 1 + (2.5 / (10 - 2.5)), m_drone = (0 - 1) / (10 - 2.5);
        for (int i = 0; i < N; ++i) {
            size_t ai = (size_t)e * N + i;
            double px = s->pos[2 * ai], py = s->pos[2 * ai + 1];
            int ncoll = 0, last_coll = -1, nearest = -1;
            double shortest = INFINITY, dist[64];
            int nd = 0;
            for (int j = 0; j < N; ++j) {
                if (j == i) continue;
                size_t aj = (size_t)e * N + j;
                double d = npnorm(px - s->pos[2 * aj], py - s->pos[2 * aj + 1]);
                dist[nd++] = d;
                if (d < shortest) { shortest = d; nearest = j; }
                if (d <= pb * 2) { ++ncoll; last_coll = j; }
            }
            int building = 0;
            {
                double gx0 = ceil(b[0] / 10.0) * 10.0, gy0 = ceil(b[2] / 10.0) * 10.0;
                int ci = (int)floor((px - gx0) / 10.0 + 0.5), cj = (int)floor((py - gy0) / 10.0 + 0.5);
                for (int ii = ci - 1; ii <= ci + 1 && !building; ++ii)
                    for (int jj = cj - 1; jj <= cj + 1; ++jj) {
                        if (ii < 0 || jj < 0 || ii >= c->gw || jj >= c->gh) continue;
                        if (!env_occ(c, s, e)[ii * c->gh + jj]) continue;
                        if (building_hit(px, py, gx0 + 10.0 * ii, gy0 + 10.0 * jj, pb)) { building = 1; break; }
                    }
            }
            if (building) s->wall[ai] += 1;
            if (c->variant) {
                int done, cg;
                uint8_t m;
                rew[i] = wgru_reward(c, s, e, i, rmin[i], ncoll, building, &done, &cg, &m, bbc);
                o->done[ai] = (uint8_t)done;
                o->mask[ai] = m;
                any_done |= done;
                all_goal &= cg;
                all_reach &= s->reach[ai];
                continue;
            }
            double gx = s->goal[2 * ai], gy = s->goal[2 * ai + 1];
            int goal = goal_reached(px, py, gx, gy, pb);
            int cur = s->wp_cur[ai];
            const double *w0 = s->wp + ((size_t)ai * c->W + cur) * 2;
            int wpf = gdist(px, py, w0[0], w0[1]) < 5;
            double before = npnorm(s->pre_pos[2 * ai] - gx, s->pre_pos[2 * ai + 1] - gy);
            double after = npnorm(px - gx, py - gy);
            double dtg = (1 * (before - after)) / 5;
            double pen = 0;
            for (int k = 0; k < nd; ++k)
                if (dist[k] >= 2.5 && dist[k] <= 10) pen = pen + (1 * (m_drone * shortest + c_drone));
                else pen = pen + 0;
            int bnd = bound_crash(s->pre_pos[2 * ai], s->pre_pos[2 * ai + 1], px, py, pb, b);
            uint8_t m = (uint8_t)(bnd | ((ncoll > 0) << 1) | (goal << 2) | (building << 3) | (wpf << 4));
            int done = 0, cg = 0;
            double r;
            if (bnd) { r = ((0.0 - 20) - 0.0) - 0; done = 1; bbc[0] = 1; }
            else if (ncoll > 0) { r = ((0.0 - 20) - 0.0) - pen; done = 1; bbc[2] = 1; if (last_coll == nearest) bbc[3] = 1; }
            else if (goal) { r = (0.0 + 20) + 0.0; cg = 1; s->reach[ai] = 1; }
            else {
                if (wpf && s->wp_cnt[ai] - cur > 1) s->wp_cur[ai] = cur + 1;
                r = dtg - pen;
            }
            if (cg) m |= 32;
            rew[i] = r;
            o->done[ai] = (uint8_t)done;
            o->mask[ai] = m;
            any_done |= done;
            all_goal &= cg;
            all_reach &= s->reach[ai];
        }
        double team = pairwise_sum(rew, N);
        for (int i = 0; i < N; ++i) o->reward[(size_t)e * N + i] = (float)(c->team_reward ? team : rew[i]);
        for (int q = 0; q < 4; ++q) o->bbc[4 * e + q] = bbc[q];
        s->step[e] += 1;
        o->env_done[e] = (uint8_t)((c->episode_length < s->step[e]) || any_done || all_goal || all_reach);
    }
}

/* reset selected envs to the given OD and write their observation (env:199-405) */
void oc_reset(const oc_cfg *c, oc_state *s, const uint8_t *env_mask, const double *start, const double *wps,
              const int32_t *wp_cnt, const int32_t *map_idx, oc_out *o) {
    init_tables();
    const int N = c->N;
    for (int e = 0; e < c->E; ++e) {
        if (env_mask && !env_mask[e]) continue;
        for (int i = 0; i < N; ++i) {
            size_t ai = (size_t)e * N + i;
            s->pos[2 * ai] = s->pre_pos[2 * ai] = start[2 * ai];
            s->pos[2 * ai + 1] = s->pre_pos[2 * ai + 1] = start[2 * ai + 1];
            if (s->start) { s->start[2 * ai] = start[2 * ai]; s->start[2 * ai + 1] = start[2 * ai + 1]; }
            s->vel[2 * ai] = s->vel[2 * ai + 1] = 0.0;
            s->pre_vel[2 * ai] = s->pre_vel[2 * ai + 1] = 0.0;
            int n = wp_cnt[ai];
            s->wp_cnt[ai] = n;
            s->wp_cur[ai] = 0;
            memcpy(s->wp + (size_t)ai * c->W * 2, wps + (size_t)ai * c->W * 2, sizeof(double) * 2 * c->W);
            s->goal[2 * ai] = wps[((size_t)ai * c->W + n - 1) * 2];
            s->goal[2 * ai + 1] = wps[((size_t)ai * c->W + n - 1) * 2 + 1];
            s->reach[ai] = 0;
            s->wall[ai] = 0;
        }
        s->step[e] = 0;
        if (s->map_idx) s->map_idx[e] = map_idx ? map_idx[e] : 0;
        observe_env(c, s, o, e, NULL);
    }
}

/* observation only (no state change) */
void oc_observe(const oc_cfg *c, oc_state *s, oc_out *o) {
    init_tables();
    for (int e = 0; e < c->E; ++e) observe_env(c, s, o, e, NULL);
}

/* building / bound / goal predicate probes for tests */
int oc_bound_crash(double x0, double y0, double x1, double y1, const double *bound) {
    init_tables();
    return bound_crash(x0, y0, x1, y1, 2.5, bound);
}
int oc_goal_reached(double px, double py, double gx, double gy) {
    init_tables();
    return goal_reached(px, py, gx, gy, 2.5);
}
int oc_building_hit(double px, double py, double cx, double cy) {
    init_tables();
    return building_hit(px, py, cx, cy, 2.5);
}

/* cross-track probe for tests (variant 1 reference-path distance) */
double oc_cross_track(double px, double py, const double *start, const double *wp, int n) {
    return cross_track(px, py, start, wp, n);
}
