// aac_geom.h -- GEOS-shape geometry shared by the gfx950 environment kernels (aac_env.hip,
// aac_uam.hip).  Each translation unit that includes it owns a private copy of ``c_tab`` and
// uploads it with fill_tables() + hipMemcpyToSymbol at create time.
//
// The shapes are the ones shapely 2.0.1 / GEOS 3.11 builds with quad_segs = 16: Point.buffer is the
// 64-gon of createCircle (vertex angles -i 2pi/64), LineString.buffer the round-capped capsule of
// computeLineBufferCurve / addDirectedFillet.  Predicates are closed forms exact in real arithmetic
// for those convex shapes, evaluated in the operation order of the C oracle (oracle/aac_oracle.c,
// oracle/uam_ref.py); compile with -ffp-contract=off.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#ifndef NRAY
#define NRAY 18
#endif

namespace {

struct Tab {
    double circ_c[64], circ_s[64];   // GEOS createCircle unit vectors, angle 0 - i*inc
    double nrm_c[64], nrm_s[64];     // 64-gon edge normals, angle (k + 1/2) pi/32
    double ray_c[NRAY], ray_s[NRAY]; // cos/sin(math.radians(20 r))
    double apothem;                  // cos(pi/64)
    double quantum;                  // GEOS filletAngleQuantum = pi/2/16
    double cos_quantum;              // cos(quantum): bound on a fillet arc's reach along an axis
};

__constant__ Tab c_tab;

constexpr double PI_GEOS = 3.14159265358979323846;

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ inline double npnorm(double x, double y) { return sqrt(__builtin_fma(y, y, x * x)); }
__device__ inline double gdist(double ax, double ay, double bx, double by) {
    double dx = ax - bx, dy = ay - by;
    return sqrt(dx * dx + dy * dy);
}

// ------------------------------------------------------------------ GEOS-shape predicates
__device__ inline void upd(double x, double y, double &mnx, double &mxx, double &mny, double &mxy) {
    mnx = x < mnx ? x : mnx;
    mxx = x > mxx ? x : mxx;
    mny = y < mny ? y : mny;
    mxy = y > mxy ? y : mxy;
}

// One extreme (axis ax = 0 x / 1 y; the max when mx, else the min) over the vertices i = 1 .. nseg-1
// that GEOS's fillet (OffsetSegmentGenerator::addDirectedFillet, oracle/aac_oracle.c fillet_ext) has: p + r (cos a_i, sin a_i), a_i = start - i inc.  The extreme of cos(a - theta)
// over equally spaced angles sits at the vertex nearest theta (theta = 0, pi, pi/2, -pi/2), or at an
// arc end when theta is off the arc; neighbours of the winner are smaller by >= r inc^2 (~0.02 at
// r = 2.5), far above rounding.  So the three vertices around theta plus the two arc ends hold
// the extreme of the computed values: the same number as the full loop with 5 instead of 31
// fp64 cos/sin pairs per fillet.
__device__ double fillet_extreme(double px, double py, double start, double end, double r, int ax, bool mx) {
    const double total = fabs(start - end);
    const int nseg = (int)(total / c_tab.quantum + 0.5);
    double best = mx ? -INFINITY : INFINITY;
    if (nseg < 2) return best;
    const double inc = total / nseg;
    const double theta = ax == 0 ? (mx ? 0.0 : PI_GEOS) : (mx ? PI_GEOS / 2.0 : -PI_GEOS / 2.0);
    const double per = 2.0 * PI_GEOS / inc;                  // vertices per turn
    double k = (start - theta) / inc;                         // a_i = theta at i = k (mod per)
    k -= per * floor(k / per);
    const int kn = (int)floor(k + 0.5), iper = (int)floor(per + 0.5);
    const int cand[5] = {1, nseg - 1, kn - 1, kn, kn + 1};
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        int i = cand[q] % iper;
        i = i < 0 ? i + iper : i;
        if (i < 1 || i > nseg - 1) continue;
        const double a = start + (double)(-1 * i) * inc;
        const double v = ax == 0 ? px + r * cos(a) : py + r * sin(a);
        best = mx ? (v > best ? v : best) : (v < best ? v : best);
    }
    return best;
}

// LineString([p0,p1]).buffer(r, round caps) meets one of the 4 infinite lines x = b[0], x = b[1],
// y = b[2], y = b[3] (ATT/env:2507, UAM/env:4488-4491)
__device__ bool capsule_crash(double r, const double *b, double x0, double y0, double x1, double y1) {
    // every capsule vertex lies within r (1 + 1e-15) of p0 or p1: cheap exact pre-filter
    const double m = r + 1e-6;
    double lx = fmin(x0, x1), hx = fmax(x0, x1), ly = fmin(y0, y1), hy = fmax(y0, y1);
    if (lx - m > b[0] && hx + m < b[1] && ly - m > b[2] && hy + m < b[3]) return false;
    // Certain bands: every capsule vertex is within r of an endpoint, and the arc around the
    // extreme endpoint has a vertex within half a fillet step (<= quantum) of each axis
    // direction, so min x lies in [lx - r, lx - r cos(quantum)] (likewise the other sides).  A
    // line outside [min, max] of those bands is decided without building the capsule.
    const double lo = r + 1e-9, hi = r * c_tab.cos_quantum - 1e-9;
    const double mn_lo[2] = {lx - lo, ly - lo}, mn_hi[2] = {lx - hi, ly - hi};
    const double mx_lo[2] = {hx + hi, hy + hi}, mx_hi[2] = {hx + lo, hy + lo};
    int need = 0;             // bit 2q: line q needs the min of its axis, bit 2q+1: the max
    for (int q = 0; q < 4; ++q) {
        const int ax = q >> 1;
        const double v = b[q];
        if (v < mn_lo[ax] || v > mx_hi[ax]) continue;                  // certainly outside
        if (v >= mn_hi[ax] && v <= mx_lo[ax]) return true;             // certainly inside
        // uncertain: v lies in the min band (then v <= max is certain) or in the max band
        need |= (v < mn_hi[ax] ? 1 : 2) << (2 * q);
    }
    if (!need) return false;
    if (x0 == x1 && y0 == y1) {
        double mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY;
        for (int i = 0; i < 64; ++i) upd(x0 + r * c_tab.circ_c[i], y0 + r * c_tab.circ_s[i], mnx, mxx, mny, mxy);
        return (mnx <= b[0] && b[0] <= mxx) || (mnx <= b[1] && b[1] <= mxx) || (mny <= b[2] && b[2] <= mxy) ||
               (mny <= b[3] && b[3] <= mxy);
    }
    // the offset-segment vertices, then per uncertain line only the extreme it needs from the two
    // fillets (fillet_extreme): the full construction's vertex set restricted to its argmax
    double ox[2], oy[2];                 // (min, max) over the four offset points
    const double dx = x1 - x0, dy = y1 - y0;
    const double len = sqrt(dx * dx + dy * dy);
    const double ux = 1 * r * dx / len, uy = 1 * r * dy / len;
    {
        double mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY;
        upd(x1 - uy, y1 + ux, mnx, mxx, mny, mxy);
        upd(x1 + uy, y1 - ux, mnx, mxx, mny, mxy);
        upd(x0 + uy, y0 - ux, mnx, mxx, mny, mxy);
        upd(x0 - uy, y0 + ux, mnx, mxx, mny, mxy);
        ox[0] = mnx; ox[1] = mxx; oy[0] = mny; oy[1] = mxy;
    }
    const double a1 = atan2(dy, dx);
    const double a0 = atan2(y0 - y1, x0 - x1);
    for (int q = 0; q < 4; ++q) {
        const int w = (need >> (2 * q)) & 3;
        if (!w) continue;
        const int ax = q >> 1;
        const bool mx = w == 2;
        double e = ax == 0 ? ox[mx] : oy[mx];
        const double f1 = fillet_extreme(x1, y1, a1 + PI_GEOS / 2.0, a1 - PI_GEOS / 2.0, r, ax, mx);
        const double f0 = fillet_extreme(x0, y0, a0 + PI_GEOS / 2.0, a0 - PI_GEOS / 2.0, r, ax, mx);
        e = mx ? fmax(e, fmax(f1, f0)) : fmin(e, fmin(f1, f0));
        if (mx ? b[q] <= e : e <= b[q]) return true;
    }
    return false;
}

// GEOS 64-gon(p, r0) vs 64-gon(q, r1), d = q - p: both share the vertex angles k pi/32, so the
// Minkowski difference is the 64-gon of circumradius R = r0 + r1 and the shapes meet iff
// max_k d.n_k <= R cos(pi/64) (touching counts); ``strict``: interiors overlap, i.e. GEOS
// ``intersects and not touches`` (max_k d.n_k < R cos(pi/64)).  ATT/env:2266-2269 (goal),
// UAM/env:3933-3936, UAM/util:41-51, :291-297.
__device__ bool gons_meet(double dx, double dy, double R, bool strict) {
    const double thr = R * c_tab.apothem;
    // max_k d.n_k lies in [|d| cos(pi/64), |d|]: outside the band the answer is certain
    const double dist = sqrt(dx * dx + dy * dy);
    if (dist > R * (1.0 + 1e-12) + 1e-12) return false;
    if (dist < thr * (1.0 - 1e-12) - 1e-12) return true;
    double m = -INFINITY;
#pragma unroll 8
    for (int k = 0; k < 64; ++k) {
        double v = dx * c_tab.nrm_c[k] + dy * c_tab.nrm_s[k];
        m = v > m ? v : m;
    }
    return strict ? m < thr : m <= thr;
}

// Cyrus-Beck entry of segment c->e into the clockwise GEOS 64-gon of radius r at p
__device__ bool ray_poly_entry_full(double cx, double cy, double ex, double ey, double px, double py, double r,
                                    double &tout) {
    double ddx = ex - cx, ddy = ey - cy;
    double tlo = 0.0, thi = 1.0;
    double vx = px + r * c_tab.circ_c[0], vy = py + r * c_tab.circ_s[0];
    for (int k = 0; k < 64; ++k) {
        int k1 = (k + 1) & 63;
        double wx = px + r * c_tab.circ_c[k1], wy = py + r * c_tab.circ_s[k1];
        double exx = wx - vx, eyy = wy - vy;
        double a = exx * (cy - vy) - eyy * (cx - vx);
        double b = exx * ddy - eyy * ddx;
        if (b == 0.0) {
            if (a > 0.0) return false;
        } else if (b < 0.0) {
            double t = -a / b;
            tlo = t > tlo ? t : tlo;
        } else {
            double t = -a / b;
            thi = t < thi ? t : thi;
        }
        if (tlo > thi) return false;
        vx = wx;
        vy = wy;
    }
    tout = tlo;
    return true;
}

// Same result from a window of edges.  When the line crosses the inscribed circle (not near
// tangency) and c lies outside the circumscribed circle, the entry is the maximum of -a/b over
// the entering edges and every entering edge other than the one(s) holding the entry point
// gives a smaller value; that edge lies within half an edge of the ray's entry angle on the
// circumscribed circle, so the maximum over the six edges around it is the same number (same
// vertices, same arithmetic) as over all 64.  The exit lies beyond the entry, so the segment
// meets the polygon iff that maximum is <= 1.  Anything else takes the full clip.
__device__ bool ray_poly_entry(double cx, double cy, double ex, double ey, double px, double py, double r,
                               double &tout) {
    const double ddx = ex - cx, ddy = ey - cy;
    const double L2 = ddx * ddx + ddy * ddy;
    const double wx = px - cx, wy = py - cy;
    const double w2 = wx * wx + wy * wy;
    const double L = sqrt(L2);
    const double s0 = (wx * ddx + wy * ddy) / L;                   // along the ray
    const double h = fabs(wx * ddy - wy * ddx) / L;               // distance of p to the line
    const double ap = r * c_tab.apothem;
    // c strictly inside the inscribed circle (margin far above rounding): every edge has a < 0,
    // so the full clip never raises tlo from 0 and never empties the interval -- entry at c
    if (w2 < ap * ap * (1.0 - 1e-9)) {
        tout = 0.0;
        return true;
    }
    if (!(h < ap * (1.0 - 1e-9)) || !(w2 > r * r * (1.0 + 1e-9)) || !(s0 > 0.0))
        return ray_poly_entry_full(cx, cy, ex, ey, px, py, r, tout);
    const double tc = (s0 - sqrt(r * r - h * h)) / L;              // circumscribed-circle entry
    const float phi = atan2f((float)(cy + tc * ddy - py), (float)(cx + tc * ddx - px));
    // vertex angles are -i 2pi/64: nearest vertex index
    int i0 = (int)lrintf(-phi * (64.0f / 6.28318530717958647f));
    double tlo = 0.0;
    bool any = false;
#pragma unroll
    for (int dk = -3; dk <= 2; ++dk) {
        const int k = (i0 + dk) & 63, k1 = (k + 1) & 63;
        const double vx = px + r * c_tab.circ_c[k], vy = py + r * c_tab.circ_s[k];
        const double qx = px + r * c_tab.circ_c[k1], qy = py + r * c_tab.circ_s[k1];
        const double exx = qx - vx, eyy = qy - vy;
        const double a = exx * (cy - vy) - eyy * (cx - vx);
        const double b = exx * ddy - eyy * ddx;
        if (b < 0.0) {
            const double t = -a / b;
            tlo = t > tlo ? t : tlo;
            any = true;
        }
    }
    if (!any) return ray_poly_entry_full(cx, cy, ex, ey, px, py, r, tout);
    if (tlo > 1.0) return false;
    tout = tlo;
    return true;
}

__device__ bool ray_square(double cx, double cy, double ex, double ey, double x0, double x1, double y0, double y1,
                           double &dout) {
    double ddx = ex - cx, ddy = ey - cy;
    double tx0, tx1, ty0, ty1;
    // a ray running along an edge from a start point on that edge: the intersection with the
    // boundary is a segment through c, so the distance is 0 (GEOS line.intersection(boundary))
    if ((ddx == 0.0 && (cx == x0 || cx == x1) && cy >= y0 && cy <= y1) ||
        (ddy == 0.0 && (cy == y0 || cy == y1) && cx >= x0 && cx <= x1)) {
        dout = 0.0;
        return true;
    }
    if (ddx == 0.0) {
        if (cx < x0 || cx > x1) return false;
        tx0 = -INFINITY;
        tx1 = INFINITY;
    } else {
        double ta = (x0 - cx) / ddx, tb = (x1 - cx) / ddx;
        if (ta < tb) { tx0 = ta; tx1 = tb; } else { tx0 = tb; tx1 = ta; }
    }
    if (ddy == 0.0) {
        if (cy < y0 || cy > y1) return false;
        ty0 = -INFINITY;
        ty1 = INFINITY;
    } else {
        double ta = (y0 - cy) / ddy, tb = (y1 - cy) / ddy;
        if (ta < tb) { ty0 = ta; ty1 = tb; } else { ty0 = tb; ty1 = ta; }
    }
    double tin = tx0 > ty0 ? tx0 : ty0;
    double tout = tx1 < ty1 ? tx1 : ty1;
    if (tin > tout || tout < 0.0 || tin > 1.0) return false;
    double t = tin >= 0.0 ? tin : tout;
    if (t > 1.0) return false;
    dout = gdist(cx + t * ddx, cy + t * ddy, cx, cy);
    return true;
}

__device__ bool ray_vline(double cx, double cy, double ex, double ey, double lx, double &dout) {
    if (cx == lx && ex == lx) { dout = 0.0; return true; }
    if ((cx - lx) * (ex - lx) > 0.0) return false;
    double t = (lx - cx) / (ex - cx);
    dout = gdist(lx, cy + t * (ey - cy), cx, cy);
    return true;
}

__device__ bool ray_hline(double cx, double cy, double ex, double ey, double ly, double &dout) {
    if (cy == ly && ey == ly) { dout = 0.0; return true; }
    if ((cy - ly) * (ey - ly) > 0.0) return false;
    double t = (ly - cy) / (ey - cy);
    dout = gdist(cx + t * (ex - cx), ly, cx, cy);
    return true;
}

__device__ void tdcpa(double ox, double oy, double hx, double hy, double ovx, double ovy, double hvx, double hvy,
                      double pb, double &tcpa, double &dcpa, int &total) {
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
        if (d < pb + pb) total += 1;
    } else {
        t = __builtin_fma(ry, wy, rx * wx) / sq;
        d = npnorm((rx * -1) + (wx * t), (ry * -1) + (wy * t));
    }
    if (t <= 1 && t >= 0 && d < pb + pb) total += 1;
    tcpa = t;
    dcpa = d;
}

__device__ double pairwise_sum(const double *a, int n) {
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

inline void fill_tables(Tab &t) {
    const double quantum = PI_GEOS / 2.0 / 16;
    const double total = std::fabs(0.0 - 2.0 * PI_GEOS);
    const int nseg = (int)(total / quantum + 0.5);
    const double inc = total / nseg;
    for (int i = 0; i < 64; ++i) {
        double a = 0.0 + (double)(-1 * i) * inc;
        t.circ_c[i] = std::cos(a);
        t.circ_s[i] = std::sin(a);
        t.nrm_c[i] = std::cos((i + 0.5) * PI_GEOS / 32.0);
        t.nrm_s[i] = std::sin((i + 0.5) * PI_GEOS / 32.0);
    }
    for (int r = 0; r < NRAY; ++r) {
        double rad = (double)(20 * r) * (PI_GEOS / 180.0);
        t.ray_c[r] = std::cos(rad);
        t.ray_s[r] = std::sin(rad);
    }
    t.apothem = std::cos(PI_GEOS / 64.0);
    t.cos_quantum = std::cos(quantum);
    t.quantum = quantum;
}

}  // namespace
