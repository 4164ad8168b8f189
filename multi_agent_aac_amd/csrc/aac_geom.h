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
// (out of line: only the capsule's uncertain band reaches it)
__device__ __attribute__((noinline)) double fillet_extreme(double px, double py, double start, double end, double r, int ax, bool mx) {
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
__device__ __attribute__((always_inline)) bool capsule_crash(double r, const double *b, double x0, double y0, double x1, double y1) {
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
__device__ __attribute__((always_inline)) bool gons_meet(double dx, double dy, double R, bool strict) {
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


// ------------------------------------------------------------------ exact threshold predicates
// The closed forms in this file use the ideal polygons (exact edge normals / apothem); GEOS decides
// its predicates exactly (DD orientation) on the ROUNDED float vertices, ~1e-13 m away from the ideal
// ones.  Within EXACT_BAND of a threshold the ATT / OM predicates hand the decision to the exact
// separating-axis test below on those vertices (oracle/geos.py BAND: the C oracle restates it with
// 128-bit integers, the tests with rationals).  Orientation signs are exact: the coordinate
// differences are exact (Sterbenz) when the coordinates of an axis lie within a factor of 2 of each
// other -- every coordinate of the ATT / OM world ([455, 680] x [255, 385], the 15-m radar and the
// step around it) -- so orient = A B - C D with exact A, B, C, D, and its sign is that of the 4-term
// nonoverlapping expansion fl(AB) + err(AB) - fl(CD) - err(CD) (Shewchuk's Two_Two_Diff).  A
// difference that is not exact makes the test report "undecidable" and the float closed form stands.
constexpr double EXACT_BAND = 1e-9;     // metres: projections, orientations
constexpr double EXACT_BAND_T = 1e-9;   // the ray parameter t

__device__ inline void two_sum(double a, double b, double &x, double &y) {
    x = a + b;
    const double bv = x - a, av = x - bv;
    y = (a - av) + (b - bv);
}
__device__ inline void two_diff(double a, double b, double &x, double &y) {
    x = a - b;
    const double bv = a - x, av = x + bv;
    y = (a - av) + (bv - b);
}

// sign of (bx - ax)(qy - ay) - (by - ay)(qx - ax), exactly; ok = false when a difference rounds
__device__ __attribute__((always_inline)) int orient_sign(double ax, double ay, double bx, double by, double qx, double qy, bool &ok) {
    double A, B, C, D, ta, tb, tc, td;
    two_diff(bx, ax, A, ta);
    two_diff(qy, ay, B, tb);
    two_diff(by, ay, C, tc);
    two_diff(qx, ax, D, td);
    ok = ta == 0.0 && tb == 0.0 && tc == 0.0 && td == 0.0;
    const double p1 = A * B, e1 = __builtin_fma(A, B, -p1);
    const double p2 = C * D, e2 = __builtin_fma(C, D, -p2);
    // Two_Two_Diff(p1, e1, p2, e2) -> x3 x2 x1 x0 (x3 the most significant)
    double i0, x0, j, k0, x3, x2, x1, m0;
    two_diff(e1, e2, i0, x0);       // Two_One_Diff(p1, e1, e2 -> j, k0, x0)
    two_sum(p1, i0, j, k0);
    two_diff(k0, p2, m0, x1);       // Two_One_Diff(j, k0, p2 -> x3, x2, x1)
    two_sum(j, m0, x3, x2);
    const double top = x3 != 0.0 ? x3 : (x2 != 0.0 ? x2 : (x1 != 0.0 ? x1 : x0));
    return (top > 0.0) - (top < 0.0);
}

// orientation sign of q against v -> w: the float value when it is clearly away from 0, else exact
// (0 when undecidable: ok = false)
__device__ inline int orient_banded(double vx, double vy, double wx, double wy, double qx, double qy, bool &ok) {
    const double o = (wx - vx) * (qy - vy) - (wy - vy) * (qx - vx);
    ok = true;
    if (o > EXACT_BAND) return 1;
    if (o < -EXACT_BAND) return -1;
    return orient_sign(vx, vy, wx, wy, qx, qy, ok);
}

// GEOS 64-gon(p, r) meets the closed square [x0, x1] x [y0, y1], exactly on the float vertices: the
// square's axes against the 64-gon's extreme vertices (0: max x, 16: min y, 32: min x, 48: max y;
// their neighbours are r (1 - cos(pi/32)) = 0.012 m inside), then each 64-gon edge against the
// square corner nearest to it (the other corners lie >= 10 sin(pi/64) = 0.49 m further out).  A real call
// (rare; inlined into the agent phase it slowed the WGRU step by ~12 us).  1 / 0, -1 undecidable.
__device__ __attribute__((always_inline)) int gon_square_meet(double px, double py, double r, double x0, double x1, double y0, double y1) {
    if (px + r * c_tab.circ_c[32] > x1 || px + r * c_tab.circ_c[0] < x0 || py + r * c_tab.circ_s[16] > y1 ||
        py + r * c_tab.circ_s[48] < y0)
        return 0;
    int und = 0;
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
        const int k = 63 - i;            // edge i -> i + 1 has the outward normal of index 63 - i
        const double qx = c_tab.nrm_c[k] > 0.0 ? x0 : x1, qy = c_tab.nrm_s[k] > 0.0 ? y0 : y1;
        const int i1 = (i + 1) & 63;
        bool ok;
        const int sg = orient_banded(px + r * c_tab.circ_c[i], py + r * c_tab.circ_s[i], px + r * c_tab.circ_c[i1],
                                     py + r * c_tab.circ_s[i1], qx, qy, ok);
        if (!ok) und = 1;
        else if (sg > 0) return 0;       // the corner, hence the square, strictly outside this edge
    }
    return und ? -1 : 1;
}

// the same as a real call: rare, and the WGRU step kernel runs faster with it out of line
__device__ __attribute__((noinline)) int gon_square_meet_call(double px, double py, double r, double x0, double x1,
                                                             double y0, double y1) {
    return gon_square_meet(px, py, r, x0, x1, y0, y1);
}

// segment c -> e meets the GEOS 64-gon (p, r), exactly on the float vertices: no 64-gon edge has both
// endpoints strictly outside, and the vertices are not all strictly on one side of the segment's line.
// 1 / 0, -1 undecidable.
__device__ __attribute__((noinline)) int seg_gon_meet(double cx, double cy, double ex, double ey, double px, double py, double r) {
    int und = 0;
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
        const int i1 = (i + 1) & 63;
        const double vx = px + r * c_tab.circ_c[i], vy = py + r * c_tab.circ_s[i];
        const double wx = px + r * c_tab.circ_c[i1], wy = py + r * c_tab.circ_s[i1];
        bool ok;
        int sg = orient_banded(vx, vy, wx, wy, cx, cy, ok);
        if (!ok) { und = 1; continue; }
        if (sg <= 0) continue;
        sg = orient_banded(vx, vy, wx, wy, ex, ey, ok);
        if (!ok) und = 1;
        else if (sg > 0) return 0;
    }
    int pos = 0, neg = 0;
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
        bool ok;
        const int sg = orient_banded(cx, cy, ex, ey, px + r * c_tab.circ_c[i], py + r * c_tab.circ_s[i], ok);
        if (!ok) und = 1;
        pos |= sg > 0 ? 1 : 2;           // bit 1: a vertex not strictly on the left
        neg |= sg < 0 ? 1 : 2;
    }
    if (!und && (pos == 1 || neg == 1)) return 0;     // every vertex strictly on one side
    return und ? -1 : 1;
}

// segment c -> e meets the closed square, exactly: bounding boxes overlap, and the corners are not all
// strictly on one side of the segment's line.  1 / 0, -1 undecidable.
__device__ __attribute__((noinline)) int seg_square_meet(double cx, double cy, double ex, double ey, double x0, double x1, double y0, double y1) {
    if (fmax(cx, ex) < x0 || fmin(cx, ex) > x1 || fmax(cy, ey) < y0 || fmin(cy, ey) > y1) return 0;
    int pos = 0, neg = 0, und = 0;
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        bool ok;
        const int sg = orient_banded(cx, cy, ex, ey, i < 2 ? x0 : x1, (i == 1 || i == 2) ? y1 : y0, ok);
        if (!ok) und = 1;
        pos |= sg > 0 ? 1 : 2;
        neg |= sg < 0 ? 1 : 2;
    }
    if (!und && (pos == 1 || neg == 1)) return 0;
    return und ? -1 : 1;
}

// the band part of goal_meet_exact (inline, or as the real call goal_band_exact_call)
__device__ __attribute__((always_inline)) bool goal_band_exact(double px, double py, double gx, double gy, double pb,
                                                          double dx, double dy, double m, double thr, int km) {
#pragma unroll 1
    for (int c = -1; c <= 1; ++c) {
        const int k = (km + c) & 63;
        if (c != 0 && dx * c_tab.nrm_c[k] + dy * c_tab.nrm_s[k] < m - 1e-6) continue;
        const int ia = 63 - k, ib = 63 - ((k + 32) & 63);
        int sep = 3;                          // bit 0: A's edge separates, bit 1: B's facing edge
#pragma unroll 1
        for (int j = 0; j < 4; ++j) {         // one orientation at a time (registers: agent phase)
            const bool ea = j < 2;            // j 0, 1: A's edge vs B's vertices; 2, 3: B's edge vs A's
            const double ox = ea ? px : gx, oy = ea ? py : gy, orr = ea ? pb : 1.0;
            const double qx0 = ea ? gx : px, qy0 = ea ? gy : py, qr = ea ? 1.0 : pb;
            const int ie = ea ? ia : ib, iq = ((ea ? ib : ia) + (j & 1)) & 63;
            bool ok;
            const int sg = orient_banded(ox + orr * c_tab.circ_c[ie], oy + orr * c_tab.circ_s[ie],
                                         ox + orr * c_tab.circ_c[(ie + 1) & 63], oy + orr * c_tab.circ_s[(ie + 1) & 63],
                                         qx0 + qr * c_tab.circ_c[iq], qy0 + qr * c_tab.circ_s[iq], ok);
            if (!ok) return m <= thr;         // undecidable: the closed form
            if (sg <= 0) sep &= ea ? ~1 : ~2;
        }
        if (sep) return false;
    }
    return true;
}

__device__ __attribute__((noinline)) bool goal_band_exact_call(double px, double py, double gx, double gy, double pb,
                                                                double dx, double dy, double m, double thr, int km) {
    return goal_band_exact(px, py, gx, gy, pb, dx, dy, m, thr, km);
}

// 64-gon(p, pb) meets 64-gon(g, 1) (ATT/env:2266-2269): gons_meet's closed form, and within EXACT_BAND
// of the threshold the exact test on the float vertices.  Both rings have their edge normals at the
// angles (k + 1/2) pi/32, so the axis n_k separates them (ideally) iff d.n_k > (pb + 1) cos(pi/64): only
// the normals within 1e-6 of the maximum projection m (at most two adjacent ones) can separate the
// float polygons, by the A edge with outward normal n_k (vertices 63 - k, 64 - k) or the B edge facing
// it; the exact test checks each against the two vertices of the other's facing edge (the other
// vertices lie >= 1 (cos(pi/64) - cos(3 pi/64)) = 0.0096 m further out)
template <bool COLD>
__device__ __attribute__((always_inline)) bool goal_meet_exact(double px, double py, double gx, double gy, double pb) {
    const double dx = gx - px, dy = gy - py, R = pb + 1.0;
    const double thr = R * c_tab.apothem;
    const double dist = sqrt(dx * dx + dy * dy);
    if (dist > R * (1.0 + 1e-12) + 1e-12) return false;
    if (dist < thr * (1.0 - 1e-12) - 1e-12) return true;
    double m = -INFINITY;
    int km = 0;
#pragma unroll 8
    for (int k = 0; k < 64; ++k) {
        double v = dx * c_tab.nrm_c[k] + dy * c_tab.nrm_s[k];
        km = v > m ? k : km;
        m = v > m ? v : m;
    }
    if (m > thr + EXACT_BAND) return false;
    if (m < thr - EXACT_BAND) return true;
    return COLD ? goal_band_exact_call(px, py, gx, gy, pb, dx, dy, m, thr, km)
                : goal_band_exact(px, py, gx, gy, pb, dx, dy, m, thr, km);
}

// Cyrus-Beck entry of segment c->e into the clockwise GEOS 64-gon of radius r at p.  EX = 1 (the ATT / OM
// radar's threshold band; EX = 0: the float clip as it stands): an interval [tlo, thi] within
// EXACT_BAND_T of empty -- a ray touching the polygon, or starting on its boundary -- is a band case (a
// touch at the segment's end, tlo ~ 1, gives the distance L either way: the float decision stands).
// mode 1 flags it (band = true) and returns the float clip's answer; mode 2 decides it by the exact
// segment / polygon test (a real call), a touching ray entering at clamp(tlo, 0, 1).
template <int EX = 0>
__device__ __attribute__((always_inline)) bool ray_poly_entry_full(double cx, double cy, double ex, double ey,
                                                                   double px, double py, double r, double &tout,
                                                                   bool &band, int mode = 1) {
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
        if (EX == 0 ? tlo > thi : tlo - thi > EXACT_BAND_T) return false;   // (empty beyond the band: certain)
        vx = wx;
        vy = wy;
    }
    if (EX != 0 && tlo - thi >= -EXACT_BAND_T && tlo < 1.0 - EXACT_BAND_T) {
        if (mode == 1) {
            band = true;
        } else {
            const int m = seg_gon_meet(cx, cy, ex, ey, px, py, r);
            if (m == 0 || (m < 0 && tlo > thi)) return false;
            tout = tlo < 0.0 ? 0.0 : (tlo > 1.0 ? 1.0 : tlo);
            return true;
        }
    }
    if (tlo > thi) return false;
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
template <int EX = 0>
__device__ __attribute__((always_inline)) bool ray_poly_entry(double cx, double cy, double ex, double ey, double px, double py, double r,
                               double &tout, bool &band, int mode = 1) {
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
        return ray_poly_entry_full<EX>(cx, cy, ex, ey, px, py, r, tout, band, mode);
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
    if (!any) return ray_poly_entry_full<EX>(cx, cy, ex, ey, px, py, r, tout, band, mode);
    if (tlo > 1.0) return false;
    tout = tlo;
    return true;
}

// EX = 1 (ATT / OM; see ray_poly_entry_full): where the rounded slab quotients tie within EXACT_BAND_T (a
// ray through a corner) away from the segment's end, mode 1 flags a band case and mode 2 decides: the
// segment meets the square's boundary iff it meets the closed square and does not lie inside the open
// one (exact test, a real call).  Ties and exits at t ~ 1 give the distance L either way.
template <int EX = 0>
__device__ __attribute__((always_inline)) bool ray_square(double cx, double cy, double ex, double ey, double x0,
                                                          double x1, double y0, double y1, double &dout, bool &band,
                                                          int mode = 1) {
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
    if (EX != 0 && fabs(tin - tout) <= EXACT_BAND_T && tin < 1.0 - EXACT_BAND_T) {
        if (mode == 1) {
            band = true;
        } else {
            const bool inside = x0 < cx && cx < x1 && y0 < cy && cy < y1 && x0 < ex && ex < x1 && y0 < ey && ey < y1;
            int m = inside ? 0 : seg_square_meet(cx, cy, ex, ey, x0, x1, y0, y1);
            if (m < 0) m = !(tin > tout || tout < 0.0 || tin > 1.0 || (tin < 0.0 && tout > 1.0));
            if (!m) return false;
            double t = tin >= 0.0 ? tin : tout;
            t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
            dout = gdist(cx + t * ddx, cy + t * ddy, cx, cy);
            return true;
        }
    }
    if (tin > tout || tout < 0.0 || tin > 1.0) return false;
    double t = tin >= 0.0 ? tin : tout;
    if (t > 1.0) return false;
    dout = gdist(cx + t * ddx, cy + t * ddy, cx, cy);
    return true;
}

// the float-only forms (UAM radar)
__device__ inline bool ray_poly_entry(double cx, double cy, double ex, double ey, double px, double py, double r,
                                      double &tout) {
    bool band = false;
    return ray_poly_entry<0>(cx, cy, ex, ey, px, py, r, tout, band, 1);
}
__device__ inline bool ray_square(double cx, double cy, double ex, double ey, double x0, double x1, double y0,
                                  double y1, double &dout) {
    bool band = false;
    return ray_square<0>(cx, cy, ex, ey, x0, x1, y0, y1, dout, band);
}

__device__ __attribute__((always_inline)) bool ray_vline(double cx, double cy, double ex, double ey, double lx, double &dout) {
    if (cx == lx && ex == lx) { dout = 0.0; return true; }
    if ((cx - lx) * (ex - lx) > 0.0) return false;
    double t = (lx - cx) / (ex - cx);
    dout = gdist(lx, cy + t * (ey - cy), cx, cy);
    return true;
}

__device__ __attribute__((always_inline)) bool ray_hline(double cx, double cy, double ex, double ey, double ly, double &dout) {
    if (cy == ly && ey == ly) { dout = 0.0; return true; }
    if ((cy - ly) * (ey - ly) > 0.0) return false;
    double t = (ly - cy) / (ey - cy);
    dout = gdist(cx + t * (ex - cx), ly, cx, cy);
    return true;
}

__device__ __attribute__((always_inline)) void tdcpa(double ox, double oy, double hx, double hy, double ovx, double ovy, double hvx, double hvy,
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

__device__ __attribute__((always_inline)) double pairwise_sum(const double *a, int n) {
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
