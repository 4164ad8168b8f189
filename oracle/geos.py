"""GEOS (shapely 2.0.1 -> GEOS 3.11) buffer construction and the predicates the
reference evaluates on those buffers.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference builds every shape with shapely's ``buffer`` (quad_segs=16) and then
asks GEOS ``intersects``/``intersection``/``distance``.  GEOS is not installed here,
so this module restates

* the *construction* exactly, following GEOS ``OffsetSegmentGenerator``:
  ``createCircle`` (Point.buffer), ``computeLineBufferCurve`` +
  ``addLineEndCap``/``addDirectedFillet`` (LineString.buffer with round caps),
  ``computeOffsetSegment``, and the ``isRedundant`` vertex filter
  (minimum vertex distance = 1e-6 * distance);
* the *predicates* as closed forms that are exact in real arithmetic for those
  convex shapes (used by the batched oracle and by the HIP kernel, same operation
  order), plus an independent exact-rational formulation (``Fraction``) evaluated
  on the actual floating-point vertices, used only by tests to cross-check the
  closed forms.

Reference call sites: ATT/env:1080-1159 (radar), :2172-2175 (capsule, own circle),
:2243-2250 (building), :2266-2269 (goal), :2507 (bound); OM/env:1100-1141
(obstacle radar).
"""
import math
from fractions import Fraction

from .consts import MATH_PI, QUAD_SEGS, PB

FILLET_QUANTUM = MATH_PI / 2.0 / QUAD_SEGS      # OffsetSegmentGenerator ctor
VERTEX_SNAP = 1.0e-6                            # CURVE_VERTEX_SNAP_DISTANCE_FACTOR


def _fillet(px, py, start, end, direction, radius):
    """GEOS ``addDirectedFillet`` (direction -1 == CLOCKWISE)."""
    total = abs(start - end)
    nsegs = int(total / FILLET_QUANTUM + 0.5)
    if nsegs < 1:
        return []
    inc = total / nsegs
    out = []
    for i in range(nsegs):
        ang = start + float(direction * i) * inc
        out.append((px + radius * math.cos(ang), py + radius * math.sin(ang)))
    return out


class _SegList:
    """GEOS ``OffsetSegmentString`` with its ``isRedundant`` filter."""

    def __init__(self, distance):
        self.pts = []
        self.min_dist = distance * VERTEX_SNAP

    def add(self, p):
        if self.pts:
            q = self.pts[-1]
            dx, dy = p[0] - q[0], p[1] - q[1]
            if math.sqrt(dx * dx + dy * dy) < self.min_dist:
                return
        self.pts.append(p)


def circle_vertices(px, py, r):
    """Vertices of ``Point(px, py).buffer(r)`` (GEOS ``createCircle``), ring order, unclosed."""
    seg = _SegList(r)
    seg.add((px + r, py))
    for p in _fillet(px, py, 0.0, 2.0 * MATH_PI, -1, r):
        seg.add(p)
    return seg.pts


def circle_unit_table():
    """(cos, sin) of GEOS createCircle angles 0 - i*inc, i = 0..63 (i=0 gives (1, 0))."""
    total = abs(0.0 - 2.0 * MATH_PI)
    nsegs = int(total / FILLET_QUANTUM + 0.5)
    inc = total / nsegs
    return [(math.cos(0.0 + float(-1 * i) * inc), math.sin(0.0 + float(-1 * i) * inc)) for i in range(nsegs)]


def _offset_segment(p0, p1, side, distance):
    """GEOS ``computeOffsetSegment``: side +1 LEFT, -1 RIGHT."""
    dx = p1[0] - p0[0]
    dy = p1[1] - p0[1]
    ln = math.sqrt(dx * dx + dy * dy)
    ux = side * distance * dx / ln
    uy = side * distance * dy / ln
    return (p0[0] - uy, p0[1] + ux), (p1[0] - uy, p1[1] + ux)


def _line_end_cap(seg, p0, p1, distance):
    """GEOS ``addLineEndCap`` with CAP_ROUND."""
    _, l1 = _offset_segment(p0, p1, 1, distance)
    _, r1 = _offset_segment(p0, p1, -1, distance)
    ang = math.atan2(p1[1] - p0[1], p1[0] - p0[0])
    seg.add(l1)
    for p in _fillet(p1[0], p1[1], ang + MATH_PI / 2.0, ang - MATH_PI / 2.0, -1, distance):
        seg.add(p)
    seg.add(r1)


def capsule_vertices(p0, p1, r):
    """Vertices of ``LineString([p0, p1]).buffer(r, cap_style='round')`` (ATT/env:2172-2173).

    A zero-length segment collapses to a point and GEOS emits ``createCircle``.
    """
    p0 = (float(p0[0]), float(p0[1]))
    p1 = (float(p1[0]), float(p1[1]))
    if p0 == p1:
        return circle_vertices(p0[0], p0[1], r)
    seg = _SegList(r)
    # left side: initSideSegments(p0, p1, LEFT) ; addLastSegment -> offset1.p1
    _, l1 = _offset_segment(p0, p1, 1, r)
    seg.add(l1)
    _line_end_cap(seg, p0, p1, r)
    # right side, traversed backwards, still LEFT
    _, rr1 = _offset_segment(p1, p0, 1, r)
    seg.add(rr1)
    _line_end_cap(seg, p1, p0, r)
    return seg.pts


# ---------------------------------------------------------------------------
# closed forms (exact in real arithmetic; same operation order as the kernel)
# ---------------------------------------------------------------------------

def edge_normal_table():
    """Unit outward normals of the regular 64-gon edges: angle (k + 1/2) * pi/32."""
    return [(math.cos((k + 0.5) * MATH_PI / 32.0), math.sin((k + 0.5) * MATH_PI / 32.0)) for k in range(64)]


APOTHEM_UNIT = math.cos(MATH_PI / 64.0)


# Threshold bands.  The closed forms use the ideal polygon (exact edge normals / apothem); GEOS
# evaluates its predicates exactly (DD orientation) on the rounded float vertices, ~1e-13 away from
# the ideal ones.  Inside these bands around a threshold the exact formulation on the float
# vertices decides (exact-threshold states); outside them the closed form cannot
# differ from it.  BAND is in metres (projections), BAND_T in units of the ray parameter t.
BAND = 1e-9
BAND_T = 1e-9


def goal_reached(px, py, gx, gy):
    """64-gon(pos, 2.5) intersects 64-gon(goal, 1)   (ATT/env:2266-2269, :2546).

    Both shapes share the vertex angles k*pi/32, so their Minkowski difference is the
    regular 64-gon of circumradius 3.5 and the test is ``max_k d.n_k <= 3.5 cos(pi/64)``;
    within BAND of the threshold the exact test on the GEOS float vertices decides.
    """
    dx = gx - px
    dy = gy - py
    thr = (PB + 1.0) * APOTHEM_UNIT
    m = -math.inf
    for nx, ny in edge_normal_table():
        v = dx * nx + dy * ny
        if v > m:
            m = v
    if m > thr + BAND:
        return False
    if m < thr - BAND:
        return True
    return convex_polys_intersect_exact(circle_vertices(px, py, PB), circle_vertices(gx, gy, 1.0))


def building_hit_cell(px, py, cx, cy, half=5.0):
    """64-gon(pos, 2.5) intersects the closed square cell centred (cx, cy)  (ATT/env:2243-2250).

    Separating-axis test on the square axes and the 32 distinct 64-gon edge normals; an axis
    within BAND of separating hands the decision to the exact test on the float vertices.
    """
    dx = cx - px
    dy = cy - py
    unsure = False
    for v in (abs(dx), abs(dy)):
        if v > half + PB + BAND:
            return False
        if v > half + PB - BAND:
            unsure = True
    for nx, ny in edge_normal_table()[:32]:
        proj = abs(dx * nx + dy * ny)
        lim = half * (abs(nx) + abs(ny)) + PB * APOTHEM_UNIT
        if proj > lim + BAND:
            return False
        if proj > lim - BAND:
            unsure = True
    if unsure:
        sq = [(cx - half, cy - half), (cx + half, cy - half), (cx + half, cy + half), (cx - half, cy + half)]
        return convex_polys_intersect_exact(circle_vertices(px, py, PB), sq)
    return True


def capsule_extents(p0, p1, r):
    vs = capsule_vertices(p0, p1, r)
    xs = [v[0] for v in vs]
    ys = [v[1] for v in vs]
    return min(xs), max(xs), min(ys), max(ys)


def bound_crash(p0, p1, bound, r=PB):
    """Any of the 4 infinite bound lines intersects the swept capsule  (ATT/env:2507).

    The capsule is convex, so a line x=c meets it iff min_x <= c <= max_x (GEOS
    orientation predicates on the float vertices are exact for these axis lines).
    """
    mnx, mxx, mny, mxy = capsule_extents(p0, p1, r)
    return ((mnx <= bound[0] <= mxx) or (mnx <= bound[1] <= mxx)
            or (mny <= bound[2] <= mxy) or (mny <= bound[3] <= mxy))


def ray_polygon_entry(cx, cy, ex, ey, poly):
    """Parameter t in [0,1] of the first point of segment c->e inside the convex
    clockwise polygon ``poly`` (Cyrus-Beck), or None.  Same operation order as the kernel.

    When the clip's interval [t_lo, t_hi] is within BAND_T of empty (a ray touching the polygon
    at a vertex, or ending on / starting on its boundary) the exact segment-polygon test on the
    float vertices decides; a touching ray then enters at clamp(t_lo, 0, 1)."""
    ddx = ex - cx
    ddy = ey - cy
    t_lo, t_hi = 0.0, 1.0
    n = len(poly)
    for k in range(n):
        vx, vy = poly[k]
        wx, wy = poly[(k + 1) % n]
        exx = wx - vx
        eyy = wy - vy
        a = exx * (cy - vy) - eyy * (cx - vx)
        b = exx * ddy - eyy * ddx
        if b == 0.0:
            if a > 0.0:
                return None
        elif b < 0.0:
            t = -a / b
            if t > t_lo:
                t_lo = t
        else:
            t = -a / b
            if t < t_hi:
                t_hi = t
    if t_lo - t_hi > BAND_T:
        return None
    if t_lo - t_hi < -BAND_T:
        return t_lo
    if t_lo >= 1.0 - BAND_T:          # a touch at the segment's end: the distance is L either way
        return None if t_lo > t_hi else t_lo
    if segment_convex_entry_exact((cx, cy), (ex, ey), poly) is None:
        return None
    return min(max(t_lo, 0.0), 1.0)


def point_dist(ax, ay, bx, by):
    """GEOS Coordinate::distance (no FMA)."""
    dx = ax - bx
    dy = ay - by
    return math.sqrt(dx * dx + dy * dy)


def ray_square_crossing(cx, cy, ex, ey, x0, x1, y0, y1):
    """Distance from c to the nearest point of segment(c,e) ∩ boundary(square), or None
    (OM/env:1117-1126: ``line.intersection(polygon.boundary)`` then ``distance``).

    The slab parameters are rounded quotients: where they tie within BAND_T (a ray through a corner)
    away from the segment's end, the exact segment / boundary test decides (near t = 1 the distance is
    L hit or not)."""
    ddx = ex - cx
    ddy = ey - cy
    # a ray running along an edge from a start point on that edge: line.intersection(boundary) is
    # a segment through c, so the distance is 0
    if (ddx == 0.0 and cx in (x0, x1) and y0 <= cy <= y1) or (ddy == 0.0 and cy in (y0, y1) and x0 <= cx <= x1):
        return 0.0
    if ddx == 0.0:
        if cx < x0 or cx > x1:
            return None
        tx0, tx1 = -math.inf, math.inf
    else:
        ta = (x0 - cx) / ddx
        tb = (x1 - cx) / ddx
        tx0, tx1 = (ta, tb) if ta < tb else (tb, ta)
    if ddy == 0.0:
        if cy < y0 or cy > y1:
            return None
        ty0, ty1 = -math.inf, math.inf
    else:
        ta = (y0 - cy) / ddy
        tb = (y1 - cy) / ddy
        ty0, ty1 = (ta, tb) if ta < tb else (tb, ta)
    t_in = tx0 if tx0 > ty0 else ty0
    t_out = tx1 if tx1 < ty1 else ty1
    if abs(t_in - t_out) <= BAND_T and t_in < 1.0 - BAND_T:
        if ray_square_boundary_t_exact((cx, cy), (ex, ey), x0, x1, y0, y1) is None:
            return None
        t = t_in if t_in >= 0.0 else t_out
        t = min(max(t, 0.0), 1.0)
        return point_dist(cx + t * ddx, cy + t * ddy, cx, cy)
    if t_in > t_out or t_out < 0.0 or t_in > 1.0:
        return None
    t = t_in if t_in >= 0.0 else t_out
    if t > 1.0:
        return None
    return point_dist(cx + t * ddx, cy + t * ddy, cx, cy)


def ray_vline_crossing(cx, cy, ex, ey, lx):
    """Distance from c to segment(c,e) ∩ (x = lx) (OM/env:1127-1141), or None."""
    if cx == lx and ex == lx:
        return 0.0  # collinear: intersection LineString contains c
    if (cx - lx) * (ex - lx) > 0.0:
        return None
    ddx = ex - cx
    t = (lx - cx) / ddx
    return point_dist(lx, cy + t * (ey - cy), cx, cy)


def ray_hline_crossing(cx, cy, ex, ey, ly):
    if cy == ly and ey == ly:
        return 0.0
    if (cy - ly) * (ey - ly) > 0.0:
        return None
    ddy = ey - cy
    t = (ly - cy) / ddy
    return point_dist(cx + t * (ex - cx), ly, cx, cy)


# ---------------------------------------------------------------------------
# point -> LineString nearest point (shapely.ops.nearest_points, GEOS DistanceOp)
# WGRU/env:2621-2632 cross_track_error; WGRU/env:1882 (the reference path of reset_world :343)
# ---------------------------------------------------------------------------

def point_to_segment(px, py, ax, ay, bx, by):
    """GEOS 3.11 algorithm::Distance::pointToSegment."""
    if ax == bx and ay == by:
        return point_dist(px, py, ax, ay)
    len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay)
    r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2
    if r <= 0.0:
        return point_dist(px, py, ax, ay)
    if r >= 1.0:
        return point_dist(px, py, bx, by)
    s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2
    return abs(s) * math.sqrt(len2)


def _projection_factor(px, py, ax, ay, bx, by):
    """GEOS LineSegment::projectionFactor."""
    if px == ax and py == ay:
        return 0.0
    if px == bx and py == by:
        return 1.0
    dx, dy = bx - ax, by - ay
    len2 = dx * dx + dy * dy
    if len2 == 0.0:                     # C++ division: NaN (or +-inf); never > 0 and < 1 below
        return math.nan
    return ((px - ax) * dx + (py - ay) * dy) / len2


def segment_closest_point(px, py, ax, ay, bx, by):
    """GEOS LineSegment::closestPoint (project() inside the open segment, else the nearer end)."""
    f = _projection_factor(px, py, ax, ay, bx, by)
    if f > 0 and f < 1:
        if (px == ax and py == ay) or (px == bx and py == by):
            return px, py
        return ax + f * (bx - ax), ay + f * (by - ay)
    d0 = point_dist(ax, ay, px, py)
    d1 = point_dist(bx, by, px, py)
    return (ax, ay) if d0 < d1 else (bx, by)


def nearest_point_on_linestring(px, py, pts):
    """DistanceOp::computeMinDistance(line, point): the first segment with the strictly smallest
    pointToSegment distance gives the nearest point; stops at distance 0 (terminateDistance)."""
    best, loc = math.inf, None
    for k in range(len(pts) - 1):
        (ax, ay), (bx, by) = pts[k], pts[k + 1]
        d = point_to_segment(px, py, ax, ay, bx, by)
        if d < best:
            best = d
            loc = segment_closest_point(px, py, ax, ay, bx, by)
        if best <= 0.0:
            break
    return loc


def cross_track_distance(px, py, pts):
    """cross_track_error(...)[0] (WGRU/env:2621-2632): point.distance(nearest_points(point, line)[1])."""
    nx, ny = nearest_point_on_linestring(px, py, pts)
    return point_dist(px, py, nx, ny)


# ---------------------------------------------------------------------------
# independent exact formulations (tests only): rational arithmetic on the
# actual floating-point vertices GEOS would produce.
# ---------------------------------------------------------------------------

def _fr(p):
    return (Fraction(p[0]), Fraction(p[1]))


def convex_polys_intersect_exact(A, B):
    """Closed convex polygons intersect (touching counts) -- exact separating axis test."""
    A = [_fr(p) for p in A]
    B = [_fr(p) for p in B]
    for P in (A, B):
        n = len(P)
        for k in range(n):
            (x0, y0), (x1, y1) = P[k], P[(k + 1) % n]
            nx, ny = (y1 - y0), -(x1 - x0)
            pa = [nx * x + ny * y for x, y in A]
            pb = [nx * x + ny * y for x, y in B]
            if max(pa) < min(pb) or max(pb) < min(pa):
                return False
    return True


def segment_convex_entry_exact(c, e, poly):
    """Exact parameter of the first point of segment c->e inside convex polygon, or None."""
    cx, cy = _fr(c)
    ex, ey = _fr(e)
    P = [_fr(p) for p in poly]
    # orientation of the ring
    area2 = sum(P[k][0] * P[(k + 1) % len(P)][1] - P[(k + 1) % len(P)][0] * P[k][1] for k in range(len(P)))
    sgn = -1 if area2 < 0 else 1   # clockwise rings: interior on the right
    t_lo, t_hi = Fraction(0), Fraction(1)
    ddx, ddy = ex - cx, ey - cy
    for k in range(len(P)):
        (vx, vy), (wx, wy) = P[k], P[(k + 1) % len(P)]
        exx, eyy = wx - vx, wy - vy
        a = sgn * -(exx * (cy - vy) - eyy * (cx - vx))
        b = sgn * -(exx * ddy - eyy * ddx)
        # inside  <=>  a + t b <= 0
        if b == 0:
            if a > 0:
                return None
        elif b < 0:
            t_lo = max(t_lo, -a / b)
        else:
            t_hi = min(t_hi, -a / b)
        if t_lo > t_hi:
            return None
    return t_lo


def _seg_seg_first_t_exact(c, d, a, b):
    """Exact smallest t in [0, 1] with c + t d on the closed segment a-b (Fractions), or None.
    Collinear overlaps give the first overlapping parameter."""
    ex, ey = b[0] - a[0], b[1] - a[1]
    den = d[0] * ey - d[1] * ex
    wx, wy = a[0] - c[0], a[1] - c[1]
    if den != 0:
        t = (wx * ey - wy * ex) / den
        s = (wx * d[1] - wy * d[0]) / den
        return t if (0 <= t <= 1 and 0 <= s <= 1) else None
    if wx * d[1] - wy * d[0] != 0:
        return None                      # parallel, not collinear
    dd = d[0] * d[0] + d[1] * d[1]
    ta = (wx * d[0] + wy * d[1]) / dd    # parameters of a and b along c + t d
    tb = ((b[0] - c[0]) * d[0] + (b[1] - c[1]) * d[1]) / dd
    lo, hi = (ta, tb) if ta <= tb else (tb, ta)
    lo, hi = max(lo, Fraction(0)), min(hi, Fraction(1))
    return lo if lo <= hi else None


def ray_square_boundary_t_exact(c, e, x0, x1, y0, y1):
    """Exact parameter of the point of segment c->e on the square's boundary nearest to c (the
    reference's ``line.intersection(polygon.boundary)`` + ``distance``, OM/env:1105-1116), or None:
    the union of the segment's exact intersections with the four closed edges."""
    cc, ee = _fr(c), _fr(e)
    d = (ee[0] - cc[0], ee[1] - cc[1])
    X0, X1, Y0, Y1 = Fraction(x0), Fraction(x1), Fraction(y0), Fraction(y1)
    best = None
    for a, b in (((X0, Y0), (X1, Y0)), ((X1, Y0), (X1, Y1)), ((X1, Y1), (X0, Y1)), ((X0, Y1), (X0, Y0))):
        t = _seg_seg_first_t_exact(cc, d, a, b)
        if t is not None and (best is None or t < best):
            best = t
    return best


def ray_line_t_exact(c, e, axis, value):
    """Exact parameter of segment c->e on the bound line {axis = value} (a LineString from -9999 to
    9999, ATT/env:143-146, OM/env:1117-1141), or None."""
    cc, ee = _fr(c), _fr(e)
    d = (ee[0] - cc[0], ee[1] - cc[1])
    v = Fraction(value)
    a = (v, Fraction(-9999)) if axis == 0 else (Fraction(-9999), v)
    b = (v, Fraction(9999)) if axis == 0 else (Fraction(9999), v)
    return _seg_seg_first_t_exact(cc, d, a, b)


def segment_hits_polygon_exact(p, q, poly):
    """Closed segment p-q meets the closed polygon ``poly`` (exact orientation tests on the float
    vertices): some polygon edge touches or crosses the segment, or the segment lies inside."""
    P, Q = _fr(p), _fr(q)
    V = [_fr(v) for v in poly]

    def orient(a, b, c):
        v = (b[0] - a[0]) * (c[1] - a[1]) - (b[1] - a[1]) * (c[0] - a[0])
        return (v > 0) - (v < 0)

    def on_seg(a, b, c):       # c collinear with a-b: within its box
        return min(a[0], b[0]) <= c[0] <= max(a[0], b[0]) and min(a[1], b[1]) <= c[1] <= max(a[1], b[1])

    n = len(V)
    for k in range(n):
        a, b = V[k], V[(k + 1) % n]
        o1, o2, o3, o4 = orient(P, Q, a), orient(P, Q, b), orient(a, b, P), orient(a, b, Q)
        if o1 != o2 and o3 != o4:
            return True
        if (o1 == 0 and on_seg(P, Q, a)) or (o2 == 0 and on_seg(P, Q, b)) or \
                (o3 == 0 and on_seg(a, b, P)) or (o4 == 0 and on_seg(a, b, Q)):
            return True
    # no boundary contact: inside iff P is inside (convex ring, either orientation)
    s = [orient(V[k], V[(k + 1) % n], P) for k in range(n)]
    return all(x >= 0 for x in s) or all(x <= 0 for x in s)


def point_polyline_distance_exact(p, pts):
    """Exact squared Euclidean distance from p to the polyline (Fractions): the real-arithmetic value
    the GEOS cross-track distance approximates."""
    P = _fr(p)
    best = None
    for k in range(len(pts) - 1):
        A, B = _fr(pts[k]), _fr(pts[k + 1])
        dx, dy = B[0] - A[0], B[1] - A[1]
        l2 = dx * dx + dy * dy
        if l2 == 0:
            q = A
        else:
            t = ((P[0] - A[0]) * dx + (P[1] - A[1]) * dy) / l2
            t = min(max(t, Fraction(0)), Fraction(1))
            q = (A[0] + t * dx, A[1] + t * dy)
        d2 = (P[0] - q[0]) ** 2 + (P[1] - q[1]) ** 2
        if best is None or d2 < best:
            best = d2
    return best
