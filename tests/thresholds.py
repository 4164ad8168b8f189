"""Exact-threshold env states (SURVEY.md 8(c) "hand-built edge cases").

Each env of a batch puts its agent 0 (the subject) exactly on one predicate threshold of
ATT/env:ss_reward or the radar -- and, in sibling envs, one ulp either side of it:

  drone      ||p_i - p_j|| = 5 (3-4-5 offsets; ATT/env:2228-2236, np.linalg.norm <= 2 pB)
  near*      the near-drone band's 2.5 / 10 m ends (ATT/env:2430-2432): build_near, its own batch with a
             second neighbour setting the shortest distance (else the 10-m end's term is exactly 0)
  wp         waypoint distance 5 (strict <, GEOS point distance; ATT/env:2297-2303)
  goal_apo   goal offset on the 3.5 cos(pi/64) apothem of the Minkowski 64-gon (ATT/env:2266-2269)
  goal_vtx   goal offset on a 3.5 circumradius vertex direction
  kat        ATT/geometry_test.py:13-15: pos (534.12, 355.86), goal circle (536, 356)
  bld_edge   the subject's 64-gon touching an occupied cell's edge (ATT/env:2241-2253)
  bld_corner ... touching a cell corner with a vertex direction
  bound      a stationary circle touching each bound line; an axis-parallel move whose capsule
             touches one (ATT/env:2507)
  tangent    the 0 / 180 degree ray through another agent's bottom / top vertex (ATT/env:1089-1164)
  start_on   the subject on another agent's vertex 0, its 0-degree ray leaving it
  corner     a ray through the corner of an isolated occupied cell, touching only that point
             (OM/env:1100-1141)
  edge_run   the 0-degree ray running along an occupied cell's top edge
  edge_near  the same ray along a top / bottom edge from 3 or 4.5 m: the subject's radar minimum, so the
             WGRU near-building penalty (WGRU/env ss_reward, pB <= min radar <= 5) rides on it

The subject is stationary (zero velocity, zero action), so the kinematics leave its position bit
for bit (``bound`` moves along an axis by an exact 2 m).  The other agents sit far away, out of the
subject's radar.  Test infrastructure only (no GPU needed here).
"""
import math
from fractions import Fraction

import numpy as np

from oracle import geos
from oracle.consts import BOUND, PB

GW, GH = 23, 13
# isolated occupied cells (i, j): squares [455 + 10 i, 465 + 10 i] x [255 + 10 j, 265 + 10 j]
CELLS = [(6, 5), (12, 4), (17, 7)]
HOME = (600.0, 352.0)           # a free spot for the families that need no cell


def threshold_map():
    occ = np.zeros((GW, GH), np.uint8)
    for i, j in CELLS:
        occ[i, j] = 1
    return occ


def square_of(i, j):
    return 455.0 + 10 * i, 465.0 + 10 * i, 255.0 + 10 * j, 265.0 + 10 * j


def _up(x, n=1):
    for _ in range(abs(n)):
        x = float(np.nextafter(x, math.inf if n > 0 else -math.inf))
    return x


def ray_end(c, r):
    """The radar segment's end as the kernel and the oracles compute it (radar_len * cos(radians))."""
    rad = float(20 * r) * (math.pi / 180.0)
    return c[0] + 15.0 * math.cos(rad), c[1] + 15.0 * math.sin(rad)


def _corner_start(q, r):
    """A start c with the radar ray r passing EXACTLY through the point q at a parameter t near 1/2.

    With c on its binade's grid (spacings ux, uy) the float segment's direction is exact, (nx ux, ny uy)
    in grid units (Sterbenz).  The lattice points on the segment are c + m / g (nx ux, ny uy) for the
    common divisor g of the two components in the finer unit: with g >= 2 the start c = q - m / g
    (dx, dy), m = g // 2, puts q on the segment exactly (verified with rationals)."""
    rad = float(20 * r) * (math.pi / 180.0)
    dx, dy = 15.0 * math.cos(rad), 15.0 * math.sin(rad)
    c0 = (q[0] - dx / 2, q[1] - dy / 2)
    e0 = ray_end(c0, r)
    ddx, ddy = e0[0] - c0[0], e0[1] - c0[1]
    u = min(float(np.spacing(c0[0])), float(np.spacing(c0[1])))
    nx, ny = int(Fraction(ddx) / Fraction(u)), int(Fraction(ddy) / Fraction(u))
    g = math.gcd(abs(nx), abs(ny))
    if g < 2 or Fraction(ddx) != nx * Fraction(u) or Fraction(ddy) != ny * Fraction(u):
        return None
    m = g // 2
    cx, cy = q[0] - (m * (nx // g)) * u, q[1] - (m * (ny // g)) * u
    ex, ey = ray_end((cx, cy), r)
    C, E, Q = (Fraction(cx), Fraction(cy)), (Fraction(ex), Fraction(ey)), (Fraction(q[0]), Fraction(q[1]))
    if (E[0] - C[0]) * (Q[1] - C[1]) - (E[1] - C[1]) * (Q[0] - C[0]) != 0:
        return None
    t = (Q[0] - C[0]) / (E[0] - C[0])
    return (cx, cy) if 0 < t < 1 else None


class Batch:
    """Envs of N agents; agent 0 is the subject, the others fill in far away."""

    def __init__(self, N, W=32):
        self.N, self.W = N, W
        self.rows = []          # (family, variant, pos (N,2), pre_pos, vel, goal (N,2), wps (N,W,2), cnt (N,))

    def add(self, family, variant, subject, partner=None, goal=None, wp0=None, vel=None, pre=None, partner2=None):
        N, W = self.N, self.W
        pos = np.zeros((N, 2))
        for k in range(N):                           # fillers along the top, 12 m apart
            pos[k] = (468.0 + 12.0 * k, 378.0)
        pos[0] = subject
        if partner is not None:
            pos[1] = partner
        if partner2 is not None:
            pos[2] = partner2
        goals = pos + np.array([0.0, -100.0])
        goals[0] = goal if goal is not None else (470.0, 262.0)
        wps = np.repeat(goals[:, None, :], W, axis=1).copy()
        cnt = np.ones(N, np.int32)
        if wp0 is not None:
            wps[0, 0] = wp0
            cnt[0] = 2
        v = np.zeros((N, 2))
        if vel is not None:
            v[0] = vel
        pp = pos.copy()
        if pre is not None:
            pp[0] = pre
        self.rows.append((family, variant, pos, pp, v, goals, wps, cnt))

    def arrays(self):
        f = [r[0] for r in self.rows]
        v = [r[1] for r in self.rows]
        st = {k: np.stack([r[i] for r in self.rows]) for i, k in enumerate(("pos", "pre_pos", "vel", "goal", "wp", "cnt"), 2)}
        return f, v, st


def build(N, seed=0):
    """The threshold batch for N agents (N >= 2).  Returns (families, variants, state dict, occ)."""
    rng = np.random.default_rng(seed)
    B = Batch(N)
    hx, hy = HOME
    # ---- drone contact at exactly 5 m and the near band's ends, with 1-ulp neighbours
    for fam, (a, b) in (("drone", (3.0, 4.0)),):
        for sx, sy, swap in ((1, 1, False), (-1, 1, True), (1, -1, False), (-1, -1, True)):
            ox, oy = (b, a) if swap else (a, b)
            for u in (-1, 0, 1):
                B.add(fam, u, (hx, hy), partner=(_up(hx + sx * ox, u), hy + sy * oy))
    # ---- waypoint at exactly 5 m
    for ox, oy in ((3.0, 4.0), (-4.0, 3.0), (0.0, -5.0), (5.0, 0.0)):
        for u in (-1, 0, 1):
            B.add("wp", u, (hx, hy), wp0=(_up(hx + ox, u), hy + oy))
    # ---- goal on the Minkowski 64-gon's apothem / vertex directions
    apo = (PB + 1.0) * geos.APOTHEM_UNIT
    for k in rng.choice(64, size=6, replace=False):
        for fam, ang, rad in (("goal_apo", (k + 0.5) * math.pi / 32, apo), ("goal_vtx", k * math.pi / 32, PB + 1.0)):
            gx, gy = hx + rad * math.cos(ang), hy + rad * math.sin(ang)
            for u in (-2, -1, 0, 1, 2):
                B.add(fam, u, (hx, hy), goal=(_up(gx, u), gy))
    B.add("kat", 0, (534.12, 355.86), goal=(536.0, 356.0))
    B.add("kat", 1, (530.81, 353.08), goal=(536.0, 356.0))
    # ---- building: touching an isolated cell's edge / corner
    for i, j in CELLS:
        x0, x1, y0, y1 = square_of(i, j)
        cx, cy = (x0 + x1) / 2, (y0 + y1) / 2
        for u in (-1, 0, 1):
            B.add("bld_edge", u, (_up(x1 + PB, u), cy + 1.25))          # vertex 32 (px - 2.5) on x = x1
            B.add("bld_edge", u, (_up(x0 - PB, u), cy - 2.0))           # vertex 0 (px + 2.5) on x = x0
            B.add("bld_edge", u, (cx + 0.5, _up(y1 + PB, u)))           # vertex 16 on y = y1
            B.add("bld_edge", u, (cx - 3.0, _up(y0 - PB, u)))           # vertex 48 on y = y0
        for (qx, qy), k in (((x1, y1), 24), ((x0, y1), 8), ((x0, y0), 56), ((x1, y0), 40)):
            ang = -k * math.pi / 32      # the GEOS vertex k (angle -k pi/32) points from p at the corner q
            px, py = qx - PB * math.cos(ang), qy - PB * math.sin(ang)
            for u in (-1, 0, 1):
                B.add("bld_corner", u, (_up(px, u), py))
    # ---- bound lines: stationary circles and an axis-parallel move touching them
    for u in (-1, 0, 1):
        B.add("bound", u, (_up(BOUND[0] + PB, u), 300.0))
        B.add("bound", u, (_up(BOUND[1] - PB, u), 320.0))
        B.add("bound", u, (560.0, _up(BOUND[2] + PB, u)))
        B.add("bound", u, (590.0, _up(BOUND[3] - PB, u)))
        y = _up(BOUND[3] - PB, u)
        B.add("bound_move", u, (640.0, y), vel=(4.0, 0.0))              # -> (642, y): capsule top on 385
        x = _up(BOUND[1] - PB, u)
        B.add("bound_move", u, (x, 300.0), vel=(0.0, -4.0))             # -> (x, 298): capsule right on 680
    # ---- radar: rays through another agent's vertex, a start on its boundary
    for d in (4.0, 7.25, 11.5):
        for side in (1, -1):
            for u in (-1, 0, 1):
                B.add("tangent", u, (hx, hy), partner=(hx + d, _up(hy + side * PB, u)))      # 0-degree ray
                B.add("tangent", u, (hx, hy), partner=(hx - d, _up(hy + side * PB, u)))      # 180-degree ray
    for u in (-1, 0, 1):
        B.add("start_on", u, (hx, hy), partner=(_up(hx - PB, u), hy))
    # ---- radar: rays through an isolated cell's corner touching only that point -- rays of quadrants I
    # and III through the lower-right / upper-left corners, of quadrants II and IV through the lower-left
    # / upper-right ones pass the square outside both edges at the corner -- and rays along its top edge
    for i, j in CELLS:
        x0, x1, y0, y1 = square_of(i, j)
        for q, rays in (((x1, y0), (1, 2, 3, 4, 10, 11, 12, 13)), ((x0, y1), (1, 2, 3, 4, 10, 11, 12, 13)),
                        ((x0, y0), (5, 6, 7, 8, 14, 15, 16, 17)), ((x1, y1), (5, 6, 7, 8, 14, 15, 16, 17))):
            for r in rays:
                c = _corner_start(q, r)
                if c is not None:
                    for u in (-1, 0, 1):
                        B.add("corner", u, (c[0], _up(c[1], u)))
        for u in (-1, 0, 1):
            B.add("edge_run", u, (x0 - 6.0, _up(y1, u)))
            for d in (3.0, 4.5):
                B.add("edge_near", u, (x0 - d, _up(y1, u)))
                B.add("edge_near", u, (x0 - d, _up(y0, u)))
    fam, var, st = B.arrays()
    return fam, var, st, threshold_map()


def build_near(N):
    """The near-drone band's two ends made observable: the penalty of every in-band
    neighbour is m * shortest + c (ATT/env:2420-2432), 0 at shortest = 10, so a second neighbour sets the
    shortest distance.  Families: near10 (a neighbour at 6 m, the threshold one at 10 m = the 6-8-10
    offset, +-1 ulp) and near2.5 (a neighbour at 6 m, the threshold one at 2.5 m = 1.5-2-2.5, +-1 ulp: a
    drone contact too, whose branch still subtracts the penalty).  Needs N >= 3."""
    assert N >= 3
    B = Batch(N)
    hx, hy = HOME
    for fam, (a, b) in (("near10", (6.0, 8.0)), ("near2.5", (1.5, 2.0))):
        for sx, sy, swap in ((1, 1, False), (-1, 1, True), (1, -1, False), (-1, -1, True)):
            ox, oy = (b, a) if swap else (a, b)
            for u in (-2, -1, 0, 1, 2):
                B.add(fam, u, (hx, hy), partner=(_up(hx + sx * ox, u), hy + sy * oy), partner2=(hx, hy - sy * 6.0))
    fam, var, st = B.arrays()
    return fam, var, st, threshold_map()


def near_reward(pos, vmax=5.0):
    """The subject's own ss_reward (ATT/env:2315-2580; team reward off) for a stationary subject, from
    np.linalg.norm distances: the near-drone penalty of each neighbour with 2.5 <= d <= 10 uses the
    shortest distance (ATT/env:2425-2432); a contact (d <= 5) takes the drone branch (:2537-2545)."""
    ds = [float_norm(pos[0], pos[j]) for j in range(1, len(pos))]
    shortest = min(ds)
    c_drone, m_drone = 1 + (2.5 / (10 - 2.5)), (0 - 1) / (10 - 2.5)
    pen = 0.0
    for d in ds:
        pen = pen + (1 * (m_drone * shortest + c_drone)) if 2.5 <= d <= 10 else pen + 0
    dtg = (1 * (0.0)) / vmax
    return (((0.0 - 20) - 0.0) - pen) if any(d <= 2 * PB for d in ds) else dtg - pen


# ------------------------------------------------------------------ exact expectations (rationals)
def exact_goal(p, g):
    return geos.convex_polys_intersect_exact(geos.circle_vertices(p[0], p[1], PB), geos.circle_vertices(g[0], g[1], 1.0))


def exact_building(p, occ):
    A = geos.circle_vertices(p[0], p[1], PB)
    for i, j in zip(*np.nonzero(occ)):
        x0, x1, y0, y1 = square_of(i, j)
        if abs((x0 + x1) / 2 - p[0]) > 10 or abs((y0 + y1) / 2 - p[1]) > 10:
            continue
        if geos.convex_polys_intersect_exact(A, [(x0, y0), (x1, y0), (x1, y1), (x0, y1)]):
            return True
    return False


def exact_radar(c, others, occ, mode):
    """The 18 radar distances with every hit decided and located exactly (Fractions), rounded once."""
    out = []
    others = [q for q in others if math.hypot(q[0] - c[0], q[1] - c[1]) < 15.0 + PB + 1.0]
    cells = [(i, j) for i, j in zip(*np.nonzero(occ))
             if math.hypot(460.0 + 10 * i - c[0], 260.0 + 10 * j - c[1]) < 15.0 + 7.1 + 1.0]
    for r in range(18):
        e = ray_end(c, r)
        L = geos.point_dist(e[0], e[1], c[0], c[1])
        best_d = None
        if mode != 1:
            for q in others:
                t = geos.segment_convex_entry_exact(c, e, geos.circle_vertices(q[0], q[1], PB))
                if t is not None:
                    d = float(t) * L
                    best_d = d if best_d is None or d < best_d else best_d
        dd = best_d if best_d is not None else L
        best_o = None
        if mode != 0:
            for i, j in cells:
                x0, x1, y0, y1 = square_of(i, j)
                t = geos.ray_square_boundary_t_exact(c, e, x0, x1, y0, y1)
                if t is not None:
                    d = float(t) * L
                    best_o = d if best_o is None or d < best_o else best_o
            for axis, val in ((0, BOUND[0]), (0, BOUND[1]), (1, BOUND[2]), (1, BOUND[3])):
                t = geos.ray_line_t_exact(c, e, axis, val)
                if t is not None:
                    d = float(t) * L
                    best_o = d if best_o is None or d < best_o else best_o
        do = best_o if best_o is not None else L
        out.append(dd if mode == 0 else (do if mode == 1 else min(dd, do)))
    return np.array(out)


def float_norm(a, b):
    """np.linalg.norm of a 2-vector difference (the reference's form, ATT/env:2228-2236)."""
    return float(np.linalg.norm(np.asarray(a, dtype=np.float64) - np.asarray(b, dtype=np.float64)))


RADAR_FAMILIES = ("tangent", "start_on", "corner", "edge_run", "edge_near")


def check(families, variants, post, occ, mode, mask, radar, where=""):
    """The subject's integer outputs against the reference's own semantics at each threshold:
    np.linalg.norm / GEOS point distances where the reference compares float distances (drone, near,
    wp), the exact rational predicates on the GEOS float vertices where it asks GEOS (goal, building,
    bound, radar).  post: the post-step state dict (pos, pre_pos, goal, wp).  Returns {family: set of
    expected outcomes} (so callers can require both)."""
    seen = {}
    for e, fam in enumerate(families):
        p, q = post["pos"][e], post["pre_pos"][e]
        m = int(mask[e, 0])
        if fam == "drone":
            want = float_norm(p[0], p[1]) <= 2 * PB
            got = bool(m & 2)
        elif fam == "wp":
            w = post["wp"][e, 0, 0]
            want = geos.point_dist(p[0, 0], p[0, 1], w[0], w[1]) < 5
            got = bool(m & 16)
        elif fam in ("goal_apo", "goal_vtx", "kat"):
            want = exact_goal(p[0], post["goal"][e, 0])
            got = bool(m & 4)
        elif fam in ("bld_edge", "bld_corner"):
            want = exact_building(p[0], occ)
            got = bool(m & 8)
        elif fam in ("bound", "bound_move"):
            want = geos.bound_crash(q[0], p[0], BOUND)
            got = bool(m & 1)
        elif fam in RADAR_FAMILIES:
            ex = exact_radar(tuple(p[0]), [tuple(x) for x in p[1:]], occ, mode)
            np.testing.assert_allclose(radar[e, 0], ex, rtol=0, atol=1e-5, err_msg=f"{where} {fam} env {e} radar")
            want = got = bool((ex < 15.0 - 1e-6).any())
        else:
            raise KeyError(fam)
        assert want == got, (where, fam, variants[e], e, p[0].tolist(), want, got)
        seen.setdefault(fam, set()).add(want)
    return seen


def oracle_state(co, st):
    """Install a threshold batch's pre-step state in a c_oracle.BatchedOracle."""
    co.pos[:] = st["pos"]
    co.pre_pos[:] = st["pre_pos"]
    co.vel[:] = st["vel"]
    co.pre_vel[:] = st["vel"]
    co.goal[:] = st["goal"]
    co.wp[:] = st["wp"]
    co.wp_cnt[:] = st["cnt"]
    co.wp_cur[:] = 0
    co.reach[:] = 0
    co.wall[:] = 0
    co.step_count[:] = 0
    co.start[:] = st["pos"]
