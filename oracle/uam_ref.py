"""Reference-shaped scalar restatement of the UAM variant's environment (config 5).
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

``UAM/`` = ``MADDPG_ownENV_randomOD_radar_N_model_use_tdCPA_forV2_changeskin_UAM/`` (SURVEY.md
section 0); ``UAM/env`` is its ``env_simulator_*.py``, ``UAM/util`` its ``Utilities_own_*.py``,
``UAM/main`` its ``ma_main_*.py``.  One object per agent / cloud, per-agent loops, numpy and
``math`` exactly where the reference calls them.  Shapely/GEOS calls are replaced by the GEOS
construction of ``oracle.geos`` and predicates that are exact on those float vertices (closed
forms exact in real arithmetic, cross-checked by tests against exact rational arithmetic on the
float vertices (``*_exact``).

Followed line by line (default flags of UAM/main:60-100: training mode, evaluation flags off,
include_other_AC = True, full_observable_critic_flag = False, use_nearestN_neigh_wRadar = False):
  reset                  UAM/env:551-771 ``reset_world_change_skin``; start / end sampling
                         UAM/util:165-237; clouds UAM/cloud.py:11-49
  step                   UAM/env:4667-4904: clouds (UAM/util:41-51 update_cloud_target,
                         :300-318 calculate_next_position), then drone kinematics
  neighbours             UAM/env:1198-1230 ``get_current_agent_nei(queue=True)`` (sorted)
  radar                  UAM/env:1360-1486: runway boundary, 4 bound segments, cloud
                         boundaries, other aircraft's 64-gon boundaries; default ray length
  observation            UAM/env:1616-1880 (own 7, p2 neighbours 5 each, radar 18, p3 6 each)
  reward                 UAM/env:3892-4629 ``ss_reward_Mar_changeskin``
  termination            UAM/main:624-637

Canonical-contract choices: ``ActorNetwork_TwoPortion`` /
``critic_single_TwoPortion`` read [own, radar] (UAM/maddpg:445-554), so their radar encoders are
18 wide (the reference declares (N-1)*5, which cannot run: contract R1 again).  Bug-compatible
quirks kept: the reward coefficient doubling that persists over later agents of the same call
(UAM/env:4320, :4546), the host heading as the 5th neighbour feature (UAM/env:1765), the p3
"goal diff" read from the wrong slots (UAM/env:1782-1784), the near-building penalty of the
default ray length (UAM/env:4478).
"""
import math
import random
import numpy as np

from . import geos

# --------------------------------------------------------------------------- constants
BOUND = (0.0, 40.0, 0.0, 40.0)        # xlow, xhigh, ylow, yhigh               UAM/params:32-36
DT = 0.5                              # time_step                              UAM/env:552-553
ACC_MAX = 0.5                         # acc_max -> coe_a                       UAM/main:257, UAM/env:4672
VMAX = 1.0                            # max_spd -> Agent.maxSpeed               UAM/main:255, UAM/agent:29
PB = 0.5                              # Agent.protectiveBound                   UAM/agent:39
DETECTION_RANGE = 10                  # Agent.detectionRange (diameter)          UAM/agent:38
RADAR_DIST = DETECTION_RANGE / 2      # radar_dist                              UAM/env:1351
N_RAYS = 18                           # range(0, 360, 20)                       UAM/env:1346
RUNWAY = (18.0, 22.0, 10.0, 30.0)     # Polygon (18,10)-(22,30)                 UAM/env:559
GO_AC = ((20, 20, 20, 35, 5, 35, 5, 5, 20, 5, 20, 20),      # go_0..go_3             UAM/env:562-565
         (20, 20, 20, 5, 5, 5, 5, 35, 20, 35, 20, 20),
         (20, 20, 20, 35, 35, 35, 35, 5, 20, 5, 20, 20),
         (20, 20, 20, 5, 35, 5, 35, 35, 20, 35, 20, 20))
CLOUDS = ((8, 30, 10, 10), (30, 10, 35, 30))                # cloud_a, cloud_b       UAM/env:567-568
CLOUD_RADIUS = (3.0, 1.0)             # contour_range 3 / go-around AC radius 1   UAM/cloud.py:18,46
CLOUD_VEL = (0.4, 2.0)                # cloud vel / go-around AC vel             UAM/cloud.py:21,44
START_ZONES = ((15, 17, 15, 25), (23, 25, 15, 25))          # start_zone_1/2         UAM/env:573-575
SPAWN_CLOUD, SPAWN_BOUND = 5, 5       # spawn_threshold_cloud / _boundary        UAM/env:690-691
CRASH = 50.0                          # crash_penalty_wall                       UAM/env:3901
REACH = 50.0                          # reach_target                             UAM/env:3902
DIST_COEF = 5.0                       # dist_to_goal_coeff                       UAM/env:3903
NEAR_BUILDING_COEF = 2.0              # near_building_penalty_coef               UAM/env:3904
NEAR_DRONE_COEF = 2.0                 # near_drone_penalty_coef                  UAM/env:3905
NEAR_LO, NEAR_HI = 2.0, 5.0           # dist_to_penalty_lower/upperbound         UAM/env:4307-4308
TURNING_PT = 5.0                      # turningPtConst (c = 2)                   UAM/env:4470-4476
EPISODE_LENGTH = 150                  # --episode_length                         UAM/main:1222
GOAL_R = 1.0                          # Point(goal[-1]).buffer(1)                UAM/env:3933

X_SCALE = (1 - (-1)) / (BOUND[1] - BOUND[0])
Y_SCALE = (1 - (-1)) / (BOUND[3] - BOUND[2])

APO = geos.APOTHEM_UNIT
NORMALS = geos.edge_normal_table()


# --------------------------------------------------------------------------- NormalizeData
# UAM/util:1241-1310 with x/y_min_max = bound, spd_max = 1, acc_range = [-0.5, 0.5]
def nmlz_pos(p):
    return np.array([2 * ((p[0] - BOUND[0]) / (BOUND[1] - BOUND[0])) - 1,
                     2 * ((p[1] - BOUND[2]) / (BOUND[3] - BOUND[2])) - 1])


def nmlz_pos_diff(d):
    dx_min, dx_max = BOUND[0] - BOUND[1], BOUND[1] - BOUND[0]
    dy_min, dy_max = BOUND[2] - BOUND[3], BOUND[3] - BOUND[2]
    return (2 * ((d[0] - dx_min) / (dx_max - dx_min)) - 1, 2 * ((d[1] - dy_min) / (dy_max - dy_min)) - 1)


def nmlz_vel(v):
    return np.array([v[0] / VMAX, v[1] / VMAX])


def calculate_bearing(xh, yh, xi, yi):
    """UAM/util:321-334."""
    th = math.degrees(math.atan2(yi - yh, xi - xh))
    return -th if th < 0 else 360 - th


def compute_t_cpa_d_cpa_potential_col(other_pos, host_pos, other_vel, host_vel, other_bound, host_bound,
                                      total_possible_conf):
    """UAM/util:916-938: time / distance of closest approach of the host to one neighbour, and the
    running count of potential conflicts (CPA within one time unit closer than the two bounds).
    Zero relative velocity: tcpa = -10 and d = the distance after one time unit (counted once if
    it is inside the bounds; the [0, 1] test cannot fire for -10)."""
    rel_dist_with_neg = -1 * (other_pos - host_pos)
    rel_vel = other_vel - host_vel
    sq = np.square(np.linalg.norm(rel_vel))
    if sq == 0:
        tcpa = -10
        new_nei = other_pos + (other_vel * 1)
        new_host = host_pos + (host_vel * 1)
        d_tcpa = np.linalg.norm(new_host - new_nei)
        if d_tcpa < (other_bound + host_bound):
            total_possible_conf = total_possible_conf + 1
    else:
        tcpa = np.dot(rel_dist_with_neg, rel_vel) / sq
        d_tcpa = np.linalg.norm(((rel_dist_with_neg * -1) + (rel_vel * tcpa)))
    if (tcpa <= 1) and (tcpa >= 0) and (d_tcpa < (other_bound + host_bound)):
        total_possible_conf = total_possible_conf + 1
    return tcpa, d_tcpa, total_possible_conf


def calculate_next_position(start, target, speed, dt):
    """UAM/util:300-318."""
    direction = target - start
    dist = np.linalg.norm(direction)
    unit = np.zeros(2) if dist < 1 else direction / dist
    return start + unit * (speed * dt)


# --------------------------------------------------------------------------- GEOS predicates
def _gon(c, r):
    return geos.circle_vertices(float(c[0]), float(c[1]), float(r))


def _max_normal(dx, dy):
    return max(dx * nx + dy * ny for nx, ny in NORMALS)


def _exact_sat(A, B, strict):
    """Closed convex polygons A, B: strict=False -> they intersect (touching counts);
    strict=True -> their interiors intersect.  Exact rational separating-axis test."""
    A = [geos._fr(p) for p in A]
    B = [geos._fr(p) for p in B]
    for P in (A, B):
        n = len(P)
        for k in range(n):
            (x0, y0), (x1, y1) = P[k], P[(k + 1) % n]
            nx, ny = (y1 - y0), -(x1 - x0)
            pa = [nx * x + ny * y for x, y in A]
            pb = [nx * x + ny * y for x, y in B]
            if strict:
                if max(pa) <= min(pb) or max(pb) <= min(pa):
                    return False
            elif max(pa) < min(pb) or max(pb) < min(pa):
                return False
    return True


def gons_meet(c0, r0, c1, r1, strict=False):
    """GEOS 64-gon(c0, r0) vs 64-gon(c1, r1): ``intersects`` (strict=False) or interiors overlap,
    i.e. ``intersects and not touches`` (strict=True).  Both share the vertex angles k pi/32, so
    the Minkowski difference is the 64-gon of circumradius R = r0 + r1: max_k d.n_k vs
    R cos(pi/64).  Closed form, same arithmetic as ``gons_meet`` in csrc/aac_geom.h;
    ``gons_meet_exact`` is the independent check on the float vertices."""
    dx, dy = c1[0] - c0[0], c1[1] - c0[1]
    R = r0 + r1
    thr = R * APO
    dist = math.sqrt(dx * dx + dy * dy)
    if dist > R * (1.0 + 1e-12) + 1e-12:
        return False
    if dist < thr * (1.0 - 1e-12) - 1e-12:
        return True
    m = _max_normal(dx, dy)
    return m < thr if strict else m <= thr


def gons_meet_exact(c0, r0, c1, r1, strict=False):
    return _exact_sat(_gon(c0, r0), _gon(c1, r1), strict)


def gon_rect_overlap(c, r, rect):
    """Interiors of 64-gon(c, r) and the rectangle (x0, x1, y0, y1) overlap
    (``polygons_single_cloud_conflict``, UAM/util:291-297; the rectangle cannot lie within the
    0.5 circle).  Separating axes: the rectangle's (the 64-gon reaches r along x / y) and the 32
    distinct 64-gon edge normals (reach r cos(pi/64)); touching is no overlap.  Same arithmetic
    as ``gon_rect_overlap`` in csrc/aac_uam.hip; ``gon_rect_overlap_exact`` checks it."""
    x0, x1, y0, y1 = rect
    hx, hy = (x1 - x0) / 2, (y1 - y0) / 2
    dx, dy = (x0 + x1) / 2 - c[0], (y0 + y1) / 2 - c[1]
    if abs(dx) >= hx + r or abs(dy) >= hy + r:
        return False
    ox, oy = max(abs(dx) - hx, 0.0), max(abs(dy) - hy, 0.0)
    dist = math.sqrt(ox * ox + oy * oy)
    if dist > r * (1.0 + 1e-12) + 1e-12:
        return False
    if dist < r * APO * (1.0 - 1e-12) - 1e-12:
        return True
    for nx, ny in NORMALS[:32]:
        if abs(dx * nx + dy * ny) >= hx * abs(nx) + hy * abs(ny) + r * APO:
            return False
    return True


def gon_rect_overlap_exact(c, r, rect):
    x0, x1, y0, y1 = rect
    return _exact_sat(_gon(c, r), [(x0, y0), (x0, y1), (x1, y1), (x1, y0)], True)


def _seg_hits(c, e, ring):
    """Nearest intersection of segment c->e with the closed polyline ``ring`` (GEOS
    ``LineString.intersection(polygon.boundary)`` + ``LineString([c, p]).length``), or None.
    Parallel edges (collinear overlaps, measure zero) are skipped, as the reference skips
    non-point results."""
    best = None
    dx, dy = e[0] - c[0], e[1] - c[1]
    n = len(ring)
    for k in range(n):
        v, w = ring[k], ring[(k + 1) % n]
        ex, ey = w[0] - v[0], w[1] - v[1]
        den = dx * ey - dy * ex
        if den == 0.0:
            continue
        qx, qy = v[0] - c[0], v[1] - c[1]
        t = (qx * ey - qy * ex) / den
        s = (qx * dy - qy * dx) / den
        if 0.0 <= t <= 1.0 and 0.0 <= s <= 1.0:
            d = geos.point_dist(c[0] + t * dx, c[1] + t * dy, c[0], c[1])
            if best is None or d < best:
                best = d
    return best


def _seg_gon(c, e, p, r):
    # exact pre-filter: the 64-gon lies within the circle of radius r (1 + 1e-15) around p
    dx, dy = e[0] - c[0], e[1] - c[1]
    wx, wy = p[0] - c[0], p[1] - c[1]
    tt = (wx * dx + wy * dy) / (dx * dx + dy * dy)
    tt = min(max(tt, 0.0), 1.0)
    qx, qy = tt * dx - wx, tt * dy - wy
    if qx * qx + qy * qy > (r + 1e-6) ** 2:
        return None
    return _seg_hits(c, e, _gon(p, r))


def _seg_seg(c, e, a, b):
    """Segment c->e vs segment a-b (the 4 bound LineStrings, UAM/env:594-598): point distance."""
    dx, dy = e[0] - c[0], e[1] - c[1]
    ex, ey = b[0] - a[0], b[1] - a[1]
    den = dx * ey - dy * ex
    if den == 0.0:
        return None
    qx, qy = a[0] - c[0], a[1] - c[1]
    t = (qx * ey - qy * ex) / den
    s = (qx * dy - qy * dx) / den
    if 0.0 <= t <= 1.0 and 0.0 <= s <= 1.0:
        return geos.point_dist(c[0] + t * dx, c[1] + t * dy, c[0], c[1])
    return None


# --------------------------------------------------------------------------- agents / clouds
class Agent:
    """Attributes of UAM/agent:14-59 the hot path reads or writes."""

    def __init__(self, idx):
        self.agent_name = "agent_%s" % idx
        self.pos = self.pre_pos = self.ini_pos = None
        self.vel = self.pre_vel = None
        self.acc = np.zeros(2)
        self.goal = None
        self.waypoints = None
        self.heading = None
        self.maxSpeed = VMAX
        self.protectiveBound = PB
        self.detectionRange = DETECTION_RANGE
        self.surroundingNeighbor = {}
        self.pre_surroundingNeighbor = {}
        self.observableSpace = []
        self.reach_target = False
        self.bound_collision = self.cloud_collision = self.drone_collision = False


class Cloud:
    """UAM/cloud.py:11-49; cloud 0 drifts to its goal, cloud 1 is the go-around aircraft."""

    def __init__(self, idx, setting):
        self.radius = CLOUD_RADIUS[idx]
        self.vel = CLOUD_VEL[idx]
        self.pos = np.array([float(setting[0]), float(setting[1])])
        self.pre_pos = self.pos.copy()
        self.goal = np.array([float(setting[2]), float(setting[3])])
        self.path = None
        self.target = None
        if len(setting) > 4:
            self.path = [(float(setting[i]), float(setting[i + 1])) for i in range(0, len(setting), 2)]
            self.target = 1


def preset_target_index(path, t):
    """``cloud_path.index(cloud.previous_target)`` (UAM/util:45): the FIRST equal point."""
    return path.index(path[t])


# --------------------------------------------------------------------------- OD sampling
def no_spawn_zones(cloud0):
    """UAM/env:683-707 (the aerodrome / start-zone entries are discarded by ``no_spawn_zone = []``)."""
    z = []
    for s in (CLOUDS[cloud0], GO_AC[0]):
        z.append((s[0] - SPAWN_CLOUD, s[0] + SPAWN_CLOUD, s[1] - SPAWN_CLOUD, s[1] + SPAWN_CLOUD))
    b = BOUND
    z += [(b[0], b[1], b[2], b[2] + SPAWN_BOUND), (b[0], b[1], b[3] - SPAWN_BOUND, b[3]),
          (b[0], b[0] + SPAWN_BOUND, b[2], b[3]), (b[1] - SPAWN_BOUND, b[1], b[2], b[3])]
    return z


def end_regions(cloud0, x_start):
    """The region subtraction of ``generate_random_end_pos`` (UAM/util:188-232), filtered to the
    start's side of the runway."""
    regions = [(BOUND[0], BOUND[1], BOUND[2], BOUND[3])]
    for nx0, nx1, ny0, ny1 in no_spawn_zones(cloud0):
        new = []
        for rx0, rx1, ry0, ry1 in regions:
            if rx0 < nx1 and rx1 > nx0 and ry0 < ny1 and ry1 > ny0:
                if rx0 < nx0:
                    new.append((rx0, nx0, ry0, ry1))
                if rx1 > nx1:
                    new.append((nx1, rx1, ry0, ry1))
                if ry0 < ny0:
                    new.append((max(rx0, nx0), min(rx1, nx1), ry0, ny0))
                if ry1 > ny1:
                    new.append((max(rx0, nx0), min(rx1, nx1), ny1, ry1))
            else:
                new.append((rx0, rx1, ry0, ry1))
        regions = new
    if x_start < RUNWAY[0]:
        return [r for r in regions if r[1] <= RUNWAY[0]]
    return [r for r in regions if r[0] >= RUNWAY[1]]


def sample_episode(N, py_rng, np_rng):
    """One episode's draws in the reference's order (UAM/env:575-747): cloud choices, then per
    agent the (unused) pool indices, start (re-drawn until > 3 pB from earlier starts) and end.
    ``py_rng`` stands for Python ``random``, ``np_rng`` (RandomState) for ``np.random``."""
    c0 = py_rng.choice(range(len(CLOUDS)))
    c1 = py_rng.choice(range(len(GO_AC)))
    starts, goals = [], []
    for _ in range(N):
        k = py_rng.randint(0, 3)
        py_rng.choice(list(range(0, k)) + list(range(k + 1, 4)))

        def draw():
            z = py_rng.choice(START_ZONES)
            return [np_rng.uniform(z[0], z[1]), np_rng.uniform(z[2], z[3])]
        s = draw()
        if starts:
            while len(starts) < N:
                s = draw()
                if all(np.linalg.norm(np.array(s) - p) > PB * 3 for p in starts):
                    break
        regs = end_regions(c0, s[0])
        r = regs[np_rng.randint(0, len(regs))]
        g = [np_rng.uniform(r[0], r[1]), np_rng.uniform(r[2], r[3])]
        starts.append(np.array(s))
        goals.append(g)
    return np.array(starts), np.array(goals), c0, c1


# --------------------------------------------------------------------------- environment
class UAMEnv:
    """One UAM environment instance with N aircraft, reference-shaped."""

    def __init__(self, N, episode_length=EPISODE_LENGTH):
        self.N = N
        self.episode_length = episode_length
        self.all_agents = {i: Agent(i) for i in range(N)}
        self.step_count = 0
        b = BOUND
        self.boundaries = [((b[0], b[2]), (b[0], b[3])), ((b[1], b[2]), (b[1], b[3])),
                           ((b[0], b[3]), (b[1], b[3])), ((b[0], b[2]), (b[1], b[2]))]   # UAM/env:594-598
        x0, x1, y0, y1 = RUNWAY
        self.runway_ring = [(x0, y0), (x0, y1), (x1, y1), (x1, y0)]
        self.clouds = []
        self.stats = None

    def reset(self, starts, goals, cloud0, cloud1):
        """State part of ``reset_world_change_skin`` (UAM/env:551-771) for drawn OD + clouds."""
        self.clouds = [Cloud(0, CLOUDS[cloud0]), Cloud(1, GO_AC[cloud1])]
        for i, ag in self.all_agents.items():
            s = np.array(starts[i], dtype=float)
            g = [float(goals[i][0]), float(goals[i][1])]
            ag.pos, ag.pre_pos, ag.ini_pos = s.copy(), s.copy(), s.copy()
            ag.reach_target = False
            ag.bound_collision = ag.cloud_collision = ag.drone_collision = False
            ag.goal = [g]
            ag.waypoints = [list(g)]
            ag.heading = math.atan2(ag.goal[0][1] - ag.pos[1], ag.goal[0][0] - ag.pos[0])
            ag.vel = np.array([0 * math.cos(ag.heading), 0 * math.sin(ag.heading)])
            ag.pre_vel = ag.vel.copy()
        self.step_count = 0
        return self.observe()

    # ------------------------------------------------------------------ step (UAM/env:4667-4904)
    def step(self, actions):
        for c in self.clouds:
            c.pre_pos = c.pos.copy()
            start = np.array([c.pos[0], c.pos[1]])
            if c.path is not None:
                # corridor = LineString([pre_pos, pos]).buffer(radius) is the 64-gon at pos
                # (zero length); target zone = target.buffer(0.5)   (UAM/util:41-51)
                if gons_meet(c.pos, c.radius, c.path[c.target], 0.5):
                    c.target = (preset_target_index(c.path, c.target) + 1) % len(c.path)
                target = np.array(c.path[c.target])
            else:
                target = c.goal
            c.pos = calculate_next_position(start, target, c.vel, DT)
        coe_a = ACC_MAX
        for (idx, ag), act in zip(self.all_agents.items(), actions):
            ag.pre_surroundingNeighbor = dict(ag.surroundingNeighbor)
            ag.pre_pos = ag.pos.copy()
            ag.pre_vel = ag.vel.copy()
            ax, ay = act[0] * coe_a, act[1] * coe_a
            ag.acc = np.array([ax, ay])
            cvx = ag.vel[0] + ax * DT
            cvy = ag.vel[1] + ay * DT
            nh = math.atan2(cvy, cvx)
            if np.linalg.norm([cvx, cvy]) >= ag.maxSpeed:
                ag.vel = np.array([ag.maxSpeed * math.cos(nh), ag.maxSpeed * math.sin(nh)])
            else:
                ag.vel = np.array([cvx, cvy])
            if ag.reach_target:
                dx = dy = 0
            else:
                dx = ag.vel[0] * DT
                dy = ag.vel[1] * DT
            h = math.atan2(dy, dx)
            if not ag.reach_target:
                ag.heading = h
            ag.pos = np.array([ag.pos[0] + dx, ag.pos[1] + dy])
        return self.observe()

    # ------------------------------------------------------------------ observation
    def neighbours(self, cur):
        """get_current_agent_nei(queue=True) (UAM/env:1198-1230): stable sort by distance."""
        lst = []
        for j, ag in self.all_agents.items():
            if ag.agent_name == cur.agent_name:
                continue
            d = np.linalg.norm(ag.pos - cur.pos)
            if d < 10000:
                lst.append((d, j, np.array([ag.pos[0], ag.pos[1], ag.vel[0], ag.vel[1], ag.protectiveBound])))
                lst.sort(key=lambda x: x[0])
        return {j: v for _, j, v in lst}

    def radar(self, i):
        """UAM/env:1360-1486: min over the runway boundary, the 4 bound segments, the clouds'
        boundaries and the other aircraft's 64-gon boundaries; default = the ray's length."""
        ag = self.all_agents[i]
        c = (float(ag.pos[0]), float(ag.pos[1]))
        out = []
        for deg in range(0, 360, 20):
            e = (c[0] + RADAR_DIST * math.cos(math.radians(deg)), c[1] + RADAR_DIST * math.sin(math.radians(deg)))
            best = geos.point_dist(e[0], e[1], c[0], c[1])
            d = _seg_hits(c, e, self.runway_ring)
            if d is not None and d < best:
                best = d
            for a, b in self.boundaries:
                d = _seg_seg(c, e, a, b)
                if d is not None and d < best:
                    best = d
            for cl in self.clouds:
                d = _seg_gon(c, e, cl.pos, cl.radius)
                if d is not None and d < best:
                    best = d
            for j, other in self.all_agents.items():
                if j == i:
                    continue
                d = _seg_gon(c, e, other.pos, ag.protectiveBound)
                if d is not None and d < best:
                    best = d
            out.append(best)
        return np.array(out)

    def observe(self):
        """cur_state_norm_state_v3 (UAM/env:1294-1919): normalised (own, p2, radar, p3).
        The tdCPA values of UAM/env:1738-1745 (current state, and ``pre_pos`` / ``pre_vel``) are
        kept in ``self.tdcpa_out`` = (tcpa[N][K], dcpa[N][K], conf_cur[N], conf_pre[N]) in the
        sorted neighbour order; ``ss_reward`` recomputes the same values from the same state and
        neighbour dict (UAM/env:4001-4010), so one copy serves both call sites."""
        own, p2, rad, p3 = [], [], [], []
        tc_all, dc_all, cc_all, cp_all = [], [], [], []
        for i, ag in self.all_agents.items():
            ag.surroundingNeighbor = self.neighbours(ag)
            ag.observableSpace = self.radar(i)
            norm_pos = nmlz_pos([ag.pos[0], ag.pos[1]])
            norm_vel = nmlz_vel([ag.vel[0], ag.vel[1]])
            norm_G = nmlz_pos([ag.goal[-1][0], ag.goal[-1][1]])
            o = np.append(np.concatenate([norm_pos, norm_vel, norm_G - norm_pos]), ag.heading)
            nb, n3 = [], []
            cc = cp = 0
            tcs, dcs = [], []
            for j, other in ag.surroundingNeighbor.items():
                oa = self.all_agents[j]
                tc, dc, cc = compute_t_cpa_d_cpa_potential_col(oa.pos, ag.pos, oa.vel, ag.vel,
                                                               oa.protectiveBound, ag.protectiveBound, cc)
                _, _, cp = compute_t_cpa_d_cpa_potential_col(oa.pre_pos, ag.pre_pos, oa.pre_vel, ag.pre_vel,
                                                             oa.protectiveBound, ag.protectiveBound, cp)
                tcs.append(float(tc))
                dcs.append(float(dc))
                norm_delta = norm_pos - nmlz_pos([oa.pos[0], oa.pos[1]])
                nb.append(np.append(np.concatenate([norm_delta, nmlz_vel([oa.vel[0], oa.vel[1]])]), ag.heading))
                npd = nmlz_pos_diff([other[0] - ag.pos[0], other[1] - ag.pos[1]])
                ngd = nmlz_pos_diff([other[-2] - other[0], other[-1] - other[1]])
                nv = tuple(nmlz_vel([other[2], other[3]]))
                n3.append(np.array(list(npd + ngd + nv)))
            own.append(o)
            p2.append(np.concatenate(nb))
            rad.append(ag.observableSpace.copy())
            p3.append(np.array(n3))
            tc_all.append(tcs)
            dc_all.append(dcs)
            cc_all.append(cc)
            cp_all.append(cp)
        self.tdcpa_out = (np.array(tc_all), np.array(dc_all), np.array(cc_all, dtype=np.int32),
                          np.array(cp_all, dtype=np.int32))
        return np.array(own), np.array(p2), np.array(rad), np.array(p3)

    # ------------------------------------------------------------------ reward
    def ss_reward(self):
        """ss_reward_Mar_changeskin (UAM/env:3892-4629), training mode, individual rewards.
        Returns reward[N], done[N], check_goal[N], bbc[4], mask[N] (bit0 bound, bit1 cloud /
        runway, bit2 drone collision, bit3 goal touch, bit4 goal branch, bit5 previous-nearest-two)."""
        N = self.N
        crash = CRASH
        ndc = NEAR_DRONE_COEF
        bbc = [False] * 4
        reward, done, check_goal, mask = [], [], [False] * N, []
        for i, ag in self.all_agents.items():                                   # UAM/env:3929-3936
            if gons_meet(ag.pos, ag.protectiveBound, ag.goal[-1], GOAL_R):
                ag.reach_target = True
        c_drone = 1 + (NEAR_LO / (NEAR_HI - NEAR_LO))
        m_drone = (0 - 1) / (NEAR_HI - NEAR_LO)
        for i, ag in self.all_agents.items():
            collision = []
            nearest, shortest, bearing, coll_bearing = None, math.inf, None, None
            for j in ag.surroundingNeighbor:                                    # UAM/env:4001-4083
                other = self.all_agents[j]
                diff = ag.pos - other.pos
                d = np.linalg.norm(diff)
                if d < shortest:
                    shortest = d
                    bearing = calculate_bearing(ag.pos[0], ag.pos[1], other.pos[0], other.pos[1])
                    nearest = j
                if np.linalg.norm(diff) <= ag.protectiveBound * 2:
                    if not (other.reach_target or ag.reach_target):
                        coll_bearing = calculate_bearing(ag.pos[0], ag.pos[1], other.pos[0], other.pos[1])
                        collision.append(j)
                        ag.drone_collision = True
            prev_two = 0                                                        # UAM/env:4084-4093
            for cnt, j in enumerate(ag.pre_surroundingNeighbor):
                if j in collision:
                    prev_two = 1
                    break
                if cnt + 1 > 1:
                    break
            cloud = 0                                                           # UAM/env:4095-4115
            if not ag.reach_target:
                if gon_rect_overlap(ag.pos, ag.protectiveBound, RUNWAY):
                    cloud = 1
                for cl in self.clouds:
                    if gons_meet(ag.pos, ag.protectiveBound, cl.pos, cl.radius, strict=True):
                        cloud = 1
                        break
            if cloud:
                ag.cloud_collision = True
            goal = gons_meet(ag.pos, ag.protectiveBound, ag.goal[-1], GOAL_R)
            # dist_to_goal = 5 (1 - total_length_to_end_of_line / L)            UAM/env:4202-4208
            s, g = ag.ini_pos, np.array(ag.goal[0])
            L = geos.point_dist(g[0], g[1], s[0], s[1])
            ddx, ddy = g[0] - s[0], g[1] - s[1]
            fr = ((ag.pos[0] - s[0]) * ddx + (ag.pos[1] - s[1]) * ddy) / (ddx * ddx + ddy * ddy)
            fr = min(max(fr, 0.0), 1.0)
            near = (s[0] + fr * ddx, s[1] + fr * ddy)
            left = geos.point_dist(ag.pos[0], ag.pos[1], near[0], near[1]) + (L - fr * L)
            dist_to_goal = DIST_COEF * (1 - (left / L))
            if nearest is not None and NEAR_LO <= shortest <= NEAR_HI:          # UAM/env:4311-4327
                if 90.0 <= bearing <= 180:
                    ndc = ndc * 2
                near_drone = ndc * (m_drone * shortest + c_drone)
            else:
                near_drone = ndc * 0
            min_dist = float(np.min(ag.observableSpace))                        # UAM/env:4466-4481
            m = (0 - 1) / (TURNING_PT - ag.protectiveBound)
            if ag.protectiveBound <= min_dist <= TURNING_PT:
                near_building = NEAR_BUILDING_COEF * (m * min_dist + 2)
            else:
                near_building = 0
            bnd = geos.bound_crash(ag.pre_pos, ag.pos, BOUND, ag.protectiveBound)
            mk = int(bnd) | (cloud << 1) | ((len(collision) > 0) << 2) | (int(goal) << 3)
            if bnd:                                                             # UAM/env:4488-4601
                ag.bound_collision = True
                rew = 0 - crash
                done.append(True)
                bbc[0] = True
            elif cloud == 1:
                done.append(True)
                bbc[1] = True
                rew = 0 - crash
            elif collision:
                done.append(True)
                bbc[2] = True
                if 90.0 <= coll_bearing <= 180:
                    crash = crash * 2
                rew = 0 - crash
                if prev_two:
                    bbc[3] = True
                    mk |= 32
            elif goal:
                ag.reach_target = True
                check_goal[i] = True
                rew = 0 + REACH + 0
                done.append(False)
                mk |= 16
            else:
                rew = 0 + dist_to_goal - near_building - near_drone
                done.append(False)
            reward.append(rew)
            mask.append(mk)
        return np.array(reward), np.array(done), np.array(check_goal), np.array(bbc), np.array(mask, dtype=np.uint8)

    def episode_over(self, done):
        """UAM/main:624-637 (step already incremented)."""
        return (self.episode_length < self.step_count or any(done)
                or all(a.reach_target for a in self.all_agents.values()))

    def full_step(self, actions):
        obs = self.step(actions)
        r, d, cg, bbc, mk = self.ss_reward()
        self.step_count += 1
        return obs, r, d, cg, bbc, mk, self.episode_over(d)

    def cloud_state(self):
        return [(c.pos.copy(), c.pre_pos.copy(), c.target) for c in self.clouds]


def env_from_state(s, e, N, episode_length=EPISODE_LENGTH):
    """A ``UAMEnv`` holding env ``e`` of a device state dict (``BatchedUAM.get_state`` as numpy):
    used to check one device step from an identical pre-step state."""
    env = UAMEnv(N, episode_length)
    kinds = s["cloud_kind"][e]
    env.clouds = [Cloud(0, CLOUDS[int(kinds[0])]), Cloud(1, GO_AC[int(kinds[1])])]
    for k, c in enumerate(env.clouds):
        c.pos = np.array(s["clouds"][e, k], dtype=float)
        c.pre_pos = c.pos.copy()
    env.clouds[1].target = int(s["cloud_tgt"][e])
    for i, ag in env.all_agents.items():
        ag.pos = np.array(s["pos"][e, i], dtype=float)
        ag.vel = np.array(s["vel"][e, i], dtype=float)
        ag.pre_pos = np.array(s["pre_pos"][e, i], dtype=float)
        ag.pre_vel = np.array(s["pre_vel"][e, i], dtype=float)
        ag.ini_pos = np.array(s["start"][e, i], dtype=float)
        g = [float(s["goal"][e, i, 0]), float(s["goal"][e, i, 1])]
        ag.goal, ag.waypoints = [g], [list(g)]
        ag.heading = float(s["heading"][e, i])
        ag.reach_target = bool(s["reach"][e, i])
        first = [int(j) for j in s["top2"][e, i] if int(j) != 255]
        ag.surroundingNeighbor = {j: None for j in first + [j for j in range(N) if j != i and j not in first]}
    env.step_count = int(s["step"][e])
    return env


def state_of(env):
    """The device state layout of one ``UAMEnv`` (numpy, one env)."""
    N = env.N
    ags = [env.all_agents[i] for i in range(N)]
    top2 = np.full((N, 2), 255, dtype=np.uint8)
    for i, ag in enumerate(ags):
        keys = list(ag.surroundingNeighbor)[:2]
        top2[i, :len(keys)] = keys
    return dict(pos=np.array([a.pos for a in ags]), vel=np.array([a.vel for a in ags]),
                pre_pos=np.array([a.pre_pos for a in ags]), pre_vel=np.array([a.pre_vel for a in ags]),
                goal=np.array([a.goal[-1] for a in ags], dtype=float), start=np.array([a.ini_pos for a in ags]),
                heading=np.array([a.heading for a in ags]), reach=np.array([a.reach_target for a in ags], dtype=np.uint8),
                clouds=np.array([c.pos for c in env.clouds]), cloud_tgt=np.int32(env.clouds[1].target),
                step=np.int32(env.step_count), top2=top2)
