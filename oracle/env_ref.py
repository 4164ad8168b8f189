"""Reference-shaped scalar restatement of the ``one_model_att`` environment step.
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

One Python object per agent, per-agent loops, ``np.linalg.norm`` / ``np.dot`` /
``math.atan2|cos|sin`` exactly where the reference calls them, so its arithmetic
is the reference's arithmetic.  Shapely/GEOS calls are replaced by the GEOS
construction + closed-form predicates of ``oracle.geos``.

Followed line by line:
  kinematics             ATT/env:2627-2713 (``step``)
  neighbours             ATT/env:758-773   (``get_current_agent_nei``)
  radar                  ATT/env:1051-1170 (drones), OM/env:1049-1148 (obstacles),
                         ATT/env:879-1048 (combined, min of both -- contract R6)
  observation            ATT/env:1285-1296, :1357-1469; NormalizeData ATT/util:554-607
  tdCPA                  ATT/util:308-329 (called ATT/env:1384-1391, :2189-2196)
  predicates + reward    ATT/env:2105-2618 (``ss_reward``)
  termination            ATT/main:448-462

Canonical-contract choices: D0 = 6+4(N-1) (R1); neighbour
tensor (K, 6) (R2); bug-compatible quirks kept when ``compat`` is True (R7).
"""
import math

import numpy as np

from . import geos
from .consts import (ACC_MAX, BOUND, CRASH_PENALTY, DT, GRID_LEN, NEAR_HI, NEAR_LO, PB,
                     RADAR_DIST, REACH_REWARD, VMAX, WP_REACH, X_SCALE, Y_SCALE, EPISODE_LENGTH)

RADAR_DRONES, RADAR_OBSTACLES, RADAR_COMBINED = 0, 1, 2


class Agent:
    """The attributes of ATT/agent:14-55 that the hot path reads or writes."""

    def __init__(self, idx):
        self.agent_name = "agent_%s" % idx
        self.pos = None
        self.pre_pos = None
        self.ini_pos = None
        self.vel = None
        self.pre_vel = None
        self.acc = np.zeros(2)
        self.goal = None
        self.waypoints = None
        self.protectiveBound = PB
        self.maxSpeed = VMAX
        self.observableSpace = []
        self.surroundingNeighbor = {}
        self.reach_target = False
        self.collide_wall_count = 0
        self.removed_goal = None


# NormalizeData (ATT/util:554-607), bound = [455, 680, 255, 385]
def scale_pos(p):
    return np.array([-1 + (p[0] - BOUND[0]) * X_SCALE, -1 + (p[1] - BOUND[2]) * Y_SCALE])


def nmlz_pos(p):
    return (2 * ((p[0] - BOUND[0]) / (BOUND[1] - BOUND[0])) - 1,
            2 * ((p[1] - BOUND[2]) / (BOUND[3] - BOUND[2])) - 1)


def norm_scale(d):
    return np.array([X_SCALE * d[0], Y_SCALE * d[1]])


def nmlz_pos_diff(d):
    dx_min = BOUND[0] - BOUND[1]
    dx_max = BOUND[1] - BOUND[0]
    dy_min = BOUND[2] - BOUND[3]
    dy_max = BOUND[3] - BOUND[2]
    return (2 * ((d[0] - dx_min) / (dx_max - dx_min)) - 1,
            2 * ((d[1] - dy_min) / (dy_max - dy_min)) - 1)


def nmlz_vel(v):
    return np.array([v[0] / VMAX, v[1] / VMAX])


def compute_t_cpa_d_cpa_potential_col(other_pos, host_pos, other_vel, host_vel, other_bound, host_bound, total):
    """ATT/util:308-329, verbatim arithmetic."""
    rel_dist_withNeg = -1 * (other_pos - host_pos)
    rel_vel = other_vel - host_vel
    rel_vel_norm_withSQ = np.square(np.linalg.norm(rel_vel))
    if rel_vel_norm_withSQ == 0:
        tcpa = -10
        new_nei_pos = other_pos + (other_vel * 1)
        new_host_pos = host_pos + (host_vel * 1)
        d_tcpa = np.linalg.norm(new_host_pos - new_nei_pos)
        if d_tcpa < (other_bound + host_bound):
            total = total + 1
    else:
        tcpa = np.dot(rel_dist_withNeg, rel_vel) / rel_vel_norm_withSQ
        d_tcpa = np.linalg.norm(((rel_dist_withNeg * -1) + (rel_vel * tcpa)))
    if (tcpa <= 1) and (tcpa >= 0) and (d_tcpa < (other_bound + host_bound)):
        total = total + 1
    return tcpa, d_tcpa, total


class ScalarEnv:
    """Single environment instance with N agents, reference-shaped."""

    def __init__(self, n_agents, occ, radar_mode=RADAR_DRONES, compat=True, episode_length=EPISODE_LENGTH):
        self.N = n_agents
        self.occ = np.asarray(occ, dtype=np.uint8)      # (23, 13) x-major, 1 = occupied
        self.radar_mode = radar_mode
        self.compat = compat
        self.episode_length = episode_length
        self.all_agents = {i: Agent(i) for i in range(n_agents)}
        self.step_count = 0
        w, h = self.occ.shape
        self.cells = []   # occupied squares (x0, x1, y0, y1), ATT/grid:174-180
        for i in range(w):
            for j in range(h):
                if self.occ[i, j]:
                    cx = (i + math.ceil(BOUND[0] / GRID_LEN)) * GRID_LEN
                    cy = (j + math.ceil(BOUND[2] / GRID_LEN)) * GRID_LEN
                    self.cells.append((float(cx), float(cy)))
        self.tdcpa = None

    # ------------------------------------------------------------------ reset
    def reset(self, starts, goal_lists):
        """State part of ``reset_world`` (ATT/env:292-372) for an already-drawn OD."""
        for i, ag in self.all_agents.items():
            ag.pos = np.array(starts[i], dtype=float)
            ag.pre_pos = np.array(starts[i], dtype=float)
            ag.ini_pos = np.array(starts[i], dtype=float)
            ag.removed_goal = None
            ag.reach_target = False
            ag.collide_wall_count = 0
            ag.goal = [list(g) for g in goal_lists[i]]
            ag.waypoints = [list(g) for g in goal_lists[i]]
            ag.vel = np.array([0.0, 0.0])
            ag.pre_vel = np.array([0.0, 0.0])
        self.step_count = 0
        return self.cur_state_norm_state_v3()

    # ------------------------------------------------------------------ step
    def step(self, actions, acc_max=ACC_MAX):
        """ATT/env:2627-2720."""
        coe_a = acc_max
        for (idx, ag), act in zip(self.all_agents.items(), actions):
            ag.pre_pos = ag.pos.copy()
            ag.pre_vel = ag.vel.copy()
            ax, ay = act[0], act[1]
            ax = ax * coe_a
            ay = ay * coe_a
            ag.acc = np.array([ax, ay])
            cvx = ag.vel[0] + ax * DT
            cvy = ag.vel[1] + ay * DT
            nh = math.atan2(cvy, cvx)
            if np.linalg.norm([cvx, cvy]) >= ag.maxSpeed:
                ag.vel = np.array([ag.maxSpeed * math.cos(nh), ag.maxSpeed * math.sin(nh)])
            else:
                ag.vel = np.array([cvx, cvy])
            dx = ag.vel[0] * DT
            dy = ag.vel[1] * DT
            ag.pos = np.array([ag.pos[0] + dx, ag.pos[1] + dy])
        return self.cur_state_norm_state_v3()

    def get_current_agent_nei(self, cur):
        for j, ag in self.all_agents.items():
            if ag.agent_name == cur.agent_name:
                continue
            if np.linalg.norm(ag.pos - cur.pos) <= 10000:
                cur.surroundingNeighbor[j] = np.array([ag.pos[0], ag.pos[1], ag.vel[0], ag.vel[1], ag.protectiveBound])
        return cur.surroundingNeighbor

    # radar ------------------------------------------------------------------
    def _ray_end(self, c, deg):
        return (c[0] + RADAR_DIST * math.cos(math.radians(deg)),
                c[1] + RADAR_DIST * math.sin(math.radians(deg)))

    def _radar_drones(self, i, c, e, length):
        shortest = math.inf
        out = length
        for j, other in self.all_agents.items():
            if j == i:
                continue
            poly = geos.circle_vertices(other.pos[0], other.pos[1], self.all_agents[i].protectiveBound)
            t = geos.ray_polygon_entry(c[0], c[1], e[0], e[1], poly)
            if t is None:
                continue
            px = c[0] + t * (e[0] - c[0])
            py = c[1] + t * (e[1] - c[1])
            d = geos.point_dist(px, py, c[0], c[1])
            if d < shortest:
                shortest = d
                out = d
        return out

    def _radar_obstacles(self, c, e, length):
        min_d = length
        for cx, cy in self.cells:
            d = geos.ray_square_crossing(c[0], c[1], e[0], e[1], cx - 5.0, cx + 5.0, cy - 5.0, cy + 5.0)
            if d is not None and d <= min_d:
                min_d = d
        for lx in (float(BOUND[0]), float(BOUND[1])):
            d = geos.ray_vline_crossing(c[0], c[1], e[0], e[1], lx)
            if d is not None and d < min_d:
                min_d = d
        for ly in (float(BOUND[2]), float(BOUND[3])):
            d = geos.ray_hline_crossing(c[0], c[1], e[0], e[1], ly)
            if d is not None and d < min_d:
                min_d = d
        return min_d

    def radar(self, i):
        ag = self.all_agents[i]
        c = (ag.pos[0], ag.pos[1])
        out = []
        for deg in range(0, 360, 20):
            e = self._ray_end(c, deg)
            length = geos.point_dist(e[0], e[1], c[0], c[1])
            if self.radar_mode == RADAR_DRONES:
                out.append(self._radar_drones(i, c, e, length))
            elif self.radar_mode == RADAR_OBSTACLES:
                out.append(self._radar_obstacles(c, e, length))
            else:
                dd = self._radar_drones(i, c, e, length)
                do = self._radar_obstacles(c, e, length)
                out.append(dd if dd < do else do)
        return np.array(out)

    # observation ------------------------------------------------------------
    def cur_state_norm_state_v3(self):
        """Returns (own (N, D0), radar (N, 18), nei (N, K, 6)) normalised, float64."""
        own_all, radar_all, nei_all = [], [], []
        tcpa_rows = []
        for i, ag in self.all_agents.items():
            nb = self.get_current_agent_nei(ag)
            ag.observableSpace = self.radar(i)
            norm_pos = scale_pos([ag.pos[0], ag.pos[1]])
            norm_vel = nmlz_vel([ag.vel[0], ag.vel[1]])
            norm_G = nmlz_pos([ag.goal[-1][0], ag.goal[-1][1]])
            norm_deltaG = norm_G - norm_pos
            p1_norm, p3_norm, trow = [], [], []
            cur_conf = 0
            pre_conf = 0
            for j, other in nb.items():
                if j == i:
                    continue
                o = self.all_agents[j]
                dxh = o.pos[0] - ag.pos[0]
                dyh = o.pos[1] - ag.pos[1]
                if self.compat:
                    norm_delta_pos = scale_pos([dxh, dyh])
                else:
                    norm_delta_pos = norm_scale([dxh, dyh])
                norm_neigh_vel = nmlz_vel([o.vel[0], o.vel[1]])
                tcpa, dtcpa, cur_conf = compute_t_cpa_d_cpa_potential_col(o.pos, ag.pos, o.vel, ag.vel, PB, PB, cur_conf)
                ptcpa, pdtcpa, pre_conf = compute_t_cpa_d_cpa_potential_col(o.pre_pos, ag.pre_pos, o.pre_vel, ag.pre_vel, PB, PB, pre_conf)
                trow.append((tcpa, dtcpa))
                p1_norm.append(np.concatenate([norm_delta_pos, norm_neigh_vel]))
                npd = nmlz_pos_diff([other[0] - ag.pos[0], other[1] - ag.pos[1]])
                if self.compat:
                    ngd = nmlz_pos_diff([other[-2] - other[0], other[-1] - other[1]])
                else:
                    ngd = nmlz_pos_diff([o.goal[-1][0] - other[0], o.goal[-1][1] - other[1]])
                nv = tuple(nmlz_vel([other[2], other[3]]))
                p3_norm.append(list(npd + ngd + nv))
            own = np.concatenate([np.concatenate([norm_pos, norm_vel, norm_deltaG]), np.concatenate(p1_norm)])
            own_all.append(own)
            radar_all.append(ag.observableSpace)
            nei_all.append(np.array(p3_norm))
            tcpa_rows.append((trow, cur_conf, pre_conf))
        self.tdcpa = tcpa_rows
        return np.stack(own_all), np.stack(radar_all), np.stack(nei_all)

    # reward -----------------------------------------------------------------
    def ss_reward(self):
        """ATT/env:2105-2618 with full_observable_critic_flag=True, xy=(None, None).

        Returns (reward list, done list, check_goal list, bbc[4], masks list) where
        masks[i] = bit0 bound | bit1 drone | bit2 goal | bit3 building | bit4 wp | bit5 check_goal.
        """
        bbc = [False] * 4
        reward, done, masks = [], [], []
        check_goal = [False] * self.N
        c_drone = 1 + (NEAR_LO / (NEAR_HI - NEAR_LO))
        m_drone = (0 - 1) / (NEAR_HI - NEAR_LO)
        for idx, ag in self.all_agents.items():
            collision_drones = []
            nearest_key = None
            shortest = math.inf
            all_dist = []
            for k in ag.surroundingNeighbor:
                diff = ag.pos - self.all_agents[k].pos
                d = np.linalg.norm(diff)
                all_dist.append(d)
                if d < shortest:
                    shortest = d
                    nearest_key = k
                if np.linalg.norm(diff) <= ag.protectiveBound * 2:
                    collision_drones.append(k)
            building = 0
            for cx, cy in self.cells:
                if geos.building_hit_cell(ag.pos[0], ag.pos[1], cx, cy):
                    building = 1
                    ag.collide_wall_count += 1
                    break
            goal_hit = geos.goal_reached(ag.pos[0], ag.pos[1], float(ag.goal[-1][0]), float(ag.goal[-1][1]))
            wp0 = ag.waypoints[0]
            wp_flag = geos.point_dist(ag.pos[0], ag.pos[1], float(wp0[0]), float(wp0[1])) < WP_REACH
            before = np.linalg.norm(ag.pre_pos - ag.goal[-1])
            after = np.linalg.norm(ag.pos - ag.goal[-1])
            dist_to_goal = 1 * (before - after)
            dist_to_goal = dist_to_goal / ag.maxSpeed
            near_pen = 0
            for d in all_dist:
                if d >= NEAR_LO and d <= NEAR_HI:
                    near_pen = near_pen + (1 * (m_drone * shortest + c_drone))
                else:
                    near_pen = near_pen + 1 * 0
            bound_hit = geos.bound_crash(ag.pre_pos, ag.pos, BOUND, ag.protectiveBound)
            m = (bound_hit << 0) | ((len(collision_drones) > 0) << 1) | (goal_hit << 2) | (building << 3) | (wp_flag << 4)
            if bound_hit:
                rew = 0 - CRASH_PENALTY - 0.0 - 0
                done.append(True)
                bbc[0] = True
            elif len(collision_drones) > 0:
                done.append(True)
                bbc[2] = True
                rew = 0 - CRASH_PENALTY - 0.0 - near_pen
                if collision_drones[-1] == nearest_key:
                    bbc[3] = True
            elif goal_hit:
                check_goal[idx] = True
                ag.reach_target = True
                rew = 0 + REACH_REWARD + 0.0
                done.append(False)
            else:
                if wp_flag and len(ag.waypoints) > 1:
                    ag.removed_goal = ag.waypoints.pop(0)
                rew = 0 + 0.0 + dist_to_goal - 0.0 + 0.0 - 0 + 0 - 0 - near_pen - 0
                done.append(False)
            reward.append(np.array(rew))
            masks.append(int(m) | (32 if check_goal[idx] else 0))
        team = np.sum(reward)
        reward = [team for _ in reward]
        return reward, done, check_goal, bbc, masks

    def episode_over(self, done, check_goal):
        """ATT/main:448-462 (step already incremented)."""
        return (self.episode_length < self.step_count or (True in done) or all(check_goal)
                or all(a.reach_target for a in self.all_agents.values()))

    def full_step(self, actions):
        obs = self.step(actions)
        r, d, cg, bbc, masks = self.ss_reward()
        self.step_count += 1
        over = self.episode_over(d, cg)
        return obs, r, d, cg, bbc, masks, over
