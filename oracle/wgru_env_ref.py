"""Reference-shaped scalar restatement of the ``randomOD_Wgru_radar`` environment step (config 4).
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

``WGRU/`` is ``/root/reference/MADDPG_ownENV_randomOD_Wgru_radar/``; ``env`` its
``env_simulator_randomOD_Wgru_radar.py``.  One object per agent and per-agent loops, as
``oracle/env_ref.py`` does for the ATT env; GEOS calls are replaced by ``oracle.geos``.

Followed line by line:
  kinematics     WGRU/env:2048-2131 (coe_a = 8; max_spd = 10, WGRU/ma_main:409)
  radar          WGRU/env:866-965 -- obstacle cells + the 4 bound lines, the OM/env:1049-1148 form
                 (``ScalarEnv._radar_obstacles``)
  observation    WGRU/env:969-990: own = [scale_pos(pos), scale_vel(vel), nmlz_pos(goal[-1]) -
                 scale_pos(pos)] (6 values); the neighbour part (:1009-1036) is written with the
                 ATT layout (all N-1 others) -- the WGRU learner never reads it (WGRU/maddpg:237-247
                 stacks state parts 0 and 1 only)
  ss_reward      WGRU/env:1666-2039 (per-agent reward, crash 5 / reach 5, next-waypoint progress,
                 cross-track reward against the reference path, small-step and near-building
                 penalties, waypoint bonus)
  termination    WGRU/ma_main:653-661
"""
import math

import numpy as np

from . import geos
from .consts import BOUND, PB, X_SCALE, Y_SCALE
from .env_ref import RADAR_OBSTACLES, ScalarEnv, nmlz_pos, scale_pos

VMAX = 10                 # max_spd                                   WGRU/ma_main:409
ACC = 8                   # coe_a                                     WGRU/env:2056
DT = 0.5                  # time_step                                 WGRU/env:201
EPISODE_LENGTH = 150      # --episode_length                          WGRU/ma_main:1044
CRASH_PENALTY = 5         # crash_penalty_wall                        WGRU/env:1673
REACH_REWARD = 5          # reach_target                              WGRU/env:1677
WP_REACH = 5              # wp_reach_threshold_dist                   WGRU/env:1816
COEF_REF_LINE = 3         # coef_ref_line                             WGRU/env:1880
SMALL_STEP_COEF = 3       # small_step_penalty_coef                   WGRU/env:1896
NEAR_BUILDING_COEF = 3    # near_building_penalty_coef                WGRU/env:1918
TURNING_PT = 5            # turningPtConst (c = 2)                    WGRU/env:1924-1928


def scale_vel(v):
    """NormalizeData.scale_vel (WGRU/util:187-188)."""
    return np.array([X_SCALE * v[0], Y_SCALE * v[1]])


class WgruEnv(ScalarEnv):
    """One WGRU environment instance (N agents), reference-shaped."""

    D_OWN = 6

    def __init__(self, n_agents, occ, compat=True, episode_length=EPISODE_LENGTH):
        super().__init__(n_agents, occ, radar_mode=RADAR_OBSTACLES, compat=compat, episode_length=episode_length)

    def reset(self, starts, goal_lists):
        """State part of reset_world (WGRU/env:292-343): goal = the waypoints after the start;
        ref_line = LineString(start + waypoints) (``goalPt_withini``, :339-343)."""
        for i, ag in self.all_agents.items():
            ag.ref_line = [tuple(float(v) for v in starts[i])] + [tuple(float(v) for v in g) for g in goal_lists[i]]
        return super().reset(starts, goal_lists)

    def step(self, actions, acc_max=ACC):
        """WGRU/env:2048-2131."""
        for (idx, ag), act in zip(self.all_agents.items(), actions):
            ag.pre_pos = ag.pos.copy()
            ag.pre_vel = ag.vel.copy()
            ax, ay = act[0], act[1]
            ax = ax * acc_max
            ay = ay * acc_max
            cvx = ag.vel[0] + ax * DT
            cvy = ag.vel[1] + ay * DT
            nh = math.atan2(cvy, cvx)
            if np.linalg.norm([cvx, cvy]) >= VMAX:
                ag.vel = np.array([VMAX * math.cos(nh), VMAX * math.sin(nh)])
            else:
                ag.vel = np.array([cvx, cvy])
            dx = ag.vel[0] * DT
            dy = ag.vel[1] * DT
            ag.acc = np.array([ax, ay])
            ag.pos = np.array([ag.pos[0] + dx, ag.pos[1] + dy])
        return self.cur_state_norm_state_v3()

    def cur_state_norm_state_v3(self):
        """WGRU/env:824-1054 -> (own (N, 6), radar (N, 18), nei (N, K, 6))."""
        own_all, radar_all, nei_all = [], [], []
        for i, ag in self.all_agents.items():
            nb = self.get_current_agent_nei(ag)
            ag.observableSpace = self.radar(i)
            norm_pos = scale_pos([ag.pos[0], ag.pos[1]])
            norm_vel = scale_vel([ag.vel[0], ag.vel[1]])
            norm_G = np.array(nmlz_pos([ag.goal[-1][0], ag.goal[-1][1]]))
            norm_deltaG = norm_G - norm_pos
            own_all.append(np.concatenate([norm_pos, norm_vel, norm_deltaG], axis=0))
            p3 = []
            for j, other in nb.items():
                if j == i:
                    continue
                npd = _nmlz_pos_diff([other[0] - ag.pos[0], other[1] - ag.pos[1]])
                ngd = _nmlz_pos_diff([other[-2] - other[0], other[-1] - other[1]])
                nv = (other[2] / VMAX, other[3] / VMAX)
                p3.append(list(npd + ngd + nv))
            radar_all.append(ag.observableSpace)
            nei_all.append(np.array(p3))
        self.tdcpa = None
        return np.stack(own_all), np.stack(radar_all), np.stack(nei_all)

    def get_current_agent_nei(self, cur):
        # the ATT neighbour layout (every other agent); see the module docstring
        for j, ag in self.all_agents.items():
            if ag.agent_name == cur.agent_name:
                continue
            cur.surroundingNeighbor[j] = np.array([ag.pos[0], ag.pos[1], ag.vel[0], ag.vel[1], ag.protectiveBound])
        return cur.surroundingNeighbor

    def ss_reward(self):
        """WGRU/env:1666-2039 with xy = (None, None).  Returns (reward list (per agent), done list,
        check_goal list, bbc[4] = [bound, building, 0, 0], masks) where masks[i] = bit0 bound | bit1
        drone contact | bit2 goal | bit3 building | bit4 wp_intersect_flag | bit5 check_goal."""
        bbc = [False] * 4
        reward, done, masks = [], [], []
        check_goal = [False] * self.N
        for idx, ag in self.all_agents.items():
            collision = False
            for k in ag.surroundingNeighbor:
                if np.linalg.norm(ag.pos - self.all_agents[k].pos) <= ag.protectiveBound * 2:
                    collision = True                     # recorded only (:1732-1737)
            building = 0
            for cx, cy in self.cells:
                if geos.building_hit_cell(ag.pos[0], ag.pos[1], cx, cy):
                    building = 1
                    ag.collide_wall_count += 1
                    break
            # tar_circle from goal[-1] before the waypoint search below (:1803-1806)
            goal_hit = geos.goal_reached(ag.pos[0], ag.pos[1], float(ag.goal[-1][0]), float(ag.goal[-1][1]))
            # ---------- the next waypoint (:1815-1832)
            smallest = math.inf
            wp_flag = False
            next_wp = None
            for wpidx, wp in enumerate(ag.goal):
                d = geos.point_dist(ag.pos[0], ag.pos[1], float(wp[0]), float(wp[1]))
                if d < smallest:
                    smallest = d
                    next_wp = np.array(wp, dtype=float)
                    if smallest < WP_REACH:
                        wp_flag = True
                        if len(ag.goal) > 1:
                            ag.removed_goal = ag.goal.pop(wpidx)
                            best, pick = math.inf, None
                            for g in ag.goal:             # min(points_list, key=distance): first minimum
                                dd = geos.point_dist(float(g[0]), float(g[1]), ag.pos[0], ag.pos[1])
                                if dd < best:
                                    best, pick = dd, g
                            next_wp = np.array(pick, dtype=float)
                        break
            before = np.linalg.norm(ag.pre_pos - next_wp)
            after = np.linalg.norm(ag.pos - next_wp)
            dist_to_goal = 1 * (before - after)
            cross = geos.cross_track_distance(ag.pos[0], ag.pos[1], ag.ref_line)
            if cross <= ag.protectiveBound:
                m = (0 - 1) / (ag.protectiveBound - 0)
                dist_to_ref_line = COEF_REF_LINE * (m * cross + 1)
            else:
                dist_to_ref_line = -COEF_REF_LINE * 1
            thr = 2 * ag.protectiveBound
            small_step_penalty = SMALL_STEP_COEF * ((thr - np.clip(np.linalg.norm(ag.vel), 0, thr)) * (1.0 / thr))
            min_dist = np.min(ag.observableSpace)
            m = (0 - 1) / (TURNING_PT - ag.protectiveBound)
            if min_dist >= ag.protectiveBound and min_dist <= TURNING_PT:
                near_building_penalty = NEAR_BUILDING_COEF * (m * min_dist + 2)
            else:
                near_building_penalty = 0
            bound_hit = geos.bound_crash(ag.pre_pos, ag.pos, BOUND, ag.protectiveBound)
            msk = (bound_hit << 0) | (collision << 1) | (goal_hit << 2) | (building << 3) | (wp_flag << 4)
            rew = 0
            if bound_hit:
                rew = rew + dist_to_ref_line - CRASH_PENALTY + dist_to_goal - small_step_penalty + 0 - \
                    near_building_penalty
                done.append(True)
                bbc[0] = True
            elif building == 1:
                done.append(True)
                bbc[1] = True
                rew = rew + dist_to_ref_line - CRASH_PENALTY + dist_to_goal - small_step_penalty + 0 - \
                    near_building_penalty
            elif goal_hit:
                check_goal[idx] = True
                ag.reach_target = True
                rew = rew + REACH_REWARD + 0
                done.append(False)
            else:
                if wp_flag and len(ag.goal) > 1:
                    rew = rew + COEF_REF_LINE
                rew = rew + dist_to_ref_line + dist_to_goal - small_step_penalty + 0 - near_building_penalty + 0
                done.append(False)
            reward.append(np.array(rew))
            masks.append(int(msk) | (32 if check_goal[idx] else 0))
        return reward, done, check_goal, bbc, masks

    def episode_over(self, done, check_goal):
        """WGRU/ma_main:653-661 (step already incremented)."""
        return (self.episode_length < self.step_count or (True in done)
                or all(a.reach_target for a in self.all_agents.values()))


def _nmlz_pos_diff(d):
    dx_min, dx_max = BOUND[0] - BOUND[1], BOUND[1] - BOUND[0]
    dy_min, dy_max = BOUND[2] - BOUND[3], BOUND[3] - BOUND[2]
    return (2 * ((d[0] - dx_min) / (dx_max - dx_min)) - 1, 2 * ((d[1] - dy_min) / (dy_max - dy_min)) - 1)


__all__ = ["WgruEnv", "VMAX", "EPISODE_LENGTH", "PB"]
