"""Environment API over libaac_env.so.

``BatchedEnv``  -- E independent envs x N agents on one GPU; all buffers are torch tensors on the
                   device and every call is a kernel launch on torch's current stream.
``env_simulator`` -- drop-in facade with the reference's method surface
                   (ATT/env:41 ``__init__``, :84 ``create_world``, :199 ``reset_world``,
                   :2627 ``step``, :2105 ``ss_reward``, ``all_agents[i]`` attribute views) so an
                   unchanged ``ma_main`` loop can drive the GPU path with E = 1.
"""
import copy
import ctypes
import math
from dataclasses import dataclass, fields
from typing import Optional

import numpy as np
import torch

from . import _native
from . import world as _world

RADAR_MODES = {"drones": 0, "obstacles": 1, "combined": 2}
N_RAYS = 18


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@dataclass
class StepBuffers:
    """Device outputs of one env step / reset (layouts in include/aac_env.h)."""
    own: torch.Tensor
    radar: torch.Tensor
    nei: torch.Tensor
    reward: torch.Tensor
    done: torch.Tensor
    mask: torch.Tensor
    env_done: torch.Tensor
    bbc: torch.Tensor
    tcpa: Optional[torch.Tensor] = None
    dcpa: Optional[torch.Tensor] = None
    conf_cur: Optional[torch.Tensor] = None
    conf_pre: Optional[torch.Tensor] = None

    def c_struct(self):
        return _native.StepOut(*[(t.data_ptr() if t is not None else None)
                                 for t in (getattr(self, f.name) for f in fields(self))])


VARIANTS = {"att": 0, "wgru": 1}


class BatchedEnv:
    """E x N vectorised ``one_model_att`` environment on one MI355X.

    ``variant="wgru"``: the ``randomOD_Wgru_radar`` env of config 4 (WGRU/env:824-2131,
    WGRU/ma_main:653-661): obstacle radar, 6-wide own rows, per-agent reward; its defaults are
    max_spd 10 (WGRU/ma_main:409) and episode_length 150 (WGRU/ma_main:1044)."""

    def __init__(self, E, N, occ, radar_mode=None, compat=True, team_reward=None, max_wp=32,
                 episode_length=None, device=None, bound=_world.BOUND, cell=_world.CELL, tdcpa=False,
                 dt=0.5, acc_max=8.0, vmax=None, pB=2.5, radar_len=15.0, variant="att"):
        if not torch.cuda.is_available():
            raise RuntimeError("BatchedEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        occ = np.asarray(occ, dtype=np.uint8)
        if occ.ndim == 2:
            occ = occ[None]
        self.occ = np.ascontiguousarray(occ)
        self.E, self.N, self.K = int(E), int(N), int(N) - 1
        self.variant = VARIANTS[variant]
        # per-variant defaults for the arguments left at None; an explicit value is kept as given
        # (variant 1 supports only the obstacle radar and per-agent rewards, so asking it for
        # anything else raises instead of being overwritten)
        d_radar, d_team, d_vmax, d_ep = (("obstacles", False, 10.0, 150) if self.variant else ("drones", True, 5.0, 50))
        if self.variant:
            if radar_mode is not None and RADAR_MODES.get(radar_mode, radar_mode) != RADAR_MODES["obstacles"]:
                raise ValueError("variant 'wgru' uses the obstacle radar (WGRU/env:990-1054); got radar_mode=%r"
                                 % (radar_mode,))
            if team_reward:
                raise ValueError("variant 'wgru' computes per-agent rewards (WGRU/env:1800-1960); team_reward=True")
        radar_mode = d_radar if radar_mode is None else radar_mode
        team_reward = d_team if team_reward is None else team_reward
        vmax = d_vmax if vmax is None else vmax
        episode_length = d_ep if episode_length is None else episode_length
        self.D0 = 6 if self.variant else 6 + 4 * self.K
        self.W = int(max_wp)
        self.tdcpa = tdcpa
        self.radar_mode = RADAR_MODES[radar_mode] if isinstance(radar_mode, str) else int(radar_mode)
        cfg = _native.EnvCfg()
        cfg.E, cfg.N, cfg.R = self.E, self.N, N_RAYS
        cfg.radar_mode, cfg.compat, cfg.team_reward = self.radar_mode, int(bool(compat)), int(bool(team_reward))
        cfg.max_wp, cfg.episode_length = self.W, int(episode_length)
        cfg.n_maps, cfg.grid_w, cfg.grid_h = occ.shape
        cfg.dt, cfg.acc_max, cfg.vmax, cfg.pB, cfg.radar_len = dt, acc_max, vmax, pB, radar_len
        cfg.bound = (ctypes.c_double * 4)(*[float(b) for b in bound])
        cfg.cell = float(cell)
        cfg.occ = self.occ.ctypes.data
        cfg.variant = self.variant
        self.cfg = cfg
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        with torch.cuda.device(dev_index):
            _native.check(_native.lib().aac_env_create(ctypes.byref(cfg), dev_index, ctypes.byref(h)),
                          "aac_env_create")
        self._h = h
        self.bufs = self.alloc_buffers()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _native.lib().aac_env_destroy(h)
            except Exception:
                pass
            self._h = None

    # ----------------------------------------------------------------------- buffers
    def alloc_buffers(self):
        E, N, K, d = self.E, self.N, self.K, self.device
        f32, u8 = torch.float32, torch.uint8
        b = StepBuffers(
            own=torch.zeros(E, N, self.D0, dtype=f32, device=d),
            radar=torch.zeros(E, N, N_RAYS, dtype=f32, device=d),
            nei=torch.zeros(E, N, K, 6, dtype=f32, device=d),
            reward=torch.zeros(E, N, dtype=f32, device=d),
            done=torch.zeros(E, N, dtype=u8, device=d),
            mask=torch.zeros(E, N, dtype=u8, device=d),
            env_done=torch.zeros(E, dtype=u8, device=d),
            bbc=torch.zeros(E, 4, dtype=u8, device=d))
        if self.tdcpa:
            b.tcpa = torch.zeros(E, N, K, dtype=torch.float64, device=d)
            b.dcpa = torch.zeros(E, N, K, dtype=torch.float64, device=d)
            b.conf_cur = torch.zeros(E, N, dtype=torch.int32, device=d)
            b.conf_pre = torch.zeros(E, N, dtype=torch.int32, device=d)
        return b

    # ----------------------------------------------------------------------- calls
    def reset(self, start, wps, wp_cnt, map_idx=None, env_mask=None, out: Optional[StepBuffers] = None):
        """Install an explicit OD for the masked envs and write their observation rows."""
        out = out or self.bufs
        d = self.device
        st = torch.as_tensor(start, dtype=torch.float64, device=d).contiguous()
        w = torch.as_tensor(wps, dtype=torch.float64, device=d).contiguous()
        c = torch.as_tensor(wp_cnt, dtype=torch.int32, device=d).contiguous()
        assert st.shape == (self.E, self.N, 2) and w.shape == (self.E, self.N, self.W, 2) and c.shape == (self.E, self.N)
        if int(c.min()) < 1 or int(c.max()) > self.W:
            raise ValueError("waypoint counts must be in [1, max_wp]")
        mi = None if map_idx is None else torch.as_tensor(map_idx, dtype=torch.int32, device=d).contiguous()
        m = None if env_mask is None else torch.as_tensor(env_mask, dtype=torch.uint8, device=d).contiguous()
        o = out.c_struct()
        _native.check(_native.lib().aac_env_reset(self._h, _ptr(m), _ptr(st), _ptr(w), _ptr(c), _ptr(mi),
                                                  ctypes.byref(o), _stream()), "aac_env_reset")
        self._keep = (st, w, c, mi, m)   # keep alive until the stream consumes them
        return out

    def step(self, actions, out: Optional[StepBuffers] = None):
        """Kinematics + observation + ss_reward + termination for all envs (one kernel)."""
        out = out or self.bufs
        a = actions
        if a.dtype != torch.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        assert a.shape == (self.E, self.N, 2), a.shape
        o = out.c_struct()
        _native.check(_native.lib().aac_env_step(self._h, _ptr(a), ctypes.byref(o), _stream()), "aac_env_step")
        return out

    def step_tail(self, actions, out: Optional[StepBuffers] = None, replay=None, srcs=None, zero_rows=None,
                  auto_reset=True, pos_io=None):
        """``step`` + ``replay.push_batch(*srcs)`` + zeroing ``zero_rows`` ([E][...] float32) of the
        finished envs + ``auto_reset(out.env_done, out)``, fused into the one step launch
        (aac_env_step_tail).  ``srcs`` may name this step's outputs (``out.reward`` ...): the push reads
        the terminal rows before the reset overwrites them.  Same results as the four calls."""
        out = out or self.bufs
        a = actions
        if a.dtype != torch.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        assert a.shape == (self.E, self.N, 2), a.shape
        t = _native.StepTail()
        if replay is not None:
            for k, v in replay.tail_push(srcs, self.E).items():
                setattr(t, k, v)
            if pos_io is not None:
                # graph replays: the ring position is read from / advanced into device int64 words
                # (alternate the pair between steps); the replay's host mirror advances as usual
                pin, pout = pos_io
                assert pin.dtype == torch.int64 and pout.dtype == torch.int64 and pin.data_ptr() != pout.data_ptr()
                t.pos_in, t.pos_out = pin.data_ptr(), pout.data_ptr()
        if zero_rows is not None:
            assert zero_rows.dtype == torch.float32 and zero_rows.is_contiguous() and zero_rows.shape[0] == self.E
            assert zero_rows.device == self.device
            t.zero_rows = zero_rows.data_ptr()
            t.zero_width = zero_rows.numel() // self.E
        t.auto_reset = int(bool(auto_reset))
        o = out.c_struct()
        _native.check(_native.lib().aac_env_step_tail(self._h, _ptr(a), ctypes.byref(o), ctypes.byref(t), _stream()),
                      "aac_env_step_tail")
        return out

    def set_od_bank(self, bank, seed=0):
        """Install the device OD bank for auto-reset: a ``world.ODBank`` (one map), or a
        ``world.MapBanks`` for a map stack (each auto-reset draws the env's map, then its OD).

        The device bank is re-allocated and the draw seed changes: a graph captured around
        ``step_tail`` / ``auto_reset`` bakes both, so ``bank_generation`` advances and the graph's
        owner must re-capture (``trainer.Trainer`` checks it before every whole-step replay)."""
        if isinstance(bank, _world.MapBanks):
            if bank.n_maps != self.occ.shape[0]:
                raise ValueError(f"{bank.n_maps} banks for {self.occ.shape[0]} maps")
            _native.check(_native.lib().aac_env_set_od_banks(self._h, bank.n_maps, bank.start.ctypes.data,
                                                             bank.wps.ctypes.data, bank.cnt.ctypes.data,
                                                             bank.counts.ctypes.data, ctypes.c_uint64(seed)),
                          "aac_env_set_od_banks")
        else:
            _native.check(_native.lib().aac_env_set_od_bank(self._h, bank.start.ctypes.data, bank.wps.ctypes.data,
                                                            bank.cnt.ctypes.data, bank.n_pairs,
                                                            ctypes.c_uint64(seed)), "aac_env_set_od_bank")
        self.bank = bank
        self.bank_seed = int(seed)
        self.bank_generation = getattr(self, "bank_generation", 0) + 1

    def band_max(self):
        """(most radar rays one launch flagged for the exact threshold fix-up -- variant 1: or rewards
        listed for the exact radar minimum --, the lists' capacity): aac_env_band_max (synchronises)."""
        n, cap = ctypes.c_int32(0), ctypes.c_int32(0)
        _native.check(_native.lib().aac_env_band_max(self._h, ctypes.byref(n), ctypes.byref(cap), _stream()),
                      "aac_env_band_max")
        return n.value, cap.value

    def check_band_capacity(self):
        """Raise if any launch flagged more threshold-band rays (or variant-1 rewards) than the fix-up
        list holds: the surplus would have kept their float decisions.  Synchronises; the trainers call
        it once at the end of a run."""
        most, cap = self.band_max()
        if most > cap:
            raise RuntimeError(f"exact threshold fix-up list overflowed: {most} entries in one launch, capacity {cap}")
        return most, cap

    def use_episode_buffer(self, episode: torch.Tensor):
        """Keep the per-env episode counter (advanced by every auto-reset) in ``episode`` (int32 [E],
        on this device): a trainer's noise schedule then reads it with no per-step update."""
        assert episode.dtype == torch.int32 and episode.shape == (self.E,) and episode.is_contiguous()
        assert episode.device == self.device
        _native.check(_native.lib().aac_env_use_episode_buffer(self._h, _ptr(episode), _stream()),
                      "aac_env_use_episode_buffer")
        self._episode_buf = episode
        return episode

    def auto_reset(self, env_done=None, out: Optional[StepBuffers] = None):
        """Redraw OD from the device bank for envs with env_done != 0 (None = all envs)."""
        out = out or self.bufs
        o = out.c_struct()
        _native.check(_native.lib().aac_env_auto_reset(self._h, _ptr(env_done), ctypes.byref(o), _stream()),
                      "aac_env_auto_reset")
        return out

    def get_state(self):
        E, N, W, d = self.E, self.N, self.W, self.device
        f64 = dict(dtype=torch.float64, device=d)
        i32 = dict(dtype=torch.int32, device=d)
        s = dict(pos=torch.empty(E, N, 2, **f64), vel=torch.empty(E, N, 2, **f64),
                 pre_pos=torch.empty(E, N, 2, **f64), pre_vel=torch.empty(E, N, 2, **f64),
                 goal=torch.empty(E, N, 2, **f64), wp=torch.empty(E, N, W, 2, **f64),
                 wp_cur=torch.empty(E, N, **i32), wp_cnt=torch.empty(E, N, **i32),
                 reach=torch.empty(E, N, dtype=torch.uint8, device=d), wall=torch.empty(E, N, **i32),
                 step=torch.empty(E, **i32), map_idx=torch.empty(E, **i32), start=torch.empty(E, N, 2, **f64))
        _native.check(_native.lib().aac_env_get_state(self._h, *[_ptr(s[k]) for k in _STATE_KEYS], _stream()),
                      "aac_env_get_state")
        return s

    def set_state(self, **kw):
        d = self.device
        dt = dict(pos=torch.float64, vel=torch.float64, pre_pos=torch.float64, pre_vel=torch.float64,
                  goal=torch.float64, wp=torch.float64, wp_cur=torch.int32, wp_cnt=torch.int32,
                  reach=torch.uint8, wall=torch.int32, step=torch.int32, map_idx=torch.int32, start=torch.float64)
        t = {k: (torch.as_tensor(v, dtype=dt[k], device=d).contiguous() if v is not None else None)
             for k, v in kw.items()}
        for k in t:
            if k not in dt:
                raise KeyError(k)
        _native.check(_native.lib().aac_env_set_state(self._h, *[_ptr(t.get(k)) for k in _STATE_KEYS], _stream()),
                      "aac_env_set_state")
        torch.cuda.current_stream().synchronize()


_STATE_KEYS = ("pos", "vel", "pre_pos", "pre_vel", "goal", "wp", "wp_cur", "wp_cnt", "reach", "wall", "step",
               "map_idx", "start")


# =========================================================================== facade
class Agent:
    """Attribute view of ATT/agent:14-55 kept in sync with the device state (E = 1)."""

    def __init__(self, n_actions, agent_idx, gamma, tau, max_nei_num, maxSPD):
        self.gamma, self.tau, self.n_actions = gamma, tau, n_actions
        self.agent_name = "agent_%s" % agent_idx
        self.max_nei = max_nei_num
        self.pos = self.ini_pos = self.pre_pos = self.vel = self.pre_vel = None
        self.acc = np.zeros(2)
        self.pre_acc = np.zeros(2)
        self.maxSpeed = maxSPD
        self.goal = self.waypoints = self.ref_line = self.heading = None
        self.detectionRange = 30
        self.protectiveBound = 2.5
        self.pre_surroundingNeighbor = {}
        self.surroundingNeighbor = {}
        self.observableSpace = []
        self.target_update_step = None
        self.removed_goal = None
        self.update_count = 0
        self.reach_target = False
        self.collide_wall_count = 0


class env_simulator:
    """Reference-compatible facade (E = 1) over ``BatchedEnv``.

    ``world_map`` is the x-major occupancy grid (the reference passes the bounded map built
    from the shapefile, ATT/params:61); ``building_polygons``/``allGridPoly`` are accepted for
    signature compatibility but the geometry is rebuilt from ``world_map`` (10 m cells).
    """

    def __init__(self, world_map, building_polygons=None, grid_length=10, bound=None, allGridPoly=None,
                 agentConfig=None, radar_mode="drones", compat=True, seed=None):
        occ = np.asarray(world_map, dtype=np.uint8)
        self.world_map_2D = occ
        self.buildingPolygons = building_polygons
        self.world_map_2D_polyList = allGridPoly
        self.agentConfig = agentConfig
        self.gridlength = grid_length
        self.bound = list(bound) if bound is not None else list(_world.BOUND)
        self.global_time = 0.0
        self.time_step = 0.5
        self.all_agents = None
        self.radar_mode = radar_mode
        self.compat = compat
        self._rng = np.random.default_rng(seed)
        self._env = None

    def create_world(self, total_agentNum, n_actions, gamma, tau, target_update, largest_Nsigma, smallest_Nsigma,
                     ini_Nsigma, max_xy, max_spd, acc_range, full_observable_critic_flag=True):
        """ATT/env:84-197 (pools, agents) + native handle creation."""
        self.max_spd = max_spd
        self.all_agents = {}
        for i in range(total_agentNum):
            ag = Agent(n_actions, i, gamma, tau, total_agentNum, max_spd)
            ag.target_update_step = target_update
            self.all_agents[i] = ag
        self.dummy_agent = self.all_agents[0]
        self.target_pool = _world.target_pools(self.world_map_2D, self.bound, self.gridlength)
        self._team = full_observable_critic_flag
        self._env = BatchedEnv(1, total_agentNum, self.world_map_2D, radar_mode=self.radar_mode, compat=self.compat,
                               team_reward=True, vmax=float(max_spd), acc_max=float(abs(acc_range[1])),
                               bound=self.bound, cell=float(self.gridlength))
        self._env_agentwise = None

    # ---------------------------------------------------------------- OD (ATT/env:251-347)
    def _draw_od(self, N):
        starts, goals = [], []
        pools = self.target_pool
        for a in range(N):
            while True:
                qs = int(self._rng.integers(0, 4))
                qt = int(self._rng.choice([q for q in range(4) if q != qs]))
                s = pools[qs][int(self._rng.integers(0, len(pools[qs])))]
                if all(np.linalg.norm(np.array(s) - np.array(p)) > 2.5 * 2 for p in starts):
                    break
            t = pools[qt][int(self._rng.integers(0, len(pools[qt])))]
            ox, oy = math.ceil(self.bound[0] / self.gridlength), math.ceil(self.bound[2] / self.gridlength)
            path = _world.astar(self.world_map_2D, (int(s[0] / self.gridlength) - ox, int(s[1] / self.gridlength) - oy),
                                (int(t[0] / self.gridlength) - ox, int(t[1] / self.gridlength) - oy))
            refined = [path[0]]
            for k in range(2, len(path)):
                if (path[k][0] - path[k - 1][0], path[k][1] - path[k - 1][1]) != \
                        (path[k - 1][0] - path[k - 2][0], path[k - 1][1] - path[k - 2][1]):
                    refined.append(path[k - 1])
            refined.append(path[-1])
            g = [[(p[0] + ox) * self.gridlength, (p[1] + oy) * self.gridlength] for p in refined]
            g = [p for p in g if not (p[0] == s[0] and p[1] == s[1])]
            starts.append(s)
            goals.append(g)
        return starts, goals

    def reset_world(self, total_agentNum, actor_dim=None, show=0, starts=None, goals=None):
        """ATT/env:199-511.  ``starts``/``goals`` inject an OD (e.g. fixedDrone fixtures)."""
        self.global_time = 0.0
        if starts is None:
            starts, goals = self._draw_od(total_agentNum)
        W = self._env.W
        wps = np.zeros((1, total_agentNum, W, 2))
        cnt = np.zeros((1, total_agentNum), dtype=np.int32)
        for i, g in enumerate(goals):
            if len(g) > W:
                raise ValueError("waypoint list longer than max_wp")
            wps[0, i, :len(g)] = g
            wps[0, i, len(g):] = g[-1]
            cnt[0, i] = len(g)
        st = np.array(starts, dtype=np.float64)[None]
        self._env.reset(st, wps, cnt)
        for i, ag in self.all_agents.items():
            ag.pos = np.array(starts[i], dtype=float)
            ag.pre_pos = ag.pos.copy()
            ag.ini_pos = ag.pos.copy()
            ag.removed_goal = None
            ag.reach_target = False
            ag.collide_wall_count = 0
            ag.goal = [list(p) for p in goals[i]]
            ag.waypoints = copy.deepcopy(ag.goal)
            ag.heading = math.atan2(ag.goal[0][1] - ag.pos[1], ag.goal[0][0] - ag.pos[0])
            ag.vel = np.array([0.0, 0.0])
            ag.pre_vel = np.array([0.0, 0.0])
        return self._states()

    def _sync_agents(self):
        s = self._env.get_state()
        s = {k: v.cpu().numpy() for k, v in s.items()}
        for i, ag in self.all_agents.items():
            ag.pre_pos = s["pre_pos"][0, i].copy()
            ag.pos = s["pos"][0, i].copy()
            ag.pre_vel = s["pre_vel"][0, i].copy()
            ag.vel = s["vel"][0, i].copy()
            cur = int(s["wp_cur"][0, i])
            while len(ag.waypoints) > int(s["wp_cnt"][0, i]) - cur:
                ag.removed_goal = ag.waypoints.pop(0)
            ag.reach_target = bool(s["reach"][0, i])
            ag.collide_wall_count = int(s["wall"][0, i])
        return s

    def _states(self):
        """(state, norm_state) in the reference's list format (ATT/env:1483-1491)."""
        b = self._env.bufs
        own = b.own[0].cpu().numpy().astype(np.float64)
        radar = b.radar[0].cpu().numpy().astype(np.float64)
        nei = b.nei[0].cpu().numpy().astype(np.float64)
        norm = [[own[i] for i in range(self._env.N)], [radar[i] for i in range(self._env.N)],
                [[nei[i, k][None] for k in range(self._env.K)] for i in range(self._env.N)]]
        raw_own, raw_nei = [], []
        for i, ag in self.all_agents.items():
            p1 = [ag.pos[0], ag.pos[1], ag.vel[0], ag.vel[1], ag.goal[-1][0] - ag.pos[0], ag.goal[-1][1] - ag.pos[1]]
            p3 = []
            for j, o in self.all_agents.items():
                if j == i:
                    continue
                p1 += [o.pos[0] - ag.pos[0], o.pos[1] - ag.pos[1], o.vel[0], o.vel[1]]
                p3.append(np.array([[o.pos[0] - ag.pos[0], o.pos[1] - ag.pos[1], o.vel[1] - o.pos[0],
                                     ag.protectiveBound - o.pos[1], o.vel[0], o.vel[1]]]))
            raw_own.append(np.array(p1))
            raw_nei.append(p3)
            ag.observableSpace = radar[i]
        state = [raw_own, [radar[i] for i in range(self._env.N)], raw_nei]
        return state, norm

    def step(self, actions, current_ts=0, acc_max=8, actor_dim=None):
        """ATT/env:2627 (actor_dim optional: contract R5).  Reward/done are computed in the same
        kernel and handed out by the following ``ss_reward`` call."""
        a = torch.as_tensor(np.asarray(actions, dtype=np.float32)).reshape(1, -1, 2)
        self._env.step(a)
        b = self._env.bufs
        self._last = {k: getattr(b, k)[0].cpu().numpy() for k in ("reward", "done", "mask", "bbc")}
        self._sync_agents()
        state, norm = self._states()
        return state, norm, [], [], [], [], [], []

    def ss_reward(self, current_ts, step_reward_record, eps_status_holder, step_collision_record, xy=(None, None),
                  full_observable_critic_flag=True, args=None):
        """ATT/env:2105 -- returns the kernel's reward/done/check_goal/bbc of the last step."""
        last = self._last
        mask = last["mask"]
        N = self._env.N
        if full_observable_critic_flag:
            reward = [np.float64(last["reward"][i]) for i in range(N)]
        else:
            raise NotImplementedError("per-agent reward: construct BatchedEnv(team_reward=False)")
        done = [bool(last["done"][i]) for i in range(N)]
        check_goal = [bool(mask[i] & 32) for i in range(N)]
        for i in range(N):
            if step_collision_record is not None:
                step_collision_record[i].append([0, 0, 0, int(bool(mask[i] & 8)), 0, 0])
            if step_reward_record is not None:
                step_reward_record[i] = [0.0, None]
        bbc = [bool(v) for v in last["bbc"]]
        return reward, done, check_goal, step_reward_record, eps_status_holder, step_collision_record, bbc
