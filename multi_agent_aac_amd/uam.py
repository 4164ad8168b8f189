"""UAM environment over libaac_env.so (include/aac_uam.h).

``BatchedUAM``     -- E independent UAM envs x N aircraft on one GPU, float64 device buffers,
                      every call one kernel launch on torch's current stream.
``env_simulator``  -- drop-in facade with the reference's method surface for E = 1
                      (UAM/env:45 ``__init__``, :94 ``create_world``, :551
                      ``reset_world_change_skin``, :4667 ``step``, :3892
                      ``ss_reward_Mar_changeskin``, ``all_agents[i]`` / ``cloud_config`` views).
``build_bank``     -- whole episodes drawn with the reference's OD rules (native, host side).

UAM/ = MADDPG_ownENV_randomOD_radar_N_model_use_tdCPA_forV2_changeskin_UAM.
"""
import ctypes
import math
from dataclasses import dataclass, fields
from typing import Optional

import numpy as np
import torch

from . import _native

vp = ctypes.c_void_p
i32 = ctypes.c_int32
N_RAYS = 18
BOUND = (0.0, 40.0, 0.0, 40.0)               # UAM/params:32-36
EXPORTS = ("aac_uam_create", "aac_uam_destroy", "aac_uam_last_error", "aac_uam_reset", "aac_uam_step",
           "aac_uam_set_bank", "aac_uam_auto_reset", "aac_uam_bank_build", "aac_uam_get_state",
           "aac_uam_set_state", "aac_uam_actor", "aac_uam_actor_last_error", "aac_uam_set_reset_compact",
           "aac_uam_use_episode_buffer")


class UamCfg(ctypes.Structure):
    _fields_ = [("E", i32), ("N", i32), ("episode_length", i32),
                ("dt", ctypes.c_double), ("acc_max", ctypes.c_double), ("vmax", ctypes.c_double),
                ("pB", ctypes.c_double), ("radar_len", ctypes.c_double), ("bound", ctypes.c_double * 4)]


class UamOut(ctypes.Structure):
    _fields_ = [(n, vp) for n in ("own", "radar", "nei", "nei6", "reward", "done", "mask", "env_done", "bbc",
                                  "tcpa", "dcpa", "conf_cur", "conf_pre")]


_L = None


def lib():
    global _L
    if _L is None:
        L = _native.lib()
        L.aac_uam_last_error.restype = ctypes.c_char_p
        L.aac_uam_create.argtypes = [ctypes.POINTER(UamCfg), ctypes.c_int, ctypes.POINTER(vp)]
        L.aac_uam_destroy.argtypes = [vp]
        L.aac_uam_destroy.restype = None
        L.aac_uam_reset.argtypes = [vp, vp, vp, vp, vp, ctypes.POINTER(UamOut), vp]
        L.aac_uam_step.argtypes = [vp, vp, ctypes.POINTER(UamOut), vp]
        L.aac_uam_set_bank.argtypes = [vp, vp, vp, vp, i32, ctypes.c_uint64]
        L.aac_uam_auto_reset.argtypes = [vp, vp, ctypes.POINTER(UamOut), vp]
        L.aac_uam_set_reset_compact.argtypes = [i32]
        L.aac_uam_set_reset_compact.restype = None
        L.aac_uam_use_episode_buffer.argtypes = [vp, vp, vp]
        L.aac_uam_bank_build.argtypes = [i32, i32, ctypes.c_uint64, vp, vp, vp]
        L.aac_uam_get_state.argtypes = [vp] + [vp] * 13 + [vp]
        L.aac_uam_set_state.argtypes = [vp] + [vp] * 13 + [vp]
        L.aac_uam_actor_last_error.restype = ctypes.c_char_p
        L.aac_uam_actor.argtypes = [vp, vp, i32] + [vp] * 9 + [i32, vp, i32, ctypes.c_double, ctypes.c_double,
                                                            ctypes.c_uint64, vp, i32, vp]
        for name in EXPORTS:
            getattr(L, name)
        _L = L
    return _L


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {lib().aac_uam_last_error().decode(errors='replace')}")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Bank:
    """n whole episodes: start / goal float64[n][N][2], clouds int32[n][2] (cloud_0, cloud_1)."""

    def __init__(self, start, goal, clouds):
        self.start = np.ascontiguousarray(start, dtype=np.float64)
        self.goal = np.ascontiguousarray(goal, dtype=np.float64)
        self.clouds = np.ascontiguousarray(clouds, dtype=np.int32)
        self.n = self.start.shape[0]


def build_bank(n, N, seed=0):
    """``aac_uam_bank_build``: the reference's draw rules (UAM/env:575-747, UAM/util:165-237)."""
    st = np.zeros((n, N, 2))
    go = np.zeros((n, N, 2))
    cl = np.zeros((n, 2), dtype=np.int32)
    _chk(lib().aac_uam_bank_build(n, N, ctypes.c_uint64(seed), st.ctypes.data, go.ctypes.data, cl.ctypes.data),
         "aac_uam_bank_build")
    return Bank(st, go, cl)


@dataclass
class UamBuffers:
    """Device outputs of one step / reset (layouts in include/aac_uam.h)."""
    own: torch.Tensor
    radar: torch.Tensor
    nei: Optional[torch.Tensor]
    nei6: Optional[torch.Tensor]
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
        return UamOut(*[(t.data_ptr() if t is not None else None) for t in (getattr(self, f.name) for f in fields(self))])


_STATE = (("pos", torch.float64, (2,)), ("vel", torch.float64, (2,)), ("pre_pos", torch.float64, (2,)),
          ("pre_vel", torch.float64, (2,)), ("goal", torch.float64, (2,)), ("start", torch.float64, (2,)),
          ("heading", torch.float64, ()), ("reach", torch.uint8, ()), ("clouds", torch.float64, (2, 2)),
          ("cloud_kind", torch.int32, (2,)), ("cloud_tgt", torch.int32, ()), ("step", torch.int32, ()),
          ("top2", torch.uint8, (2,)))
_PER_ENV = {"clouds", "cloud_kind", "cloud_tgt", "step"}


class BatchedUAM:
    """E x N vectorised UAM environment on one MI355X (float64 state and observations)."""

    def __init__(self, E, N, episode_length=150, device=None, neighbours=True, p3=False, tdcpa=False,
                 dt=0.5, acc_max=0.5, vmax=1.0, pB=0.5, radar_len=5.0, bound=BOUND):
        if not torch.cuda.is_available():
            raise RuntimeError("BatchedUAM needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.E, self.N, self.K = int(E), int(N), int(N) - 1
        self.neighbours, self.p3, self.tdcpa = neighbours, p3, tdcpa
        cfg = UamCfg()
        cfg.E, cfg.N, cfg.episode_length = self.E, self.N, int(episode_length)
        cfg.dt, cfg.acc_max, cfg.vmax, cfg.pB, cfg.radar_len = dt, acc_max, vmax, pB, radar_len
        cfg.bound = (ctypes.c_double * 4)(*[float(b) for b in bound])
        self.cfg = cfg
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device.index):
            _chk(lib().aac_uam_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)), "aac_uam_create")
        self._h = h
        self.bufs = self.alloc_buffers()
        self.bank = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().aac_uam_destroy(h)
            except Exception:
                pass
            self._h = None

    def alloc_buffers(self):
        E, N, K, d = self.E, self.N, self.K, self.device
        f64, u8 = dict(dtype=torch.float64, device=d), dict(dtype=torch.uint8, device=d)
        b = UamBuffers(own=torch.zeros(E, N, 7, **f64), radar=torch.zeros(E, N, N_RAYS, **f64),
                       nei=torch.zeros(E, N, K, 5, **f64) if self.neighbours else None,
                       nei6=torch.zeros(E, N, K, 6, **f64) if self.p3 else None,
                       reward=torch.zeros(E, N, **f64), done=torch.zeros(E, N, **u8), mask=torch.zeros(E, N, **u8),
                       env_done=torch.zeros(E, **u8), bbc=torch.zeros(E, 4, **u8))
        if self.tdcpa:
            b.tcpa, b.dcpa = torch.zeros(E, N, K, **f64), torch.zeros(E, N, K, **f64)
            b.conf_cur = torch.zeros(E, N, dtype=torch.int32, device=d)
            b.conf_pre = torch.zeros(E, N, dtype=torch.int32, device=d)
        return b

    def reset(self, start, goal, clouds, env_mask=None, out: Optional[UamBuffers] = None):
        """reset_world_change_skin (UAM/env:551-771) with an injected episode for the masked envs."""
        out = out or self.bufs
        d = self.device
        st = torch.as_tensor(start, dtype=torch.float64, device=d).contiguous()
        go = torch.as_tensor(goal, dtype=torch.float64, device=d).contiguous()
        cl = torch.as_tensor(clouds, dtype=torch.int32, device=d).contiguous()
        assert st.shape == (self.E, self.N, 2) and go.shape == (self.E, self.N, 2) and cl.shape == (self.E, 2)
        c = cl.cpu()
        if int(c[:, 0].min()) < 0 or int(c[:, 0].max()) > 1 or int(c[:, 1].min()) < 0 or int(c[:, 1].max()) > 3:
            raise ValueError("clouds: cloud_0 in {0, 1}, cloud_1 in {0..3}")
        m = None if env_mask is None else torch.as_tensor(env_mask, dtype=torch.uint8, device=d).contiguous()
        o = out.c_struct()
        _chk(lib().aac_uam_reset(self._h, _ptr(m), _ptr(st), _ptr(go), _ptr(cl), ctypes.byref(o), _stream()),
             "aac_uam_reset")
        self._keep = (st, go, cl, m)
        return out

    def step(self, actions, out: Optional[UamBuffers] = None):
        """Clouds + kinematics + observation + ss_reward_Mar_changeskin + termination (one kernel)."""
        out = out or self.bufs
        a = actions
        if a.dtype != torch.float64 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.float64).contiguous()
        assert a.shape == (self.E, self.N, 2), a.shape
        o = out.c_struct()
        _chk(lib().aac_uam_step(self._h, _ptr(a), ctypes.byref(o), _stream()), "aac_uam_step")
        return out

    def set_bank(self, bank: Bank, seed=0):
        assert bank.start.shape[1] == self.N
        _chk(lib().aac_uam_set_bank(self._h, bank.start.ctypes.data, bank.goal.ctypes.data, bank.clouds.ctypes.data,
                                    bank.n, ctypes.c_uint64(seed)), "aac_uam_set_bank")
        self.bank = bank
        self.bank_seed = int(seed)
        # graphs captured around auto_reset bake the bank pointers and seed: owners
        # re-capture when this advances (see env.BatchedEnv.set_od_bank)
        self.bank_generation = getattr(self, "bank_generation", 0) + 1

    def use_episode_buffer(self, episode: torch.Tensor):
        """Keep the per-env episode counter (advanced by every auto-reset) in ``episode`` (int32 [E])."""
        assert episode.dtype == torch.int32 and episode.shape == (self.E,) and episode.is_contiguous()
        assert episode.device == self.device
        _chk(lib().aac_uam_use_episode_buffer(self._h, _ptr(episode), _stream()), "aac_uam_use_episode_buffer")
        self._episode_buf = episode
        return episode

    def auto_reset(self, env_done=None, out: Optional[UamBuffers] = None):
        """Reset every env with env_done != 0 (None = all) to a fresh bank episode."""
        out = out or self.bufs
        o = out.c_struct()
        _chk(lib().aac_uam_auto_reset(self._h, _ptr(env_done), ctypes.byref(o), _stream()), "aac_uam_auto_reset")
        return out

    def get_state(self):
        E, N, d = self.E, self.N, self.device
        s = {k: torch.empty(*((E,) if k in _PER_ENV else (E, N)), *shp, dtype=dt, device=d) for k, dt, shp in _STATE}
        _chk(lib().aac_uam_get_state(self._h, *[_ptr(s[k]) for k, _, _ in _STATE], _stream()), "aac_uam_get_state")
        return s

    def set_state(self, **kw):
        dts = {k: dt for k, dt, _ in _STATE}
        for k in kw:
            if k not in dts:
                raise KeyError(k)
        t = {k: (torch.as_tensor(v, dtype=dts[k], device=self.device).contiguous() if v is not None else None)
             for k, v in kw.items()}
        _chk(lib().aac_uam_set_state(self._h, *[_ptr(t.get(k)) for k, _, _ in _STATE], _stream()),
             "aac_uam_set_state")
        torch.cuda.current_stream().synchronize()


# =========================================================================== facade
GO_AC = ((20, 20, 20, 35, 5, 35, 5, 5, 20, 5, 20, 20), (20, 20, 20, 5, 5, 5, 5, 35, 20, 35, 20, 20),
         (20, 20, 20, 35, 35, 35, 35, 5, 20, 5, 20, 20), (20, 20, 20, 5, 35, 5, 35, 35, 20, 35, 20, 20))
CLOUDS = ((8, 30, 10, 10), (30, 10, 35, 30))


class Agent:
    """Attribute view of UAM/agent:14-59, synchronised from the device after each call (E = 1)."""

    def __init__(self, n_actions, agent_idx, gamma, tau, max_nei_num, maxSPD):
        self.gamma, self.tau, self.n_actions = gamma, tau, n_actions
        self.agent_name = "agent_%s" % agent_idx
        self.max_nei = max_nei_num
        self.pos = self.ini_pos = self.pre_pos = self.vel = self.pre_vel = None
        self.acc = np.zeros(2)
        self.pre_acc = np.zeros(2)
        self.maxSpeed = maxSPD
        self.goal = self.waypoints = self.ref_line = self.heading = None
        self.detectionRange = 10
        self.protectiveBound = 0.5
        self.pre_surroundingNeighbor = {}
        self.surroundingNeighbor = {}
        self.observableSpace = []
        self.removed_goal = None
        self.reach_target = False
        self.bound_collision = self.building_collision = self.cloud_collision = self.drone_collision = False
        self.collide_wall_count = 0
        self.eta = None


class CloudView:
    """cloud_agent (UAM/cloud.py:11-49) view: pos / goal / preset trajectory of a cloud."""

    def __init__(self, idx):
        self.agent_name = "cloud_%s" % idx
        self.agent_essence = "cloud" if idx == 0 else "go_aircraft"
        self.radius = 3 if idx == 0 else 1
        self.vel = 0.4 if idx == 0 else 2
        self.pos = self.goal = None
        self.preset_traj = []
        self.previous_target = None


class env_simulator:
    """Reference-compatible facade (E = 1) over ``BatchedUAM``.  The UAM map has no buildings in
    the observation or reward path (radar and conflicts use the runway, the bound, the clouds and
    the other aircraft), so ``world_map`` / ``building_polygons`` are accepted and kept only."""

    def __init__(self, world_map=None, building_polygons=None, grid_length=1, bound=None, allGridPoly=None,
                 agentConfig=None, seed=None):
        self.world_map_2D = world_map
        self.buildingPolygons = building_polygons
        self.world_map_2D_polyList = allGridPoly
        self.agentConfig = agentConfig
        self.gridlength = grid_length
        self.bound = list(bound) if bound is not None else list(BOUND)
        self.global_time = 0.0
        self.time_step = 0.5
        self.all_agents = None
        self.cloud_config = None
        self._seed = 0 if seed is None else int(seed)
        self._draws = 0
        self._env = None

    def create_world(self, total_agentNum, n_actions, gamma, tau, target_update, largest_Nsigma, smallest_Nsigma,
                     ini_Nsigma, max_xy, max_spd, acc_range):
        """UAM/env:94-207 (agents) + native handle creation."""
        self.all_agents = {}
        for i in range(total_agentNum):
            ag = Agent(n_actions, i, gamma, tau, total_agentNum, max_spd)
            ag.target_update_step = target_update
            self.all_agents[i] = ag
        self.dummy_agent = self.all_agents[0]
        self._env = BatchedUAM(1, total_agentNum, vmax=float(max_spd), acc_max=float(abs(acc_range[1])),
                               bound=self.bound, p3=True)

    def reset_world_change_skin(self, total_agentNum, full_observable_critic_flag=False, evaluation_by_fixed_ar=False,
                                include_other_AC=True, use_nearestN_neigh_wRadar=False, N_neigh=2, args=None,
                                show=0, starts=None, goals=None, clouds=None):
        """UAM/env:551-771.  ``starts``/``goals``/``clouds`` inject an episode; otherwise one is
        drawn with the reference's rules (``build_bank``)."""
        if include_other_AC is not True or use_nearestN_neigh_wRadar or evaluation_by_fixed_ar:
            raise NotImplementedError("UAM facade: the default flags of UAM/main:60-100 only")
        self.global_time = 0.0
        if starts is None:
            bank = build_bank(1, total_agentNum, seed=self._seed * 1000003 + self._draws)
            self._draws += 1
            starts, goals, clouds = bank.start[0], bank.goal[0], bank.clouds[0]
        self._env.reset(np.asarray(starts, dtype=np.float64)[None], np.asarray(goals, dtype=np.float64)[None],
                        np.asarray(clouds, dtype=np.int32)[None])
        self.cloud_config = [CloudView(0), CloudView(1)]
        c0, c1 = int(clouds[0]), int(clouds[1])
        self.cloud_config[0].goal = np.array(CLOUDS[c0][2:4], dtype=float)
        self.cloud_config[1].preset_traj = [np.array(GO_AC[c1][k:k + 2], dtype=float) for k in range(0, 12, 2)]
        for i, ag in self.all_agents.items():
            ag.ini_pos = np.array(starts[i], dtype=float)
            ag.goal = [list(map(float, goals[i]))]
            ag.waypoints = [list(map(float, goals[i]))]
            ag.removed_goal = None
            ag.bound_collision = ag.building_collision = ag.cloud_collision = ag.drone_collision = False
        self._sync()
        return self._states()

    def _sync(self):
        s = {k: v.cpu().numpy() for k, v in self._env.get_state().items()}
        for i, ag in self.all_agents.items():
            ag.pos, ag.pre_pos = s["pos"][0, i].copy(), s["pre_pos"][0, i].copy()
            ag.vel, ag.pre_vel = s["vel"][0, i].copy(), s["pre_vel"][0, i].copy()
            ag.heading = float(s["heading"][0, i])
            ag.reach_target = bool(s["reach"][0, i])
        for k, c in enumerate(self.cloud_config):
            c.pos = s["clouds"][0, k].copy()
            if k == 1:
                c.previous_target = c.preset_traj[int(s["cloud_tgt"][0])]
        return s

    def _states(self):
        """(state, norm_state) = ([own, p2, radar, p3] raw, normalised), UAM/env:1888-1917."""
        b = self._env.bufs
        N, K = self._env.N, self._env.K
        own, radar = b.own[0].cpu().numpy(), b.radar[0].cpu().numpy()
        nei, nei6 = b.nei[0].cpu().numpy(), b.nei6[0].cpu().numpy()
        norm = [[own[i] for i in range(N)], [nei[i].reshape(-1) for i in range(N)], [radar[i] for i in range(N)],
                [[nei6[i, k][None] for k in range(K)] for i in range(N)]]
        raw_own, raw_p2, raw_p3 = [], [], []
        for i, ag in self.all_agents.items():
            raw_own.append(np.array([ag.pos[0], ag.pos[1], ag.vel[0], ag.vel[1], ag.goal[-1][0] - ag.pos[0],
                                     ag.goal[-1][1] - ag.pos[1], ag.heading]))
            order = sorted((j for j in self.all_agents if j != i),
                           key=lambda j: np.linalg.norm(self.all_agents[j].pos - ag.pos))
            ag.pre_surroundingNeighbor = ag.surroundingNeighbor
            ag.surroundingNeighbor = {j: np.array([*self.all_agents[j].pos, *self.all_agents[j].vel,
                                                   self.all_agents[j].protectiveBound]) for j in order}
            p2, p3 = [], []
            for j in order:
                o = self.all_agents[j]
                p2.append(np.array([o.pos[0] - ag.pos[0], o.pos[1] - ag.pos[1], o.vel[0], o.vel[1], o.heading]))
                p3.append(np.array([[o.pos[0] - ag.pos[0], o.pos[1] - ag.pos[1], o.vel[1] - o.pos[0],
                                     o.protectiveBound - o.pos[1], o.vel[0], o.vel[1]]]))
            raw_p2.append(np.concatenate(p2))
            raw_p3.append(p3)
            ag.observableSpace = radar[i]
        state = [raw_own, raw_p2, [radar[i] for i in range(N)], raw_p3]
        return state, norm

    def step(self, actions, current_ts=0, acc_max=0.5, args=None, evaluation_by_episode=True,
             full_observable_critic_flag=False, evaluation_by_fixed_ar=False, include_other_AC=True,
             use_nearestN_neigh_wRadar=False, N_neigh=2):
        """UAM/env:4667.  Reward / done are computed in the same kernel and handed out by the
        following ``ss_reward_Mar_changeskin`` call."""
        a = torch.as_tensor(np.asarray(actions, dtype=np.float64)).reshape(1, -1, 2)
        self._env.step(a)
        b = self._env.bufs
        self._last = {k: getattr(b, k)[0].cpu().numpy() for k in ("reward", "done", "mask", "bbc")}
        self._sync()
        state, norm = self._states()
        return state, norm, [], [], [], [], [], []

    def ss_reward_Mar_changeskin(self, current_ts, step_reward_record, step_collision_record, xy=(None, None),
                                 full_observable_critic_flag=False, args=None, evaluation_by_episode=True,
                                 evaluation_by_fixed_ar=False):
        """UAM/env:3892 -- the kernel's reward / done / check_goal / bbc of the last step."""
        last = self._last
        N = self._env.N
        mask = last["mask"]
        reward = [np.array(float(last["reward"][i])) for i in range(N)]
        if full_observable_critic_flag:
            reward = [np.sum(reward) for _ in reward]
        done = [bool(last["done"][i]) for i in range(N)]
        check_goal = [bool(mask[i] & 16) for i in range(N)]
        eps_status_holder = [{} for _ in range(N)]
        for i, ag in self.all_agents.items():
            ag.bound_collision |= bool(mask[i] & 1)
            ag.cloud_collision |= bool(mask[i] & 2)
            ag.drone_collision |= bool(mask[i] & 4)
            if step_collision_record is not None:
                step_collision_record[i].append([0, 0, 0, 0, 0, 0])
            if step_reward_record is not None:
                step_reward_record[i] = [0, float(reward[i])]
        bbc = [bool(v) for v in last["bbc"]]
        return reward, done, check_goal, step_reward_record, eps_status_holder, step_collision_record, bbc

    def episode_over(self, step, episode_length=150):
        """UAM/main:624-637 with ``step`` the already-incremented step counter."""
        return episode_length < step or any(bool(d) for d in self._last["done"]) or \
            all(ag.reach_target for ag in self.all_agents.values())
