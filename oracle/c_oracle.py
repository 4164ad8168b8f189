"""ctypes wrapper of oracle/aac_oracle.c (TEST INFRASTRUCTURE ONLY).

``BatchedOracle`` keeps the batched environment state in numpy arrays with the same
SoA layout as the GPU handle, so tests can compare state, observations, rewards and
masks element for element.
"""
import ctypes
import os
import subprocess

import numpy as np

from .consts import BOUND, EPISODE_LENGTH, N_RAYS

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libaac_oracle.so")


def build():
    """Compile the C oracle in place (``make -C oracle``)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


class _Cfg(ctypes.Structure):
    _fields_ = [("E", ctypes.c_int32), ("N", ctypes.c_int32), ("W", ctypes.c_int32),
                ("radar_mode", ctypes.c_int32), ("compat", ctypes.c_int32), ("team_reward", ctypes.c_int32),
                ("episode_length", ctypes.c_int32), ("gw", ctypes.c_int32), ("gh", ctypes.c_int32),
                ("bound", ctypes.c_double * 4), ("occ", ctypes.c_void_p), ("n_maps", ctypes.c_int32),
                ("variant", ctypes.c_int32), ("vmax", ctypes.c_double)]


class _State(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("pos", "vel", "pre_pos", "pre_vel", "goal", "wp", "wp_cur", "wp_cnt", "reach", "wall", "step",
                 "map_idx", "start")]


class _Out(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("own", "radar", "nei", "reward", "done", "mask", "env_done", "bbc", "tcpa", "dcpa",
                 "conf_cur", "conf_pre")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        _lib = ctypes.CDLL(_SO)
        _lib.oc_step.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(_State), ctypes.c_void_p, ctypes.POINTER(_Out)]
        _lib.oc_reset.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(_State), ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(_Out)]
        _lib.oc_observe.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(_State), ctypes.POINTER(_Out)]
        _lib.oc_bound_crash.argtypes = [ctypes.c_double] * 4 + [ctypes.c_void_p]
        for f in (_lib.oc_goal_reached, _lib.oc_building_hit):
            f.argtypes = [ctypes.c_double] * 4
        _lib.oc_cross_track.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int]
        _lib.oc_cross_track.restype = ctypes.c_double
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class BatchedOracle:
    def __init__(self, E, N, occ, W=32, radar_mode=0, compat=True, episode_length=EPISODE_LENGTH,
                 bound=BOUND, with_tdcpa=False, team_reward=True, variant="att"):
        """variant "att" (one_model_att) or "wgru" (randomOD_Wgru_radar, config 4: obstacle radar,
        6-wide own rows, per-agent WGRU ss_reward, max_spd 10, episode_length 150 by default)."""
        self.E, self.N, self.W = E, N, W
        self.K = N - 1
        self.variant = {"att": 0, "wgru": 1}[variant]
        vmax = 5.0
        if self.variant:
            from .wgru_env_ref import EPISODE_LENGTH as WGRU_LEN, VMAX as WGRU_VMAX
            assert W <= 32, "the WGRU goal list is a 32-bit removal mask"
            radar_mode, team_reward, vmax = 1, False, float(WGRU_VMAX)
            episode_length = WGRU_LEN if episode_length == EPISODE_LENGTH else episode_length
        self.D0 = 6 if self.variant else 6 + 4 * self.K
        occ = np.asarray(occ, dtype=np.uint8)
        self.occ = np.ascontiguousarray(occ[None] if occ.ndim == 2 else occ)      # [n_maps][gw][gh]
        self.cfg = _Cfg(E, N, W, radar_mode, 1 if compat else 0, 1 if team_reward else 0, episode_length,
                        self.occ.shape[1], self.occ.shape[2], (ctypes.c_double * 4)(*[float(b) for b in bound]),
                        _p(self.occ), self.occ.shape[0], self.variant, vmax)
        z = lambda *s, dt=np.float64: np.zeros(s, dtype=dt)
        self.pos, self.vel, self.pre_pos, self.pre_vel, self.goal = (z(E, N, 2) for _ in range(5))
        self.wp = z(E, N, W, 2)
        self.wp_cur = z(E, N, dt=np.int32)
        self.wp_cnt = z(E, N, dt=np.int32)
        self.reach = z(E, N, dt=np.uint8)
        self.wall = z(E, N, dt=np.int32)
        self.step_count = z(E, dt=np.int32)
        self.map_idx = z(E, dt=np.int32)
        self.start = z(E, N, 2)
        self.state = _State(*[_p(a) for a in (self.pos, self.vel, self.pre_pos, self.pre_vel, self.goal, self.wp,
                                               self.wp_cur, self.wp_cnt, self.reach, self.wall, self.step_count,
                                               self.map_idx, self.start)])
        self.own = z(E, N, self.D0, dt=np.float32)
        self.radar = z(E, N, N_RAYS, dt=np.float32)
        self.nei = z(E, N, self.K, 6, dt=np.float32)
        self.reward = z(E, N, dt=np.float32)
        self.done = z(E, N, dt=np.uint8)
        self.mask = z(E, N, dt=np.uint8)
        self.env_done = z(E, dt=np.uint8)
        self.bbc = z(E, 4, dt=np.uint8)
        if with_tdcpa:
            self.tcpa, self.dcpa = z(E, N, self.K), z(E, N, self.K)
            self.conf_cur, self.conf_pre = z(E, N, dt=np.int32), z(E, N, dt=np.int32)
        else:
            self.tcpa = self.dcpa = self.conf_cur = self.conf_pre = None
        self.out = _Out(*[_p(a) for a in (self.own, self.radar, self.nei, self.reward, self.done, self.mask,
                                           self.env_done, self.bbc, self.tcpa, self.dcpa, self.conf_cur,
                                           self.conf_pre)])

    def reset(self, start, wps, wp_cnt, env_mask=None, map_idx=None):
        """Install OD (and, with a map stack, each env's map) for the masked envs (all if None)."""
        if map_idx is not None:
            map_idx = np.ascontiguousarray(map_idx, dtype=np.int32)
            assert map_idx.shape == (self.E,) and map_idx.min() >= 0 and map_idx.max() < self.occ.shape[0]
        start = np.ascontiguousarray(start, dtype=np.float64)
        wps = np.ascontiguousarray(wps, dtype=np.float64)
        wp_cnt = np.ascontiguousarray(wp_cnt, dtype=np.int32)
        m = None if env_mask is None else np.ascontiguousarray(env_mask, dtype=np.uint8)
        lib().oc_reset(ctypes.byref(self.cfg), ctypes.byref(self.state), _p(m), _p(start), _p(wps), _p(wp_cnt),
                       _p(map_idx), ctypes.byref(self.out))

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.float32)
        assert a.shape == (self.E, self.N, 2)
        lib().oc_step(ctypes.byref(self.cfg), ctypes.byref(self.state), _p(a), ctypes.byref(self.out))

    def observe(self):
        lib().oc_observe(ctypes.byref(self.cfg), ctypes.byref(self.state), ctypes.byref(self.out))


def bound_crash(x0, y0, x1, y1, bound=BOUND):
    b = np.array(bound, dtype=np.float64)
    return bool(lib().oc_bound_crash(x0, y0, x1, y1, _p(b)))


def goal_reached(px, py, gx, gy):
    return bool(lib().oc_goal_reached(px, py, gx, gy))


def building_hit(px, py, cx, cy):
    return bool(lib().oc_building_hit(px, py, cx, cy))


def cross_track(px, py, start, wps):
    """The C oracle's WGRU cross-track distance to the path start, wps[0..n)."""
    st = np.ascontiguousarray(start, dtype=np.float64)
    w = np.ascontiguousarray(wps, dtype=np.float64)
    return float(lib().oc_cross_track(px, py, _p(st), _p(w), len(w)))
