"""MPE ``simple_spread`` on the device: SURVEY.md section 8(f) row f4 (config 1, MADDPG_SS_baseV3).

``BatchedSpread`` runs E simple_spread worlds per launch (include/aac_mpe.h): fp64 state in HBM,
one thread per world.  ``make_env("simple_spread")`` returns a ``MultiAgentEnv`` facade with the
reference's surface (SS/env/make_env.py, SS/env/multiagent/environment.py:80-122): ``n``,
``action_space`` / ``observation_space`` shapes, ``reset() -> obs_n`` and
``step(action_n) -> (obs_n, reward_n, done_n, info_n)``, so ``SS/ma_main_MADDPGv3_ss.py`` drives it
unchanged.  The facade's reset draws positions with numpy's global RNG in the reference's order
(agents, then landmarks, simple_spread.py:38-44), so a seeded run starts from the same worlds;
the physics, rewards and observations run on the GPU.  The vendored ``_set_action`` scales each
policy action row by 5 in place (environment.py:193-197); with ``compat=True`` the facade does
the same to float32 numpy rows it is given.
"""
import ctypes
from types import SimpleNamespace

import numpy as np
import torch

from . import _native

vp, i32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64
_L = None


def lib():
    global _L
    if _L is None:
        L = _native.lib()
        L.aac_mpe_last_error.restype = ctypes.c_char_p
        L.aac_mpe_step.argtypes = [vp, vp, vp, vp, i32, i32, i32, vp, vp, vp]
        L.aac_mpe_observe.argtypes = [vp, vp, vp, i32, i32, i32, vp, vp, vp]
        L.aac_mpe_reset.argtypes = [vp, vp, vp, i32, i32, i32, vp, u64, vp, vp]
        _L = L
    return _L


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().aac_mpe_last_error().decode(errors='replace')}")


def _p(t):
    return None if t is None else vp(t.data_ptr())


def _s():
    return vp(torch.cuda.current_stream().cuda_stream)


class BatchedSpread:
    """E simple_spread worlds (N agents, L landmarks) on one GPU."""

    def __init__(self, E, N=3, L=3, device="cuda", seed=0):
        self.E, self.N, self.L = E, N, L
        self.obs_dim = 4 + 2 * L + 4 * (N - 1)
        d = torch.device(device)
        f64 = dict(dtype=torch.float64, device=d)
        self.pos, self.vel = torch.zeros(E, N, 2, **f64), torch.zeros(E, N, 2, **f64)
        self.lmk = torch.zeros(E, L, 2, **f64)
        self.obs = torch.zeros(E, N, self.obs_dim, dtype=torch.float32, device=d)
        self.rew = torch.zeros(E, N, **f64)
        self.seed = int(seed)
        self.counter = torch.zeros(1, dtype=torch.int64, device=d)

    def reset(self, env_mask=None):
        """Device reset_world of the masked envs (hash RNG), then their observations."""
        _chk(lib().aac_mpe_reset(_p(self.pos), _p(self.vel), _p(self.lmk), self.E, self.N, self.L, _p(env_mask),
                                 u64(self.seed), _p(self.counter), _s()), "aac_mpe_reset")
        return self.observe()

    def set_state(self, pos, vel, lmk):
        self.pos.copy_(torch.as_tensor(pos, dtype=torch.float64).reshape(self.pos.shape))
        self.vel.copy_(torch.as_tensor(vel, dtype=torch.float64).reshape(self.vel.shape))
        self.lmk.copy_(torch.as_tensor(lmk, dtype=torch.float64).reshape(self.lmk.shape))

    def observe(self):
        _chk(lib().aac_mpe_observe(_p(self.pos), _p(self.vel), _p(self.lmk), self.E, self.N, self.L, _p(self.obs),
                                   _p(self.rew), _s()), "aac_mpe_observe")
        return self.obs

    def step(self, act):
        """act (E, N, 2) f32 on the device -> (obs (E, N, obs_dim) f32, rew (E, N) f64)."""
        assert act.dtype == torch.float32 and act.is_contiguous() and act.shape == (self.E, self.N, 2)
        _chk(lib().aac_mpe_step(_p(self.pos), _p(self.vel), _p(self.lmk), _p(act), self.E, self.N, self.L,
                                _p(self.obs), _p(self.rew), _s()), "aac_mpe_step")
        return self.obs, self.rew


class MultiAgentEnv:
    """SS/env/multiagent/environment.py surface over one device world (E = 1)."""

    def __init__(self, N=3, L=3, device="cuda", compat=True):
        self.core = BatchedSpread(1, N, L, device)
        self.n = N
        self.compat = compat
        self.shared_reward = False            # world.collaborative = False (simple_spread.py:12)
        self.time = 0
        self.action_space = [SimpleNamespace(n=5, shape=(2,)) for _ in range(N)]   # Discrete(5) declared
        self.observation_space = [SimpleNamespace(shape=(self.core.obs_dim,)) for _ in range(N)]
        self.world = SimpleNamespace(agents=[SimpleNamespace(name=f"agent {i}", size=0.15, state=SimpleNamespace())
                                             for i in range(N)],
                                     landmarks=[SimpleNamespace(name=f"landmark {j}", state=SimpleNamespace())
                                                for j in range(L)],
                                     dim_p=2, dim_c=2, dt=0.1, damping=0.25)
        self._act = torch.zeros(1, N, 2, dtype=torch.float32, device=self.core.pos.device)

    def _sync_world(self):
        pos, vel, lmk = self.core.pos[0].cpu().numpy(), self.core.vel[0].cpu().numpy(), self.core.lmk[0].cpu().numpy()
        for i, a in enumerate(self.world.agents):
            a.state.p_pos, a.state.p_vel, a.state.c = pos[i].copy(), vel[i].copy(), np.zeros(2)
        for j, lm in enumerate(self.world.landmarks):
            lm.state.p_pos, lm.state.p_vel = lmk[j].copy(), np.zeros(2)

    def _lists(self):
        obs = self.core.obs[0].double().cpu().numpy()
        return [obs[i] for i in range(self.n)]

    def reset(self):
        N, L = self.core.N, self.core.L
        pos = np.stack([np.random.uniform(-1, +1, 2) for _ in range(N)])
        lmk = np.stack([np.random.uniform(-1, +1, 2) for _ in range(L)])
        self.core.set_state(pos[None], np.zeros((1, N, 2)), lmk[None])
        self.core.observe()
        self._sync_world()
        return self._lists()

    def step(self, action_n):
        a = np.stack([np.asarray(x, dtype=np.float32).reshape(-1)[:2] for x in action_n])
        self._act.copy_(torch.from_numpy(a).reshape(1, self.n, 2))
        if self.compat:           # u *= sensitivity on the caller's float32 rows (environment.py:197)
            for x in action_n:
                if isinstance(x, np.ndarray) and x.dtype == np.float32:
                    x[:2] *= 5.0
        _, rew = self.core.step(self._act)
        self._sync_world()
        r = rew[0].cpu().numpy()
        reward_n = [float(v) for v in r]
        if self.shared_reward:
            reward_n = [float(np.sum(r))] * self.n
        return self._lists(), reward_n, [False] * self.n, {"n": [{} for _ in range(self.n)]}


def make_env(scenario_name, benchmark=False, device="cuda"):
    """SS/env/make_env.py for the one scenario the reference trains (simple_spread)."""
    if scenario_name != "simple_spread":
        raise NotImplementedError(f"scenario {scenario_name!r}: only simple_spread (SS/ma_main) is built")
    if benchmark:
        raise NotImplementedError("benchmark_data is not used by SS/ma_main")
    return MultiAgentEnv(device=device)
