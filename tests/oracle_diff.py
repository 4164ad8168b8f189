"""Runtime CPU-oracle diff mode (SURVEY.md section 5 debug surface).

``OracleDiff(trainer, every=k, n_envs=64)`` hooks a ``Trainer`` (its generic pre / post step hooks,
``multi_agent_aac_amd/trainer.py``): every k-th eager step it snapshots a sampled subset of the
envs' state before the step (``env.get_state``), and after the GPU step re-runs exactly those envs on
the C oracle (``oracle/c_oracle.py``, the restatement of ATT/env:2166-2520 and WGRU/env:824-2131)
from that state with the GPU's own actions, then raises ``OracleMismatch`` on the first difference:
masks / done / bbc / env_done bit-exact, reward within 1e-5 for every sampled env, the next
observation rows within 1e-5 for the sampled envs that did not finish (the fused tail has already
overwritten a finished env's rows with its reset observation).

This lives under tests/: the oracle is test infrastructure and the product never imports it; the
product only exposes the hooks.  One map (``maps == 1``) -- the oracle holds one occupancy grid.
"""
import numpy as np
import torch

from oracle import c_oracle

ATOL = 1e-5


class OracleMismatch(AssertionError):
    pass


class OracleDiff:
    def __init__(self, trainer, every=10, n_envs=64, seed=0):
        env = trainer.env
        if env.occ.shape[0] != 1:
            raise ValueError("OracleDiff: one map only (the oracle holds one occupancy grid)")
        self.tr, self.every, self.n = trainer, int(every), min(int(n_envs), env.E)
        self.rng = np.random.default_rng(seed)
        self.t, self.active, self.checked = 0, False, 0
        self.co = c_oracle.BatchedOracle(self.n, env.N, env.occ[0], W=env.W, radar_mode=env.radar_mode,
                                         variant="wgru" if env.variant else "att")
        trainer.pre_step_hooks.append(self.pre)
        trainer.post_step_hooks.append(self.post)

    def detach(self):
        self.tr.pre_step_hooks.remove(self.pre)
        self.tr.post_step_hooks.remove(self.post)

    def pre(self, tr):
        self.t += 1
        self.active = self.t % self.every == 0
        if not self.active:
            return
        self.idx = np.sort(self.rng.choice(tr.env.E, self.n, replace=False))
        sel = torch.from_numpy(self.idx).to(tr.env.device)
        s = {k: v[sel].cpu().numpy() for k, v in tr.env.get_state().items()}
        co = self.co
        co.pos[:] = s["pos"]; co.vel[:] = s["vel"]; co.pre_pos[:] = s["pre_pos"]; co.pre_vel[:] = s["pre_vel"]
        co.goal[:] = s["goal"]; co.wp[:] = s["wp"]; co.wp_cur[:] = s["wp_cur"]; co.wp_cnt[:] = s["wp_cnt"]
        co.reach[:] = s["reach"]; co.wall[:] = s["wall"]; co.step_count[:] = s["step"]
        co.start[:] = s["start"]

    def post(self, tr, act, c, n):
        if not self.active:
            return
        sel = torch.from_numpy(self.idx).to(act.device)
        a = act[sel].detach().cpu().numpy().astype(np.float32)
        self.co.step(a)
        g = {f: getattr(n, f)[sel].cpu().numpy() for f in ("reward", "mask", "done", "bbc", "env_done", "own",
                                                           "radar", "nei")}
        co, where = self.co, f"step {self.t}"
        for f in ("mask", "done", "bbc", "env_done"):
            if not np.array_equal(g[f], getattr(co, f)):
                bad = np.nonzero((g[f] != getattr(co, f)).reshape(self.n, -1).any(1))[0]
                raise OracleMismatch(f"{where}: {f} differs in envs {self.idx[bad][:8].tolist()}")
        if not np.allclose(g["reward"], co.reward, rtol=0, atol=ATOL):
            raise OracleMismatch(f"{where}: reward max |diff| {np.abs(g['reward'] - co.reward).max():.3g}")
        live = ~co.env_done.astype(bool)
        for f in ("own", "radar", "nei"):
            d = np.abs(g[f][live] - getattr(co, f)[live])
            if d.size and d.max() > ATOL:
                raise OracleMismatch(f"{where}: next {f} max |diff| {d.max():.3g}")
        self.checked += 1
