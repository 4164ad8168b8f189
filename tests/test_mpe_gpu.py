"""GPU tests of the batched MPE simple_spread (include/aac_mpe.h)
against the numpy fp64 restatement of the vendored MPE (oracle/mpe_ref.py)."""
import numpy as np
import pytest
import torch

from oracle import mpe_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _states(E, N, L, seed):
    rng = np.random.default_rng(seed)
    pos = rng.uniform(-1, 1, (E, N, 2))
    vel = rng.normal(0, 0.5, (E, N, 2))
    lmk = rng.uniform(-1, 1, (E, L, 2))
    # contact cases: agent 1 near agent 0 at distances around 2 * size = 0.3 (soft contact and the
    # reward's strict < 0.3 collision test)
    k = E // 4 if N > 1 else 0
    ang = rng.uniform(0, 2 * np.pi, k)
    if k:
        d = np.concatenate([rng.uniform(0.05, 0.35, k - 8),
                            0.3 + np.array([-1e-9, 1e-9, -1e-6, 1e-6, 0, 2e-3, -2e-3, 1e-4])])
        pos[:k, 1] = pos[:k, 0] + np.stack([np.cos(ang), np.sin(ang)], 1) * d[:, None]
    act = rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)
    return pos, vel, lmk, act


@pytest.mark.parametrize("N,L", [(3, 3), (5, 4), (1, 2)])
def test_mpe_step_matches_oracle(native_lib, N, L):
    from multi_agent_aac_amd import mpe
    E = 512
    pos, vel, lmk, act = _states(E, N, L, N * 10 + L)
    env = mpe.BatchedSpread(E, N, L, DEV)
    env.set_state(pos, vel, lmk)
    obs, rew = env.step(torch.from_numpy(act).to(DEV))
    gp, gv, go, gr = env.pos.cpu().numpy(), env.vel.cpu().numpy(), obs.cpu().numpy(), rew.cpu().numpy()
    for e in range(E):
        p, v = mpe_ref.step(pos[e], vel[e], lmk[e], act[e])
        np.testing.assert_allclose(gp[e], p, rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(gv[e], v, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(gr[e], mpe_ref.reward(p, lmk[e]), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(go[e], mpe_ref.observe(p, v, lmk[e]).astype(np.float32), rtol=1e-6, atol=1e-6)


def test_mpe_facade_100_steps(native_lib):
    """Config 1: the reference loop shape (make_env, reset, 100 x step with per-agent float32
    action rows) against the restatement from the same numpy seed."""
    from multi_agent_aac_amd import mpe
    np.random.seed(11)
    env = mpe.make_env("simple_spread")
    obs = env.reset()
    assert env.n == 3 and len(obs) == 3 and obs[0].shape == (18,)
    np.random.seed(11)
    p, v, lm = mpe_ref.reset(np.random)
    np.testing.assert_array_equal(np.stack([a.state.p_pos for a in env.world.agents]), p)
    rng = np.random.default_rng(5)
    for t in range(100):
        acts = [rng.uniform(-1, 1, 2).astype(np.float32) for _ in range(3)]
        ref_act = np.stack([a.copy() for a in acts])
        obs, rew, done, info = env.step(acts)
        p, v = mpe_ref.step(p, v, lm, ref_act)
        # contact forces are stiff (1/k = 1e3), so last-bit differences of exp/log1p grow along a
        # trajectory; each single step is checked to 1e-13 above
        np.testing.assert_allclose(np.stack(obs), mpe_ref.observe(p, v, lm), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(rew, mpe_ref.reward(p, lm), rtol=1e-5, atol=1e-5)
        assert done == [False] * 3 and len(info["n"]) == 3
        np.testing.assert_array_equal(np.stack(acts), ref_act * np.float32(5.0))   # u *= 5 in place


def test_mpe_device_reset(native_lib):
    from multi_agent_aac_amd import mpe
    E = 4096
    env = mpe.BatchedSpread(E, 3, 3, DEV, seed=4)
    env.reset()
    p0, l0 = env.pos.clone(), env.lmk.clone()
    assert float(p0.abs().max()) <= 1.0 and float(env.vel.abs().max()) == 0.0
    assert abs(float(p0.mean())) < 0.05 and abs(float(p0.std()) - 1 / np.sqrt(3)) < 0.02
    env.vel.fill_(1.0)
    mask = torch.zeros(E, dtype=torch.uint8, device=DEV)
    mask[::2] = 1
    env.reset(mask)
    assert not torch.equal(env.pos[::2], p0[::2]) and torch.equal(env.pos[1::2], p0[1::2])
    assert torch.equal(env.lmk[1::2], l0[1::2]) and float(env.vel[::2].abs().max()) == 0.0
    assert float(env.vel[1::2].min()) == 1.0 and int(env.counter) == 2
    # observe after a reset gives the reference's reset-time observation
    obs = env.observe().cpu().numpy()
    e = 6
    want = mpe_ref.observe(env.pos[e].cpu().numpy(), env.vel[e].cpu().numpy(), env.lmk[e].cpu().numpy())
    np.testing.assert_allclose(obs[e], want.astype(np.float32), rtol=1e-6, atol=1e-6)
