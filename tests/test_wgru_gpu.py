"""GPU parity of the randomOD_Wgru_radar env variant (config 4; WGRU/env:824-2131,
WGRU/ma_main:653-661) against the C oracle's variant 1, itself checked bit for bit against the
reference-shaped restatement oracle/wgru_env_ref.py (tests/test_wgru_cpu.py): masks / done / bbc /
env_done / goal-list state bit-exact, fp32 outputs within 1e-5, fp64 state within 1e-12."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from tests.helpers import W_DEFAULT, bank_draw, random_od, steer, wgru_targets
from tests.test_env_gpu import ATOL, _cmp_step, _cmp_out, _state_to_oracle

pytestmark = pytest.mark.gpu


def _env(E, N, occ, **kw):
    from multi_agent_aac_amd.env import BatchedEnv
    return BatchedEnv(E, N, occ, max_wp=W_DEFAULT, variant="wgru", **kw)


def _targets(co):
    tg = wgru_targets(co.wp, co.wp_cur, co.wp_cnt)
    tg[:, 1::2] = co.goal[:, 1::2]        # odd agents fly straight at goal[-1] (final-goal pops)
    return tg


@pytest.mark.parametrize("E,N,steps", [(96, 3, 80), (384, 8, 80), (4096, 8, 10)])
def test_wgru_step_injected_parity(native_lib, occ, E, N, steps):
    st, wps, cnt = random_od(occ, E, N, seed=300 + N)
    env = _env(E, N, occ)
    co = c_oracle.BatchedOracle(E, N, occ, W=W_DEFAULT, variant="wgru")
    assert env.D0 == co.D0 == 6
    env.reset(st, wps, cnt)
    co.reset(st, wps, cnt)
    torch.cuda.synchronize()
    _cmp_out(env.bufs, co, "reset")
    rng = np.random.default_rng(N)
    seen, moves = 0, 0
    for t in range(steps):
        _state_to_oracle(env, co)       # identical inputs (removes libm ulp drift)
        act = steer(co.pos, co.vel, _targets(co), rng)
        g0 = co.goal.copy()
        env.step(torch.from_numpy(act).cuda())
        co.step(act)
        torch.cuda.synchronize()
        _cmp_step(env.bufs, co, f"wgru N{N} t{t}")
        s = env.get_state()
        np.testing.assert_allclose(s["pos"].cpu().numpy(), co.pos, rtol=1e-12, atol=1e-12)
        assert np.array_equal(s["wp_cur"].cpu().numpy(), co.wp_cur)      # removed-waypoint bits
        assert np.array_equal(s["goal"].cpu().numpy(), co.goal)          # goal[-1] after pops
        assert np.array_equal(s["reach"].cpu().numpy(), co.reach)
        assert np.array_equal(s["wall"].cpu().numpy(), co.wall)
        seen |= int(np.bitwise_or.reduce(co.mask.ravel()))
        moves += int(np.any(co.goal != g0, -1).sum())
        done = co.env_done.astype(bool)
        if done.any():
            st2, wps2, cnt2 = random_od(occ, E, N, seed=1000 * t + N)
            env.reset(st2, wps2, cnt2, env_mask=done.astype(np.uint8))
            co.reset(st2, wps2, cnt2, env_mask=done.astype(np.uint8))
            torch.cuda.synchronize()
            _cmp_out(env.bufs, co, f"reset t{t}")
    if steps >= 80:
        # waypoint (bit4), goal (bit2 + bit5) and a building crash (bit3) seen; final goal popped
        assert seen & 0b111100 == 0b111100, bin(seen)
        assert moves > 0


def test_wgru_auto_reset_bank(native_lib, occ):
    """GPU bank auto-reset installs the drawn OD and its reference path (the start): the steps that
    follow match the oracle reset with the same draw."""
    from multi_agent_aac_amd import world
    E, N, seed = 64, 8, 777
    bank = world.ODBank(occ, n_pairs=4096, seed=9, max_wp=W_DEFAULT)
    env = _env(E, N, occ)
    env.set_od_bank(bank, seed=seed)
    env.auto_reset(None)
    st = np.zeros((E, N, 2)); wps = np.zeros((E, N, W_DEFAULT, 2)); cnt = np.zeros((E, N), np.int32)
    for e in range(E):
        idx = bank_draw(bank.start, bank.n_pairs, seed, e, 1, N)
        st[e] = bank.start[idx]; wps[e] = bank.wps[idx]; cnt[e] = bank.cnt[idx]
    co = c_oracle.BatchedOracle(E, N, occ, W=W_DEFAULT, variant="wgru")
    co.reset(st, wps, cnt)
    torch.cuda.synchronize()
    _cmp_out(env.bufs, co, "auto-reset")
    rng = np.random.default_rng(1)
    for t in range(30):
        _state_to_oracle(env, co)
        act = steer(co.pos, co.vel, _targets(co), rng)
        env.step(torch.from_numpy(act).cuda())
        co.step(act)
        torch.cuda.synchronize()
        _cmp_step(env.bufs, co, f"bank t{t}")


def test_wgru_set_state_carries_reference_path(native_lib, occ):
    """A state injected from a different OD (set_state of every key, `start` included) steps like
    the oracle reset with that OD: the cross-track reward reads the injected reference-path origin,
    not the one the env's own last reset wrote."""
    E, N = 64, 8
    st1, wps1, cnt1 = random_od(occ, E, N, seed=41)
    st2, wps2, cnt2 = random_od(occ, E, N, seed=42)
    env, donor = _env(E, N, occ), _env(E, N, occ)
    env.reset(st1, wps1, cnt1)
    donor.reset(st2, wps2, cnt2)
    torch.cuda.synchronize()
    s = donor.get_state()
    assert not np.array_equal(s["start"].cpu().numpy(), env.get_state()["start"].cpu().numpy())
    env.set_state(**s)
    np.testing.assert_array_equal(env.get_state()["start"].cpu().numpy(), st2)
    co = c_oracle.BatchedOracle(E, N, occ, W=W_DEFAULT, variant="wgru")
    co.reset(st2, wps2, cnt2)
    rng = np.random.default_rng(3)
    for t in range(5):
        _state_to_oracle(env, co)
        act = steer(co.pos, co.vel, _targets(co), rng)
        env.step(torch.from_numpy(act).cuda())
        co.step(act)
        torch.cuda.synchronize()
        _cmp_step(env.bufs, co, f"injected t{t}")


def test_wgru_config_checks(native_lib, occ):
    from multi_agent_aac_amd import _native
    from multi_agent_aac_amd.env import BatchedEnv
    env = BatchedEnv(8, 4, occ, variant="wgru")
    assert env.cfg.radar_mode == 1 and env.cfg.team_reward == 0 and env.cfg.vmax == 10.0
    assert env.cfg.episode_length == 150 and env.bufs.own.shape == (8, 4, 6)
    # explicit values are kept (5 / 50 used to be rewritten to the variant defaults)
    e2 = BatchedEnv(8, 4, occ, variant="wgru", vmax=5.0, episode_length=50)
    assert e2.cfg.vmax == 5.0 and e2.cfg.episode_length == 50
    with pytest.raises(ValueError):
        BatchedEnv(8, 4, occ, variant="wgru", radar_mode="drones")
    with pytest.raises(ValueError):
        BatchedEnv(8, 4, occ, variant="wgru", team_reward=True)
    cfg = env.cfg
    cfg.radar_mode = 0                      # variant 1 needs the obstacle radar
    import ctypes
    h = ctypes.c_void_p()
    assert _native.lib().aac_env_create(ctypes.byref(cfg), 0, ctypes.byref(h)) < 0
