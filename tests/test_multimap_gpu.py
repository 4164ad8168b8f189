"""Multi-map random OD (MADDPG_ownENV_randomOD_radar_multipleMap): a
stack of 8 synthetic maps (seeds 2026..2033), one OD bank per map, the map drawn per
env episode by the GPU auto-reset as random_map_idx = random.randrange(len(world_map_2D_collection))
(multipleMap/ma_main:464-465), radar and building predicates on the env's own map.  Checked against
the C oracle with the same per-env map index."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from tests.helpers import W_DEFAULT, bank_draw, map_draw

pytestmark = pytest.mark.gpu
SEEDS = list(range(2026, 2034))


@pytest.fixture(scope="module")
def stack():
    from multi_agent_aac_amd import world
    return world.map_stack(SEEDS)


@pytest.fixture(scope="module")
def banks(stack, native_lib):
    from multi_agent_aac_amd import world
    return world.MapBanks(stack, n_pairs=4096, seed=11, max_wp=W_DEFAULT)


def _state_to_oracle(env, co):
    s = {k: v.cpu().numpy() for k, v in env.get_state().items()}
    co.pos[:] = s["pos"]; co.vel[:] = s["vel"]; co.pre_pos[:] = s["pre_pos"]; co.pre_vel[:] = s["pre_vel"]
    co.goal[:] = s["goal"]; co.wp[:] = s["wp"]; co.wp_cur[:] = s["wp_cur"]; co.wp_cnt[:] = s["wp_cnt"]
    co.reach[:] = s["reach"]; co.wall[:] = s["wall"]; co.step_count[:] = s["step"]; co.map_idx[:] = s["map_idx"]


def test_maps_differ(stack):
    assert stack.shape == (8, 23, 13)
    assert len({m.tobytes() for m in stack}) == 8


@pytest.mark.parametrize("mode", [1, 2])
def test_injected_parity_mixed_maps(stack, banks, mode):
    """Explicit reset with a mixed per-env map index (each env's OD from its own map's bank), then
    20 steps from identical injected state: masks / done / bbc / env_done bit-exact, obs / radar /
    reward within 1e-5, positions 1e-12 (obstacle and combined radar read the env's map)."""
    from multi_agent_aac_amd.env import BatchedEnv
    E, N = 512, 5
    rng = np.random.default_rng(mode)
    mi = rng.integers(0, 8, E).astype(np.int32)
    st = np.zeros((E, N, 2)); wps = np.zeros((E, N, W_DEFAULT, 2)); cnt = np.zeros((E, N), np.int32)
    for m in range(8):
        sel = np.where(mi == m)[0]
        if len(sel):
            a, b, c = banks.banks[m].sample_env_od(len(sel), N, rng)
            st[sel], wps[sel], cnt[sel] = a, b, c
    env = BatchedEnv(E, N, stack, radar_mode=mode, max_wp=W_DEFAULT)
    co = c_oracle.BatchedOracle(E, N, stack, W=W_DEFAULT, radar_mode=mode)
    env.reset(st, wps, cnt, map_idx=mi)
    co.reset(st, wps, cnt, map_idx=mi)
    torch.cuda.synchronize()
    assert np.array_equal(env.get_state()["map_idx"].cpu().numpy(), mi)
    for name in ("own", "radar", "nei"):
        np.testing.assert_allclose(getattr(env.bufs, name).cpu().numpy(), getattr(co, name), rtol=0, atol=1e-5)
    seen = 0
    for t in range(20):
        _state_to_oracle(env, co)
        act = rng.uniform(-1, 1, size=(E, N, 2)).astype(np.float32)
        env.step(torch.from_numpy(act).cuda())
        co.step(act)
        torch.cuda.synchronize()
        b = env.bufs
        for name in ("own", "radar", "nei", "reward"):
            np.testing.assert_allclose(getattr(b, name).cpu().numpy(), getattr(co, name), rtol=0, atol=1e-5,
                                       err_msg=f"t{t} {name}")
        for name in ("mask", "done", "bbc", "env_done"):
            assert np.array_equal(getattr(b, name).cpu().numpy(), getattr(co, name)), (t, name)
        np.testing.assert_allclose(env.get_state()["pos"].cpu().numpy(), co.pos, rtol=1e-12, atol=1e-12)
        seen |= int(np.bitwise_or.reduce(co.mask.ravel()))
    assert seen & 0b1001 == 0b1001, bin(seen)          # bound crashes and building contacts
    # the same state on a single map gives different radar rows: the map matters
    co0 = c_oracle.BatchedOracle(E, N, stack, W=W_DEFAULT, radar_mode=mode)
    co0.reset(st, wps, cnt, map_idx=np.zeros(E, np.int32))
    co1 = c_oracle.BatchedOracle(E, N, stack, W=W_DEFAULT, radar_mode=mode)
    co1.reset(st, wps, cnt, map_idx=mi)
    assert not np.array_equal(co0.radar, co1.radar)


def test_auto_reset_draws_map_then_od(stack, banks):
    """Bank auto-reset with per-map banks: env e's map is the restated draw for (seed, e, episode),
    its agents' ODs are the restated draws from that map's bank, and the observation equals the C
    oracle's on that map."""
    from multi_agent_aac_amd.env import BatchedEnv
    E, N, seed = 96, 5, 4242
    env = BatchedEnv(E, N, stack, radar_mode="combined", max_wp=W_DEFAULT)
    env.set_od_bank(banks, seed=seed)
    env.auto_reset(None)
    torch.cuda.synchronize()
    s = {k: v.cpu().numpy() for k, v in env.get_state().items()}
    st = np.zeros((E, N, 2)); wps = np.zeros((E, N, W_DEFAULT, 2)); cnt = np.zeros((E, N), np.int32)
    mi = np.zeros(E, np.int32)
    for e in range(E):
        m = map_draw(seed, e, 1, 8)
        mi[e] = m
        off, n = int(banks.offsets[m]), int(banks.counts[m])
        idx = bank_draw(banks.start, n, seed, e, 1, N, off=off)
        st[e], wps[e], cnt[e] = banks.start[idx], banks.wps[idx], banks.cnt[idx]
    assert np.array_equal(s["map_idx"], mi)
    assert np.array_equal(s["pos"], st) and np.array_equal(s["wp"], wps) and np.array_equal(s["wp_cnt"], cnt)
    co = c_oracle.BatchedOracle(E, N, stack, W=W_DEFAULT, radar_mode=2)
    co.reset(st, wps, cnt, map_idx=mi)
    for name in ("own", "radar", "nei"):
        np.testing.assert_allclose(getattr(env.bufs, name).cpu().numpy(), getattr(co, name), rtol=0, atol=1e-5)


def test_map_draw_uniform(stack, banks):
    """Over 4 auto-resets of 8192 envs the drawn map is uniform over the 8 maps (chi-square, 7 dof,
    p ~ 1e-6 bound) and each env's map changes between episodes."""
    from multi_agent_aac_amd.env import BatchedEnv
    E, N = 8192, 3
    env = BatchedEnv(E, N, stack, radar_mode="obstacles", max_wp=W_DEFAULT)
    env.set_od_bank(banks, seed=7)
    counts = np.zeros(8)
    prev = None
    changed = 0
    ones = torch.ones(E, dtype=torch.uint8, device="cuda")
    for k in range(4):
        env.auto_reset(None if k == 0 else ones)
        mi = env.get_state()["map_idx"].cpu().numpy()
        counts += np.bincount(mi, minlength=8)
        if prev is not None:
            changed += int((mi != prev).sum())
        prev = mi
    exp = counts.sum() / 8
    chi2 = float(((counts - exp) ** 2 / exp).sum())
    assert chi2 < 35.0, (chi2, counts)
    assert changed > 0.8 * 3 * E          # ~7/8 of the redraws land on another map


def test_single_bank_refused_for_stack(stack):
    from multi_agent_aac_amd import world
    from multi_agent_aac_amd.env import BatchedEnv
    env = BatchedEnv(16, 3, stack, max_wp=W_DEFAULT)
    with pytest.raises(RuntimeError, match="one OD bank per map"):
        env.set_od_bank(world.ODBank(stack[0], n_pairs=256, seed=1, max_wp=W_DEFAULT))
