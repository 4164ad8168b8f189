"""CPU parity of the randomOD_Wgru_radar env variant (config 4): the reference-shaped scalar
restatement oracle/wgru_env_ref.py (WGRU/env:824-2131, WGRU/ma_main:653-661) against the batched C
oracle's variant 1, bit for bit; and the GEOS cross-track distance (WGRU/env:2621-2632) against an
exact-rational formulation."""
import math

import numpy as np
import pytest

from oracle import c_oracle, geos, wgru_env_ref, world_ref
from tests.helpers import W_DEFAULT, draw_env_od, pack_od, steer, wgru_targets


@pytest.mark.parametrize("N", [3, 8])
def test_wgru_scalar_vs_c_oracle(occ, N):
    E, T = 6, 120
    rng = np.random.default_rng(70 + N)
    pools = world_ref.target_pools(occ)
    ods = [draw_env_od(occ, N, rng, pools) for _ in range(E)]
    st, wps, cnt = pack_od(ods)
    co = c_oracle.BatchedOracle(E, N, occ, W=W_DEFAULT, variant="wgru")
    envs = [wgru_env_ref.WgruEnv(N, occ) for _ in range(E)]
    co.reset(st, wps, cnt)
    for e, env in enumerate(envs):
        o = env.reset(*ods[e])
        assert np.array_equal(co.own[e], o[0].astype(np.float32))
        assert np.array_equal(co.radar[e], o[1].astype(np.float32))
        assert np.array_equal(co.nei[e], o[2].astype(np.float32))
    seen, goal_moves = 0, 0
    for t in range(T):
        # even agents fly the waypoints in order, odd ones straight at goal[-1]: near it with earlier
        # waypoints left, the search pops the final goal itself (goal[-1] changes, WGRU/env:1818-1831)
        tg = wgru_targets(co.wp, co.wp_cur, co.wp_cnt)
        tg[:, 1::2] = co.goal[:, 1::2]
        act = steer(co.pos, co.vel, tg, rng)
        g_before = co.goal.copy()
        co.step(act)
        goal_moves += int(np.any(co.goal != g_before, -1).sum())
        ended = np.zeros(E, np.uint8)
        for e, env in enumerate(envs):
            (o, r, n), rew, d, cg, bbc, masks, over = env.full_step(act[e])
            assert np.array_equal(co.own[e], o.astype(np.float32)), (t, e)
            assert np.array_equal(co.radar[e], r.astype(np.float32)), (t, e)
            assert np.array_equal(co.nei[e], n.astype(np.float32)), (t, e)
            assert np.array_equal(co.reward[e], np.array([float(x) for x in rew], np.float32)), (t, e)
            assert np.array_equal(co.mask[e], np.array(masks, np.uint8)), (t, e)
            assert np.array_equal(co.done[e], np.array(d, np.uint8)), (t, e)
            assert np.array_equal(co.bbc[e], np.array(bbc, np.uint8)), (t, e)
            assert bool(co.env_done[e]) == over, (t, e)
            assert np.array_equal(co.pos[e], np.array([env.all_agents[i].pos for i in range(N)]))
            assert np.array_equal(co.goal[e], np.array([env.all_agents[i].goal[-1] for i in range(N)], float))
            seen |= int(np.bitwise_or.reduce(co.mask[e]))
            if over:                   # a new episode in both: a fresh OD for this env
                ods[e] = draw_env_od(occ, N, rng, pools)
                env.reset(*ods[e])
                ended[e] = 1
        if ended.any():
            st, wps, cnt = pack_od(ods)
            co.reset(st, wps, cnt, env_mask=ended)
    assert seen & 0b10000, "no waypoint reached"
    assert goal_moves > 0, "the final goal was never popped"


def _paths(rng, n):
    for _ in range(n):
        k = int(rng.integers(1, 6))
        pts = [(float(10 * rng.integers(46, 68)), float(10 * rng.integers(26, 38)))]
        for _ in range(k):
            x, y = pts[-1]
            if rng.random() < 0.5:
                pts.append((x + 10.0 * int(rng.integers(-4, 5)), y))
            else:
                pts.append((x, y + 10.0 * int(rng.integers(-4, 5))))
            if rng.random() < 0.3:
                pts.append((pts[-1][0] + 10.0, pts[-1][1] + 10.0))   # a diagonal step
        yield pts


def test_cross_track_vs_exact_and_c():
    rng = np.random.default_rng(3)
    n = 0
    for pts in _paths(rng, 300):
        for _ in range(10):
            x0, y0 = pts[int(rng.integers(len(pts)))]
            px, py = x0 + rng.uniform(-12, 12), y0 + rng.uniform(-12, 12)
            if rng.random() < 0.1:          # points on the path: exact zero / vertex cases
                px, py = x0, y0
            d = geos.cross_track_distance(px, py, pts)
            exact = math.sqrt(float(geos.point_polyline_distance_exact((px, py), pts)))
            assert abs(d - exact) <= 1e-12 * (1 + exact), (pts, px, py, d, exact)
            dc = c_oracle.cross_track(px, py, pts[0], pts[1:])
            assert dc == d
            n += 1
    assert n == 3000


def test_wgru_numpy_matches_c_oracle(occ):
    """The vectorised NumPy WGRU env (oracle/env_np.py, CPU-baseline mode 2 of config 4) against the C
    oracle from identical state every step: integer outputs equal, floats within 1e-5."""
    from oracle import env_np
    E, N = 32, 8
    rng = np.random.default_rng(5)
    pools = world_ref.target_pools(occ)
    st, wps, cnt = pack_od([draw_env_od(occ, N, rng, pools) for _ in range(E)])
    co = c_oracle.BatchedOracle(E, N, occ, W=W_DEFAULT, variant="wgru")
    ne = env_np.NumpyEnv(E, N, occ, W=W_DEFAULT, variant="wgru")
    co.reset(st, wps, cnt)
    own, radar, nei = ne.reset(st, wps, cnt)
    np.testing.assert_allclose(own, co.own, atol=1e-5)
    seen = 0
    for t in range(60):
        for k in ("pos", "vel", "pre_pos", "pre_vel", "wp_cur", "reach", "wall", "goal"):
            getattr(ne, k)[...] = getattr(co, k)
        ne.step_count[:] = co.step_count
        tg = wgru_targets(co.wp, co.wp_cur, co.wp_cnt)
        tg[:, 1::2] = co.goal[:, 1::2]
        act = steer(co.pos, co.vel, tg, rng)
        co.step(act)
        own, radar, nei, rew, done, mask, env_done, bbc = ne.step(act)
        np.testing.assert_allclose(own, co.own, atol=1e-5, err_msg=f"t{t}")
        np.testing.assert_allclose(radar, co.radar, atol=1e-5, err_msg=f"t{t}")
        np.testing.assert_allclose(rew, co.reward, atol=1e-5, err_msg=f"t{t}")
        assert np.array_equal(mask, co.mask) and np.array_equal(done, co.done), t
        assert np.array_equal(env_done, co.env_done) and np.array_equal(bbc, co.bbc), t
        assert np.array_equal(ne.wp_cur, co.wp_cur) and np.array_equal(ne.goal, co.goal), t
        seen |= int(np.bitwise_or.reduce(co.mask.ravel()))
        d = co.env_done.astype(bool)
        if d.any():
            s2, w2, c2 = pack_od([draw_env_od(occ, N, rng, pools) for _ in range(E)])
            co.reset(s2, w2, c2, env_mask=d.astype(np.uint8))
            ne.reset(s2, w2, c2, env_mask=d)
    assert seen & 0b111100 == 0b111100, bin(seen)
