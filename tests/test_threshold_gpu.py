"""The HIP env kernel on exact-threshold states (tests/thresholds.py):
drone contact at exactly 5 m, the near band's 2.5 / 10 m ends, a waypoint at exactly 5 m, goals on the
Minkowski 64-gon's apothem and vertices, the ATT/geometry_test.py known answer, 64-gons touching a
cell's edge or corner, circles and capsules touching each bound line, radar rays through another
agent's vertex or leaving its boundary, rays through an isolated cell's corner or along its edge --
each exactly on the threshold and one ulp either side.

Three launch forms go through the C ABI: the step kernel (aac_env_step), the fused step tail with a
replay ring (aac_env_step_tail: the exact radar fix also rewrites the ring's next-radar column), and
the reset kernel's radar (aac_env_reset from the threshold positions).  Each is checked
  * bit for bit against the C oracle (masks, done, bbc, env_done, the fp32 radar; obs / reward 1e-5);
  * against the reference's own semantics at the threshold: np.linalg.norm / GEOS point distances
    where the reference compares float distances, the exact rational predicates on the GEOS float
    vertices (oracle/geos.py) where it asks GEOS -- goal, building, bound, every radar ray;
  * with both outcomes of every boolean threshold occurring."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from tests import thresholds as T

pytestmark = pytest.mark.gpu
ATOL = 1e-5


def _np(t):
    return t.detach().cpu().numpy()


def _env(E, N, occ, mode, variant="att", **kw):
    from multi_agent_aac_amd.env import BatchedEnv
    return BatchedEnv(E, N, occ, radar_mode=mode, max_wp=32, variant=variant, **kw)


# (variant, radar mode): the ATT env in its three radar modes, the WGRU env (config 4) with its obstacle
# radar -- its reward's near-building penalty takes the radar minimum, so the exact fix-up recomputes the
# rewards of agents with a flagged ray
VARIANTS = [("att", 0), ("att", 1), ("att", 2), ("wgru", 1)]


def _install(env, st):
    E, N = st["pos"].shape[:2]
    env.set_state(pos=st["pos"], pre_pos=st["pre_pos"], vel=st["vel"], pre_vel=st["vel"], goal=st["goal"],
                  wp=st["wp"], wp_cur=np.zeros((E, N), np.int32), wp_cnt=st["cnt"],
                  reach=np.zeros((E, N), np.uint8), wall=np.zeros((E, N), np.int32), step=np.zeros(E, np.int32),
                  map_idx=np.zeros(E, np.int32), start=st["pos"])


def _cmp_oracle(b, co, where):
    for f in ("mask", "done", "bbc", "env_done"):
        assert np.array_equal(_np(getattr(b, f)), getattr(co, f)), where + " " + f
    assert np.array_equal(_np(b.radar), co.radar), where + " radar (fp32 bit-exact)"
    for f in ("own", "nei", "reward"):
        np.testing.assert_allclose(_np(getattr(b, f)), getattr(co, f), rtol=0, atol=ATOL, err_msg=where + " " + f)


def _both_ways(seen):
    for f, outs in seen.items():
        if f not in ("kat",) and f not in T.RADAR_FAMILIES:
            assert outs == {True, False}, (f, outs)


@pytest.mark.parametrize("variant,mode", VARIANTS)
@pytest.mark.parametrize("N", [3, 5, 8])
def test_step_kernel_on_thresholds(native_lib, N, variant, mode):
    fam, var, st, occ = T.build(N, seed=N)
    E = len(fam)
    env = _env(E, N, occ, mode, variant)
    co = c_oracle.BatchedOracle(E, N, occ, W=32, radar_mode=mode, variant=variant)
    _install(env, st)
    T.oracle_state(co, st)
    act = np.zeros((E, N, 2), np.float32)
    env.step(torch.from_numpy(act).cuda())
    co.step(act)
    torch.cuda.synchronize()
    where = f"step N{N} {variant} mode{mode}"
    _cmp_oracle(env.bufs, co, where)
    s = env.get_state()
    post = {k: _np(s[k]) for k in ("pos", "pre_pos", "goal", "wp")}
    assert np.array_equal(post["pos"], co.pos)
    seen = T.check(fam, var, post, occ, mode, _np(env.bufs.mask), _np(env.bufs.radar), where)
    _both_ways(seen)
    kat = [e for e, f in enumerate(fam) if f == "kat"]            # ATT/geometry_test.py:13-15
    assert [bool(_np(env.bufs.mask)[e, 0] & 4) for e in kat] == [True, False]
    most, cap = env.band_max()          # the radar rays flagged for the exact fix-up all fit its list
    assert (mode == 1 or most > 0) and most <= cap, (most, cap)


@pytest.mark.parametrize("variant,mode", [("att", 0), ("att", 2), ("wgru", 1)])
def test_step_tail_on_thresholds(native_lib, variant, mode):
    """The fused step tail (the bench's launch): the threshold outcomes, and the ring rows' next-radar
    column carries the exactly-decided radar too (WGRU: and the reward column the exact radar minimum's
    near-building penalty)."""
    from multi_agent_aac_amd.memory import DeviceReplay
    N = 5
    fam, var, st, occ = T.build(N, seed=11)
    E = len(fam)
    env = _env(E, N, occ, mode, variant)
    rep = DeviceReplay(2 * E, N, env.D0, seed=0)
    c, n = env.alloc_buffers(), env.alloc_buffers()
    _install(env, st)
    co = c_oracle.BatchedOracle(E, N, occ, W=32, radar_mode=mode, variant=variant)
    T.oracle_state(co, st)
    act = np.zeros((E, N, 2), np.float32)
    a_dev = torch.from_numpy(act).cuda()
    srcs = [c.own, c.radar, c.nei, a_dev, n.reward, n.done, n.own, n.radar, n.nei]
    pos0 = rep.pos
    env.step_tail(a_dev, out=n, replay=rep, srcs=srcs, auto_reset=False)
    co.step(act)
    torch.cuda.synchronize()
    where = f"tail {variant} mode{mode}"
    _cmp_oracle(n, co, where)
    s = env.get_state()
    post = {k: _np(s[k]) for k in ("pos", "pre_pos", "goal", "wp")}
    seen = T.check(fam, var, post, occ, mode, _np(n.mask), _np(n.radar), where)
    _both_ways(seen)
    off = np.cumsum([0] + list(rep.widths))
    k = list(rep.fields).index("n_radar")
    ring = _np(rep.ring[pos0:pos0 + E])
    assert np.array_equal(ring[:, off[k]:off[k + 1]], co.radar.reshape(E, -1)), where + " ring n_radar"
    k = list(rep.fields).index("rew")
    np.testing.assert_allclose(ring[:, off[k]:off[k + 1]], co.reward, rtol=0, atol=ATOL, err_msg=where + " ring reward")
    if variant == "wgru":       # agents with a flagged ray had their reward recomputed after the launch
        most, cap = env.band_max()
        assert 0 < most <= cap


@pytest.mark.parametrize("N", [3, 5])
def test_near_band_ends_observable(native_lib, N):
    """The near-drone band's 2.5 / 10 m ends (ATT/env:2420-2432), each on the threshold and +-1-2 ulp,
    with a second neighbour at 6 m so the in-band term m * shortest + c is non-zero:
    the kernel's subject reward (team reward off) equals the reference's reward computed from
    np.linalg.norm distances, the threshold neighbour included exactly when 2.5 <= d <= 10 -- and both
    outcomes occur at both ends."""
    fam, var, st, occ = T.build_near(N)
    E = len(fam)
    env = _env(E, N, occ, 0, team_reward=False)
    co = c_oracle.BatchedOracle(E, N, occ, W=32, radar_mode=0, team_reward=False)
    _install(env, st)
    T.oracle_state(co, st)
    act = np.zeros((E, N, 2), np.float32)
    env.step(torch.from_numpy(act).cuda())
    co.step(act)
    torch.cuda.synchronize()
    _cmp_oracle(env.bufs, co, f"near N{N}")
    rew = _np(env.bufs.reward)[:, 0]
    seen = {}
    for e, f in enumerate(fam):
        pos = st["pos"][e]
        d = T.float_norm(pos[0], pos[1])
        inside = 2.5 <= d <= 10.0
        want = np.float32(T.near_reward(pos))
        assert rew[e] == want, (f, var[e], d, rew[e], want)
        # the two outcomes differ by one penalty term (>= 0.5): the reward decides which one the kernel took
        other = np.float32(T.near_reward(pos) + (1 if inside else -1) * ((-1 / 7.5) * min(d, 6.0) + 4 / 3))
        assert abs(float(rew[e]) - float(want)) < abs(float(rew[e]) - float(other))
        seen.setdefault(f, set()).add(inside)
    assert seen == {"near10": {True, False}, "near2.5": {True, False}}, seen


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_reset_radar_on_thresholds(native_lib, mode):
    """The reset kernel's radar (aac_env_reset: its own radar phase and exact fix) from the threshold
    positions as episode starts: every radar family's subject row against the exact radar."""
    N = 3
    fam, var, st, occ = T.build(N, seed=3)
    E = len(fam)
    env = _env(E, N, occ, mode)
    co = c_oracle.BatchedOracle(E, N, occ, W=32, radar_mode=mode)
    env.reset(st["pos"], st["wp"], st["cnt"])
    co.reset(st["pos"], st["wp"], st["cnt"])
    torch.cuda.synchronize()
    assert np.array_equal(_np(env.bufs.radar), co.radar), f"reset mode{mode} radar"
    radar = _np(env.bufs.radar)
    checked = 0
    for e, f in enumerate(fam):
        if f in T.RADAR_FAMILIES:
            ex = T.exact_radar(tuple(st["pos"][e, 0]), [tuple(x) for x in st["pos"][e, 1:]], occ, mode)
            np.testing.assert_allclose(radar[e, 0], ex, rtol=0, atol=ATOL, err_msg=f"reset mode{mode} {f} env {e}")
            checked += 1
    assert checked > 100
