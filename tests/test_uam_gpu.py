"""GPU parity of the UAM environment (include/aac_uam.h)
against the reference-shaped scalar restatement oracle/uam_ref.py.

Bar: integer masks / done / bbc / env_done bit-exact; float64 observations, radar and rewards within
1e-9 (the radar's intersection points are computed by different formulas on the two sides); state
within 1e-12.  Every step is checked from an identical injected pre-step state (``env_from_state``),
so libm (ocml vs glibc atan2 / cos / sin) cannot accumulate drift."""
import random

import numpy as np
import pytest
import torch

from oracle import uam_ref as U

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-9


def _episodes(E, N, seed):
    py, npr = random.Random(seed), np.random.RandomState(seed)
    st, go, cl = [], [], []
    for _ in range(E):
        s, g, c0, c1 = U.sample_episode(N, py, npr)
        st.append(s)
        go.append(g)
        cl.append((c0, c1))
    return np.array(st), np.array(go), np.array(cl, dtype=np.int32)


def _np_state(env):
    return {k: v.cpu().numpy() for k, v in env.get_state().items()}


def _check_obs(b, e, obs, nei6=True, tdcpa=None):
    own, p2, rad, p3 = obs
    N = own.shape[0]
    np.testing.assert_allclose(b.own[e].cpu().numpy(), own, rtol=0, atol=TOL)
    np.testing.assert_allclose(b.radar[e].cpu().numpy(), rad, rtol=0, atol=TOL)
    np.testing.assert_allclose(b.nei[e].cpu().numpy().reshape(N, -1), p2, rtol=0, atol=TOL)
    if nei6:
        np.testing.assert_allclose(b.nei6[e].cpu().numpy(), p3, rtol=0, atol=TOL)
    if tdcpa is not None:
        check_tdcpa(b, e, tdcpa)


def check_tdcpa(b, e, tdcpa, err=""):
    """The live tdCPA outputs (UAM/util:916-938 at UAM/env:1738-1745, :4001-4010) against the
    oracle's ``tdcpa_out``: tcpa / dcpa in the sorted neighbour order within 1e-9, the two
    potential-conflict counts bit-exact."""
    tc, dc, cc, cp = tdcpa
    np.testing.assert_allclose(b.tcpa[e].cpu().numpy(), tc, rtol=0, atol=TOL, err_msg=err + " tcpa")
    np.testing.assert_allclose(b.dcpa[e].cpu().numpy(), dc, rtol=0, atol=TOL, err_msg=err + " dcpa")
    assert np.array_equal(b.conf_cur[e].cpu().numpy(), cc), (err, b.conf_cur[e].cpu().numpy(), cc)
    assert np.array_equal(b.conf_pre[e].cpu().numpy(), cp), (err, b.conf_pre[e].cpu().numpy(), cp)


@pytest.mark.parametrize("N", [16, 5])
def test_uam_reset_matches_oracle(native_lib, N):
    from multi_agent_aac_amd import uam
    E = 6
    st, go, cl = _episodes(E, N, 100 + N)
    env = uam.BatchedUAM(E, N, p3=True, tdcpa=True)
    env.reset(st, go, cl)
    torch.cuda.synchronize()
    s = _np_state(env)
    for e in range(E):
        o = U.UAMEnv(N)
        obs = o.reset(st[e], go[e], cl[e, 0], cl[e, 1])
        _check_obs(env.bufs, e, obs, tdcpa=o.tdcpa_out)
        ref = U.state_of(o)
        for k in ("pos", "vel", "pre_pos", "pre_vel", "goal", "start", "clouds"):
            np.testing.assert_array_equal(s[k][e], ref[k], err_msg=k)
        # atan2: ocml vs glibc may differ in the last bit
        np.testing.assert_allclose(s["heading"][e], ref["heading"], rtol=0, atol=1e-15)
        assert np.array_equal(s["top2"][e], ref["top2"])
        assert s["cloud_tgt"][e] == 1 and s["step"][e] == 0


def _stepped_pair(N, E, seed, steps, act_scale=1.0):
    """Run the device free; after each step check every env against the oracle started from the
    device's own pre-step state.  Returns the per-step mask arrays."""
    from multi_agent_aac_amd import uam
    st, go, cl = _episodes(E, N, seed)
    env = uam.BatchedUAM(E, N, p3=True, tdcpa=True)
    env.reset(st, go, cl)
    rng = np.random.default_rng(seed)
    masks = []
    conf = [0, 0]          # potential conflicts counted, zero-relative-velocity pairs seen
    for k in range(steps):
        pre = _np_state(env)
        act = rng.uniform(-act_scale, act_scale, (E, N, 2))
        env.step(torch.from_numpy(act).to(DEV))
        torch.cuda.synchronize()
        b = env.bufs
        post = _np_state(env)
        for e in range(E):
            o = U.env_from_state(pre, e, N)
            obs, r, d, cg, bbc, mk, over = o.full_step(act[e])
            _check_obs(b, e, obs, tdcpa=o.tdcpa_out)
            conf[0] += int(o.tdcpa_out[2].sum())
            conf[1] += int((o.tdcpa_out[0] == -10).sum())
            np.testing.assert_allclose(b.reward[e].cpu().numpy(), r, rtol=0, atol=TOL)
            assert np.array_equal(b.mask[e].cpu().numpy(), mk), (k, e, b.mask[e].cpu().numpy(), mk)
            assert np.array_equal(b.done[e].cpu().numpy().astype(bool), d)
            assert np.array_equal(b.bbc[e].cpu().numpy().astype(bool), bbc)
            assert bool(b.env_done[e].item()) == bool(over)
            ref = U.state_of(o)
            for key in ("pos", "vel", "pre_pos", "pre_vel", "heading", "clouds"):
                np.testing.assert_allclose(post[key][e], ref[key], rtol=0, atol=1e-12, err_msg=key)
            assert np.array_equal(post["reach"][e], ref["reach"])
            assert np.array_equal(post["top2"][e], ref["top2"])
            assert post["cloud_tgt"][e] == ref["cloud_tgt"] and post["step"][e] == ref["step"]
        masks.append(b.mask.cpu().numpy().copy())
    return masks, conf


def test_uam_step_matches_oracle_n16(native_lib):
    masks, conf = _stepped_pair(16, 4, 7, 6)
    assert sum(int((m & 2).any()) for m in masks) > 0      # runway / cloud conflicts happen
    assert conf[0] > 0                                     # potential tdCPA conflicts were compared


def test_uam_step_matches_oracle_n3_long(native_lib):
    # few aircraft, small actions: long episodes reach goals, move the go-around aircraft along
    # its loop and exercise the near-drone band
    _stepped_pair(3, 8, 11, 25, act_scale=0.6)


@pytest.mark.parametrize("N", [16, 4])
def test_uam_tdcpa_branches(native_lib, N):
    """tdCPA (UAM/util:916-938) on injected states built to hit every branch: pairs flying with
    equal velocities (zero relative velocity: tcpa = -10, conflict when the one-unit look-ahead is
    inside the two bounds), head-on pairs closing inside one time unit (tcpa in [0, 1], d < 1) and
    diverging pairs (tcpa < 0).  Current and ``pre_*`` counts both compared bit-exact."""
    from multi_agent_aac_amd import uam
    E = 8
    st, go, cl = _episodes(E, N, 300 + N)
    env = uam.BatchedUAM(E, N, p3=True, tdcpa=True)
    env.reset(st, go, cl)
    s = _np_state(env)
    rng = np.random.default_rng(N)
    pos, vel = s["pos"].copy(), s["vel"].copy()
    for e in range(E):
        for i in range(0, N - 1, 2):
            c = np.array([12.0 + 2.5 * (i % 6), 8.0 + 4.0 * (i // 6)]) + rng.uniform(-0.2, 0.2, 2)
            kind = (e + i // 2) % 3
            if kind == 0:        # same velocity, 0.6 apart: zero relative velocity, conflict
                v = rng.uniform(-0.3, 0.3, 2)
                pos[e, i], pos[e, i + 1] = c, c + [0.6, 0.0]
                vel[e, i] = vel[e, i + 1] = v
            elif kind == 1:      # head-on, closing: tcpa in [0, 1], d < 1
                pos[e, i], pos[e, i + 1] = c, c + [0.9, 0.05]
                vel[e, i], vel[e, i + 1] = [0.4, 0.0], [-0.4, 0.0]
            else:                # diverging: tcpa < 0
                pos[e, i], pos[e, i + 1] = c, c + [0.9, 0.0]
                vel[e, i], vel[e, i + 1] = [-0.4, 0.0], [0.4, 0.0]
    env.set_state(pos=pos, vel=vel, pre_pos=pos, pre_vel=vel)
    pre = _np_state(env)
    act = np.zeros((E, N, 2))
    env.step(torch.from_numpy(act).to(DEV))
    torch.cuda.synchronize()
    b = env.bufs
    seen_zero = seen_conf = seen_neg = 0
    for e in range(E):
        o = U.env_from_state(pre, e, N)
        obs, *_ = o.full_step(act[e])
        _check_obs(b, e, obs, tdcpa=o.tdcpa_out)
        tc = o.tdcpa_out[0]
        seen_zero += int((tc == -10).sum())
        seen_neg += int(((tc < 0) & (tc != -10)).sum())
        seen_conf += int(o.tdcpa_out[2].sum() + o.tdcpa_out[3].sum())
    assert seen_zero > 0 and seen_conf > 0 and seen_neg > 0, (seen_zero, seen_conf, seen_neg)


def test_uam_event_coverage(native_lib):
    """Every mask bit (and the order-dependent coefficient doubling) at E = 2048 with auto-reset;
    the envs where a rare event fired are re-checked against the oracle from their pre-step state."""
    from multi_agent_aac_amd import uam
    E, N = 2048, 8
    env = uam.BatchedUAM(E, N)
    env.set_bank(uam.build_bank(4096, N, seed=3), seed=5)
    env.auto_reset()
    rng = np.random.default_rng(0)
    seen = 0
    checked = 0
    for k in range(60):
        pre = _np_state(env)
        # steer towards the goal with noise: goal reaches and crowded approaches both happen
        d = pre["goal"] - pre["pos"]
        act = np.clip(d / np.maximum(np.linalg.norm(d, axis=-1, keepdims=True), 1e-9) + rng.normal(0, 0.7, d.shape),
                      -1, 1)
        # every 4th env flies straight away from the runway: bound crashes
        out = np.where(pre["start"][..., :1] < 20, -1.0, 1.0)
        act[::4] = np.concatenate([out, np.zeros_like(out)], -1)[::4]
        env.step(torch.from_numpy(act).to(DEV))
        torch.cuda.synchronize()
        b = env.bufs
        mk = b.mask.cpu().numpy()
        seen |= int(np.bitwise_or.reduce(mk.reshape(-1)))
        rare = np.where(((mk & (4 | 16 | 32)) != 0).any(axis=1))[0][:3]
        for e in rare:
            o = U.env_from_state(pre, e, N)
            obs, r, dn, cg, bbc, m2, over = o.full_step(act[e])
            assert np.array_equal(mk[e], m2)
            np.testing.assert_allclose(b.reward[e].cpu().numpy(), r, rtol=0, atol=TOL)
            assert np.array_equal(b.bbc[e].cpu().numpy().astype(bool), bbc)
            checked += 1
        env.auto_reset(b.env_done)
    assert seen & 0x1f == 0x1f, bin(seen)
    assert checked > 0


def test_uam_facade_loop(native_lib):
    """The reference method surface (reset_world_change_skin / step / ss_reward_Mar_changeskin)
    drives an E = 1 loop like UAM/main:367-637; rewards follow the oracle's free-running loop."""
    from multi_agent_aac_amd import uam
    N = 5
    st, go, cl = _episodes(1, N, 21)
    env = uam.env_simulator(seed=1)
    env.create_world(N, 2, 0.95, 0.01, 1, 0.5, 0.15, 0.5, None, 1, [-0.5, 0.5])
    state, norm = env.reset_world_change_skin(N, starts=st[0], goals=go[0], clouds=cl[0])
    o = U.UAMEnv(N)
    ref = o.reset(st[0], go[0], cl[0, 0], cl[0, 1])
    np.testing.assert_allclose(np.stack(norm[0]), ref[0], atol=TOL)
    assert len(norm) == 4 and np.stack(norm[1]).shape == (N, 5 * (N - 1))
    rng = np.random.default_rng(2)
    for step in range(1, 30):
        act = rng.uniform(-0.5, 0.5, (N, 2))
        env.step(act, step, 0.5)
        r, d, cg, _, _, _, bbc = env.ss_reward_Mar_changeskin(step, [None] * N, [[] for _ in range(N)])
        _, r2, d2, cg2, bbc2, _, over = o.full_step(act)
        np.testing.assert_allclose(np.array(r, dtype=float), r2, atol=1e-7)
        assert list(d) == list(d2) and list(cg) == list(cg2) and bbc == list(bbc2)
        for i, ag in env.all_agents.items():
            np.testing.assert_allclose(ag.pos, o.all_agents[i].pos, atol=1e-9)
        if env.episode_over(step):
            assert over
            break


@pytest.mark.parametrize("r", [0.5, 1.0, 3.0])      # aircraft pB, go-around aircraft, cloud
def test_ray_gon_fast_paths_exact(native_lib, r):
    """The radar's ray-vs-64-gon fast paths (exact pre-filter, entry window, inside-polygon exit
    window) against the full 64-edge clip on 4M random segments around the polygon: the same hit
    flag and the same t to the last bit (aac_uam_ray_gon_check)."""
    import ctypes
    from multi_agent_aac_amd import uam
    L = uam.lib()
    L.aac_uam_ray_gon_check.argtypes = [ctypes.c_int64, ctypes.c_uint64, ctypes.c_double, ctypes.c_double,
                                        ctypes.POINTER(ctypes.c_uint64)]
    for ln in (U.RADAR_DIST, 0.7 * r):
        bad = ctypes.c_uint64(99)
        assert L.aac_uam_ray_gon_check(4_000_000, 11, r, float(ln), ctypes.byref(bad)) == 0
        assert bad.value == 0, (r, ln, bad.value)


@pytest.mark.parametrize("N,E", [(16, 1003), (5, 9001)])     # 9001: more than one 8192-env packing tile
def test_uam_compact_reset_bit_exact(native_lib, N, E):
    """The auto-reset over the compacted list of done envs (default) is bit-identical to the reset
    over contiguous env ranges: two envs from the same bank and actions, one per mode, compared on
    every output and state tensor after each step + auto-reset (E not a multiple of epb: ragged tail)."""
    from multi_agent_aac_amd import uam
    bank = uam.build_bank(2048, N, seed=9)
    envs = []
    for _ in range(2):
        env = uam.BatchedUAM(E, N, neighbours=True)
        env.set_bank(bank, seed=77)
        envs.append(env)
    rng = np.random.default_rng(4)
    lib = uam.lib()
    resets = 0
    try:
        for mode, env in zip((1, 0), envs):
            lib.aac_uam_set_reset_compact(mode)
            env.auto_reset()
        for k in range(12):
            act = torch.from_numpy(rng.uniform(-1, 1, (E, N, 2))).to(DEV)
            for mode, env in zip((1, 0), envs):
                lib.aac_uam_set_reset_compact(mode)
                env.step(act)
                env.auto_reset(env.bufs.env_done)
            torch.cuda.synchronize()
            resets += int(envs[0].bufs.env_done.sum())
            a, b = envs
            for name in a.bufs.__dict__:
                x, y = getattr(a.bufs, name), getattr(b.bufs, name)
                if isinstance(x, torch.Tensor):
                    assert torch.equal(x, y), (k, name)
            sa, sb = a.get_state(), b.get_state()
            for key in sa:
                assert torch.equal(sa[key], sb[key]), (k, key)
    finally:
        lib.aac_uam_set_reset_compact(1)
    assert resets > 0


def test_uam_episode_buffer_counts_resets(native_lib):
    from multi_agent_aac_amd import uam
    E, N = 257, 8
    env = uam.BatchedUAM(E, N)
    env.set_bank(uam.build_bank(1024, N, seed=2), seed=3)
    ep = env.use_episode_buffer(torch.zeros(E, dtype=torch.int32, device=DEV))
    env.auto_reset()
    want = torch.ones(E, dtype=torch.int32, device=DEV)
    rng = np.random.default_rng(5)
    for _ in range(10):
        env.step(torch.from_numpy(rng.uniform(-1, 1, (E, N, 2))).to(DEV))
        want += env.bufs.env_done.to(torch.int32)
        env.auto_reset(env.bufs.env_done)
    torch.cuda.synchronize()
    assert torch.equal(ep, want) and int(want.max()) > 1
