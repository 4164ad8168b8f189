"""The benchmarked env path -- ``aac_env_step_tail``: env step + ss_reward + termination, the replay
push of the E transitions and the OD-bank auto-reset of the finished envs in one launch -- against
the C oracle at the BASELINE config sizes (config 3: 4096 envs x 5 agents, combined radar; config 4:
4096 x 8, the randomOD_Wgru_radar env with hidden rows), with the grid the bench launches.

Every step:
  * the oracle steps from the GPU's pre-step state (injected: removes the ocml / glibc libm ulp
    drift of free-running trajectories) with the same actions;
  * reward / obs / radar / nei within 1e-5, masks / done / bbc / env_done bit-exact;
  * every ring row written this step equals the oracle's transition (s, a, r, d, s') of
    ATT/main:363-400: s = the oracle's observation rows of the previous step (after its resets),
    s' = the oracle's step outputs *before* the reset (the terminal rows of finished envs);
  * the finished envs are reset on the oracle side with the bank-draw rule (``bank_draw_batch``,
    the start-separation redraw of ATT/env:251-268 over the seeded OD bank) and the env state of
    every env (positions, waypoints, counters) and the reset observation rows must match.
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from tests.helpers import bank_draw_batch, steer, wgru_targets
from tests.test_env_gpu import ATOL, _state_to_oracle

pytestmark = pytest.mark.gpu

W = 32


def _np(t):
    return t.cpu().numpy()


def _att_targets(co):
    k = np.clip(co.wp_cur, 0, W - 1)
    return np.take_along_axis(co.wp, k[..., None, None].repeat(2, -1), 2)[:, :, 0]


@pytest.mark.parametrize("variant,N,E,radar,steps", [
    ("att", 5, 4096, "combined", 24),       # config 3 (bench default)
    ("wgru", 8, 4096, None, 20),            # config 4 env (bench --model gru)
])
def test_step_tail_vs_oracle_config_size(native_lib, occ, variant, N, E, radar, steps):
    from multi_agent_aac_amd import world
    from multi_agent_aac_amd.env import BatchedEnv
    from multi_agent_aac_amd.memory import DeviceReplay
    seed = 1234
    bank = world.ODBank(occ, n_pairs=65536, seed=2026, max_wp=W)           # as the bench's Trainer
    env = BatchedEnv(E, N, occ, radar_mode=radar, max_wp=W, variant=variant)
    env.set_od_bank(bank, seed=seed)
    episode = env.use_episode_buffer(torch.zeros(E, dtype=torch.int32, device="cuda"))
    H = 64 if variant == "wgru" else 0
    cap = int(2.5 * E)                        # the ring wraps on the third push
    rep = DeviceReplay(cap, N, env.D0, hidden=H, seed=0)
    bufs = [env.alloc_buffers(), env.alloc_buffers()]
    env.auto_reset(None, out=bufs[0])         # every env: episode 1 draw + first observation
    mode = {"drones": 0, "obstacles": 1, "combined": 2}[radar or "obstacles"]
    co = c_oracle.BatchedOracle(E, N, occ, W=W, radar_mode=mode, variant=variant)

    def oracle_reset(envs):
        ep = _np(episode)[envs]
        idx = bank_draw_batch(bank.start, bank.n_pairs, seed, envs, ep, N)
        st = np.zeros((E, N, 2)); wps = np.zeros((E, N, W, 2)); cnt = np.ones((E, N), np.int32)
        st[envs] = bank.start[idx]; wps[envs] = bank.wps[idx]; cnt[envs] = bank.cnt[idx]
        m = np.zeros(E, np.uint8)
        m[envs] = 1
        co.reset(st, wps, cnt, env_mask=m)

    torch.cuda.synchronize()
    assert (_np(episode) == 1).all()
    oracle_reset(np.arange(E))
    for f in ("own", "radar", "nei"):
        np.testing.assert_allclose(_np(getattr(bufs[0], f)), getattr(co, f), rtol=0, atol=ATOL, err_msg="reset " + f)
    g = torch.Generator(device="cuda").manual_seed(5)
    hid = [torch.rand(E, N, H, device="cuda", generator=g) if H else None for _ in range(2)]
    rng = np.random.default_rng(17)
    resets, seen = 0, 0
    off = [rep.widths[0]]
    for wdt in rep.widths[1:]:
        off.append(off[-1] + wdt)
    sl = {f: slice(o - wdt, o) for f, o, wdt in zip(rep.fields, off, rep.widths)}
    for t in range(steps):
        k = t % 2
        c, n = bufs[k], bufs[1 - k]
        _state_to_oracle(env, co)
        s_prev = {f: getattr(co, f).copy() for f in ("own", "radar", "nei")}
        # half the agents steer toward their current waypoint (goal / waypoint events), half fly at random
        tg = wgru_targets(co.wp, co.wp_cur, co.wp_cnt) if variant == "wgru" else _att_targets(co)
        act = steer(co.pos, co.vel, tg, rng)
        act[:, ::2] = rng.uniform(-1, 1, size=act[:, ::2].shape).astype(np.float32)
        a_dev = torch.from_numpy(act).cuda()
        srcs = [c.own, c.radar, c.nei, a_dev, n.reward, n.done, n.own, n.radar, n.nei]
        if H:
            srcs += [hid[k], hid[1 - k]]
        h_next_before = hid[1 - k].clone() if H else None
        pos0 = rep.pos
        env.step_tail(a_dev, out=n, replay=rep, srcs=srcs, zero_rows=hid[1 - k] if H else None)
        co.step(act)
        torch.cuda.synchronize()
        where = f"{variant} t{t}"
        np.testing.assert_allclose(_np(n.reward), co.reward, rtol=0, atol=ATOL, err_msg=where + " reward")
        for f in ("mask", "done", "bbc", "env_done"):
            assert np.array_equal(_np(getattr(n, f)), getattr(co, f)), where + " " + f
        seen |= int(np.bitwise_or.reduce(co.mask.ravel()))
        done = co.env_done.astype(bool)
        # the transition rows of this step (ring rows pos0 .. pos0 + E - 1, wrapping)
        rows = (pos0 + np.arange(E)) % cap
        ring = _np(rep.ring[torch.from_numpy(rows).cuda()])
        exp = {"s_own": s_prev["own"], "s_radar": s_prev["radar"], "s_nei": s_prev["nei"], "act": act,
               "rew": co.reward, "done": co.done.astype(np.float32), "n_own": co.own, "n_radar": co.radar,
               "n_nei": co.nei}
        for f, v in exp.items():
            np.testing.assert_allclose(ring[:, sl[f]], v.reshape(E, -1), rtol=0, atol=ATOL, err_msg=where + " ring " + f)
        assert np.array_equal(ring[:, sl["act"]], act.reshape(E, -1)), where + " ring act"
        assert np.array_equal(ring[:, sl["done"]], co.done.reshape(E, -1).astype(np.float32)), where + " ring done"
        if H:
            assert np.array_equal(ring[:, sl["h_cur"]], _np(hid[k]).reshape(E, -1)), where + " ring h_cur"
            assert np.array_equal(ring[:, sl["h_next"]], _np(h_next_before).reshape(E, -1)), where + " ring h_next"
            hn = _np(hid[1 - k])
            assert (hn[done] == 0).all() and np.array_equal(hn[~done], _np(h_next_before)[~done]), where + " zeroed"
        assert (rep.pos, rep.size) == ((pos0 + E) % cap, min((t + 1) * E, cap))
        assert np.array_equal(_np(rep.meta), [rep.pos, rep.size]), where + " meta"
        # the auto-reset of the finished envs: the oracle's bank draw with each env's new episode number
        envs = np.nonzero(done)[0]
        resets += len(envs)
        if len(envs):
            oracle_reset(envs)
        for f in ("own", "radar", "nei"):
            np.testing.assert_allclose(_np(getattr(n, f)), getattr(co, f), rtol=0, atol=ATOL, err_msg=where + " " + f)
        s = env.get_state()
        for key, ref in (("pos", co.pos), ("vel", co.vel), ("pre_pos", co.pre_pos), ("goal", co.goal),
                         ("start", co.start)):
            np.testing.assert_allclose(_np(s[key]), ref, rtol=0, atol=1e-12, err_msg=where + " " + key)
        assert np.array_equal(_np(s["wp"])[done], co.wp[done]), where + " reset waypoints"
        for key, ref in (("wp_cur", co.wp_cur), ("wp_cnt", co.wp_cnt), ("reach", co.reach), ("wall", co.wall),
                         ("step", co.step_count)):
            assert np.array_equal(_np(s[key]), ref), where + " " + key
        assert np.array_equal(np.asarray(_np(s["pos"])[done]), co.pos[done])       # reset starts bit-exact
    assert resets > E // 4, resets           # the in-launch reset ran on many envs
    want = 0b11 if variant == "att" else 0b1     # bound (+ drone) crashes occurred
    assert seen & want == want, bin(seen)
