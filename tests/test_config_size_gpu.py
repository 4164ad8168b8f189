"""Parity at the BASELINE.json config sizes (the shapes bench.py runs), against the oracles.

config 3  one_model_att 5 x 4096, B = 1024: the fused update_myown vs oracle/learner_ref.py over two
          updates (ATT/maddpg:219-440), and the captured graph vs eager at B = 1024
config 4  randomOD_gru_radar 8 x 4096, B = 512: the env step at E = 4096 x N = 8 vs the C oracle, and
          the GRU update vs oracle/gru_ref.py (WGRU/maddpg:211-326)
config 5  UAM 16 x 8192, B = 512: the env step at E = 8192 x N = 16 (a seeded subset of 256 envs per
          step, each from the device's own pre-step state) vs oracle/uam_ref.py (UAM/env:3892-4629),
          and the fused float64 learner vs oracle/uam_learner_ref.py
"""
import concurrent.futures as cf
import multiprocessing as mp

import numpy as np
import pytest
import torch

from oracle import c_oracle, gru_ref, learner_ref
from oracle import uam_learner_ref as UR
from tests.helpers import W_DEFAULT, uam_oracle_steps

pytestmark = pytest.mark.gpu
DEV = "cuda"
ATOL = 1e-5


# --------------------------------------------------------------------------- config 3
@pytest.mark.parametrize("eps,param_tol", [(1e-8, 4e-3), (1e-3, 1e-5)])
def test_update_b1024_matches_cpu_restatement(native_lib, eps, param_tol):
    """N = 5, B = 1024 (config 3), two update_myown calls on identical weights and sampled rows
    against the torch-CPU restatement: Q, targets and losses of every iteration within 1e-5
    (rtol 1e-5).  Parameter bound after the two updates (10 Adam steps per network):
      eps = 1e-8 (the reference's Adam): 4e-3.  Where a weight's gradient is fp32 rounding noise
        (a ReLU unit active on a handful of the 5 120 actor rows) Adam moves it by +-lr = 1e-3 per
        step whichever the sign, so summation order alone can separate the two sides by 2 lr/step;
      eps = 1e-3 on both sides: 1e-5.  Adam's step is then ~lr g / eps for such weights, so the
        parameters compare the gradients themselves."""
    from multi_agent_aac_amd.maddpg import MADDPG
    assert learner_ref.check_one_update(MADDPG, device=DEV, N=5, B=1024, E=512, tol=1e-5, iters=2, seed=3, eps=eps,
                                        param_tol=param_tol)


def test_graph_replay_equals_eager_b1024(native_lib):
    """The captured HIP graph at B = 1024 (the GEMM planner's one-tile-per-wave mode for the large
    products) is bit-equal to the eager launch list."""
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B, E = 5, 1024, 1024
    ms = []
    for _ in range(2):
        m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=N, device=DEV, seed=11, batch_size=B)
        rep = m.attach_replay(4 * E, seed=5)
        for p in range(3):
            tr = learner_ref.random_transitions(E, N, 40 + p)
            rep.push_batch(*[tr[k].to(DEV).contiguous() for k in ("s_own", "s_radar", "s_nei", "act", "rew", "done",
                                                                   "n_own", "n_radar", "n_nei")])
        ms.append(m)
    for _ in range(3):
        ms[0].update(B, use_graph=True, want_stats=False)
        ms[1].update(B, use_graph=False, want_stats=False)
    torch.cuda.synchronize()
    for a, b in ((ms[0].fa.data, ms[1].fa.data), (ms[0].fc.data, ms[1].fc.data), (ms[0].fa_t.data, ms[1].fa_t.data),
                 (ms[0].fc_t.data, ms[1].fc_t.data)):
        assert torch.equal(a, b)


# --------------------------------------------------------------------------- config 4
def _state_to_oracle(env, co):
    s = {k: v.cpu().numpy() for k, v in env.get_state().items()}
    co.pos[:] = s["pos"]; co.vel[:] = s["vel"]; co.pre_pos[:] = s["pre_pos"]; co.pre_vel[:] = s["pre_vel"]
    co.goal[:] = s["goal"]; co.wp[:] = s["wp"]; co.wp_cur[:] = s["wp_cur"]; co.wp_cnt[:] = s["wp_cnt"]
    co.reach[:] = s["reach"]; co.wall[:] = s["wall"]; co.step_count[:] = s["step"]


@pytest.mark.parametrize("E,N", [(4096, 8), (12288, 5)])
def test_env_n8_e4096_combined(native_lib, occ, E, N):
    """Config 4's env shape: E = 4096, N = 8, combined radar, 10 steps from identical injected state
    with OD-bank auto-reset: masks / done / bbc / env_done bit-exact, obs / radar / reward 1e-5,
    positions 1e-12.  E = 12288, N = 5: a grid large enough for the 50-agent workgroups (10 envs
    per workgroup, aac_env.hip's epb choice) of the step and reset kernels."""
    from multi_agent_aac_amd import world
    from multi_agent_aac_amd.env import BatchedEnv
    bank = world.ODBank(occ, n_pairs=65536, seed=2026, max_wp=W_DEFAULT)
    st, wps, cnt = bank.sample_env_od(E, N, np.random.default_rng(8))
    env = BatchedEnv(E, N, occ, radar_mode="combined", max_wp=W_DEFAULT)
    co = c_oracle.BatchedOracle(E, N, occ, W=W_DEFAULT, radar_mode=2)
    env.reset(st, wps, cnt)
    co.reset(st, wps, cnt)
    rng = np.random.default_rng(88)
    seen = 0
    for t in range(10):
        _state_to_oracle(env, co)
        act = rng.uniform(-1, 1, size=(E, N, 2)).astype(np.float32)
        env.step(torch.from_numpy(act).cuda())
        co.step(act)
        torch.cuda.synchronize()
        b = env.bufs
        w = f"t{t}"
        for name in ("own", "radar", "nei", "reward"):
            np.testing.assert_allclose(getattr(b, name).cpu().numpy(), getattr(co, name), rtol=0, atol=ATOL,
                                       err_msg=w + name)
        for name in ("mask", "done", "bbc", "env_done"):
            assert np.array_equal(getattr(b, name).cpu().numpy(), getattr(co, name)), w + name
        np.testing.assert_allclose(env.get_state()["pos"].cpu().numpy(), co.pos, rtol=1e-12, atol=1e-12)
        seen |= int(np.bitwise_or.reduce(co.mask.ravel()))
        done = co.env_done.astype(bool)
        if done.any():
            st2, wps2, cnt2 = bank.sample_env_od(E, N, np.random.default_rng(1000 + t))
            env.reset(st2, wps2, cnt2, env_mask=done.astype(np.uint8))
            co.reset(st2, wps2, cnt2, env_mask=done.astype(np.uint8))
    assert seen & 0b11 == 0b11, bin(seen)       # bound crashes and drone collisions occurred


KEYS = ("s_own", "s_radar", "s_nei", "act", "rew", "done", "n_own", "n_radar", "n_nei", "h_cur", "h_next")


def _relu_margins(critic, critic_before, actor_before, b, i, d):
    """Smallest |pre-activation| per ReLU unit (float64, over the B sampled rows) of every forward in
    agent i's update_myown iteration: the pre-update critic's encoders on [own, a] and radar, the
    pre-update actor's encoders, and the updated critic's [own, a] encoder on the policy action."""
    f = lambda lin, x: (x @ lin.weight.double().t() + lin.bias.double()).abs().min(0).values   # noqa: E731
    own, radar = b["s_own"][:, i, :d].double(), b["s_radar"][:, i].double()
    with torch.no_grad():
        a_pi = actor_before([b["s_own"][:, i, :d], b["s_radar"][:, i]], b["h_cur"][:, i])[0].double()
        return {("critic", "SA_fc"): torch.minimum(f(critic_before.SA_fc[0], torch.cat([own, b["act"][:, i].double()],
                                                                                       1)),
                                                   f(critic.SA_fc[0], torch.cat([own, a_pi], 1))),
                ("critic", "SA_grid"): f(critic_before.SA_grid[0], radar),
                ("actor", "own_fc"): f(actor_before.own_fc[0], own),
                ("actor", "own_grid"): f(actor_before.own_grid[0], radar),
                "policy_flip": float(f(critic.SA_fc[0], torch.cat([own, a_pi], 1)).min())}


def _sync_ref(m, nets, opts):
    """Copy the device parameters, targets and Adam moments into the reference nets (re-inject an
    identical state before the next iteration, as the env parity tests do per step)."""
    actors, critics, actors_t, critics_t = nets
    for flat, opt, stack, ref_nets, ref_opts in ((m.fa, m.actor_optimizer, m.actors, actors, opts[0]),
                                                  (m.fc, m.critic_optimizer, m.critics, critics, opts[1])):
        where = {p.data_ptr(): (off, k) for p, off, k in flat.slices}
        for i in range(len(ref_nets)):
            for (name, p), rp in zip(stack[i].named_parameters(), ref_nets[i].parameters()):
                off, k = where[p.data_ptr()]
                rp.data.copy_(p.detach().cpu())
                st = ref_opts[i].state[rp]
                st["exp_avg"].copy_(opt.exp_avg[off:off + k].view_as(rp).cpu())
                st["exp_avg_sq"].copy_(opt.exp_avg_sq[off:off + k].view_as(rp).cpu())
    for stack, ref_nets in ((m.actors_target, actors_t), (m.critics_target, critics_t)):
        for i in range(len(ref_nets)):
            ref_nets[i].load_state_dict({k: v.cpu() for k, v in stack[i].state_dict().items()})


def test_gru_update_n8_b512(native_lib):
    """Config 4's learner shape: 8 GRU actors / critics, B = 512, three update_myown calls against
    oracle/gru_ref.py, each from an identical injected state (device parameters, targets and Adam
    moments copied into the reference after every call).  Every call: targets / Q within 2e-5
    (relative to max(1, |.|)), losses 1e-4 relative, parameters 2e-5 (Adam eps = 1e-3 on both sides,
    as in test_gru_gpu).  The one admitted difference is a ReLU decided differently because its fp32
    pre-activation lies within rounding of 0 (|x| < 1e-5 in the float64 recompute): that unit's
    weight row and bias may differ, and the actor of an agent whose critic flips on the policy action
    (each flip is counted; at most 2 over the run)."""
    import copy
    from multi_agent_aac_amd.gru import MADDPG
    N, B, E, d = 8, 512, 256, 6
    m = MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, device=DEV, seed=8, batch_size=B)
    rep = m.attach_replay(4 * E, seed=11)
    actors = [gru_ref.RefGRUActor([6, 18, 6], 2) for _ in range(N)]
    critics = [gru_ref.RefGRUCritic([6, 18, 6], 2) for _ in range(N)]
    for i in range(N):
        actors[i].load_state_dict({k: v.cpu() for k, v in m.actors[i].state_dict().items()})
        critics[i].load_state_dict({k: v.cpu() for k, v in m.critics[i].state_dict().items()})
    actors_t, critics_t = copy.deepcopy(actors), copy.deepcopy(critics)
    host = {k: [] for k in KEYS}
    for p in range(3):
        tr = gru_ref.random_gru_transitions(E, N, 500 + p)
        rep.push_batch(*[tr[k].to(DEV).contiguous() for k in KEYS])
        for k in KEYS:
            host[k].append(tr[k])
    host = {k: torch.cat(v) for k, v in host.items()}
    gen = np.random.default_rng(17)
    eps = 1e-3
    m.actor_optimizer.eps = m.critic_optimizer.eps = eps
    opts = ([torch.optim.Adam(a.parameters(), lr=1e-3, eps=eps) for a in actors],
            [torch.optim.Adam(c.parameters(), lr=1e-3, eps=eps) for c in critics])
    flips = 0
    for it in range(3):
        idx = torch.from_numpy(gen.choice(len(rep), size=B, replace=False).astype(np.int32))
        stats = m.update(B, use_graph=False, idx=idx.to(DEV))
        b = {k: v[idx.long()].clone() for k, v in host.items()}
        b["done"] = b["done"].float()
        before, cbefore = copy.deepcopy(actors), copy.deepcopy(critics)
        rstats, opts = gru_ref.ref_gru_update(actors, critics, actors_t, critics_t, b, d, opts=opts)
        for ag, ((lq, la, q, tg), (rlq, rla, rq, rtg)) in enumerate(zip(stats, rstats)):
            dt, dqv = float((tg.cpu() - rtg).abs().max()), float((q.cpu() - rq).abs().max())
            assert dt < 2e-5 * max(1.0, float(rtg.abs().max())), ("target", it, ag, dt)
            assert dqv < 2e-5 * max(1.0, float(rq.abs().max())), ("q", it, ag, dqv)
            assert abs(float(lq) - rlq) <= 1e-4 * max(1.0, abs(rlq)), ("loss_q", it, ag, float(lq), rlq)
            assert abs(float(la) - rla) <= 1e-4 * max(1.0, abs(rla)), ("loss_a", it, ag, float(la), rla)
        for i in range(N):
            marg = _relu_margins(critics[i], cbefore[i], before[i], b, i, d)
            for tag, mine, ref in (("actor", m.actors[i], actors[i]), ("critic", m.critics[i], critics[i]),
                                   ("actor", m.actors_target[i], actors_t[i]),
                                   ("critic", m.critics_target[i], critics_t[i])):
                for (k, v), (_, rv) in zip(mine.state_dict().items(), ref.state_dict().items()):
                    diff = (v.cpu() - rv).abs()
                    if float(diff.max()) < 2e-5:
                        continue
                    if tag == "actor" and marg["policy_flip"] < 1e-5:
                        continue                   # one row of d a differs: the whole actor step does
                    unit = (tag, k.split(".")[0])
                    assert unit in marg, (it, i, tag, k, float(diff.max()))
                    rows = (diff.reshape(diff.shape[0], -1) >= 2e-5).any(1).nonzero()[:, 0]
                    assert bool((marg[unit][rows] < 1e-5).all()), (it, i, tag, k, rows.tolist(),
                                                                    marg[unit][rows].tolist())
                    flips += 1
        _sync_ref(m, (actors, critics, actors_t, critics_t), opts)
    assert flips <= 2 * 4, flips          # weight + bias, online + target, per flipped unit


# --------------------------------------------------------------------------- config 5
def test_uam_n16_e8192_subset(native_lib):
    """Config 5's env shape: E = 8192 x N = 16 with tdCPA / p3 outputs live and bank auto-reset,
    20 steps.  After each step a seeded subset of 256 envs is re-run on oracle/uam_ref.py from the
    device's own pre-step state (8 spawned CPU workers): masks / done / bbc / env_done bit-exact,
    obs / radar / reward 1e-9, state 1e-12 (the tolerances of test_uam_gpu)."""
    from multi_agent_aac_amd import uam
    E, N, S, TOL = 8192, 16, 256, 1e-9
    env = uam.BatchedUAM(E, N, p3=True, tdcpa=True)
    env.set_bank(uam.build_bank(16384, N, seed=2026), seed=1234)
    env.auto_reset()
    rng = np.random.default_rng(55)
    pick = np.random.default_rng(56)
    checked = 0
    seen = 0
    conf = 0
    with cf.ProcessPoolExecutor(8, mp_context=mp.get_context("spawn")) as pool:
        for k in range(20):
            pre = {key: v.cpu().numpy() for key, v in env.get_state().items()}
            act = rng.uniform(-1, 1, (E, N, 2))
            env.step(torch.from_numpy(act).to(DEV))
            torch.cuda.synchronize()
            b = env.bufs
            post = {key: v.cpu().numpy() for key, v in env.get_state().items()}
            out = {name: getattr(b, name).cpu().numpy() for name in ("own", "radar", "nei", "nei6", "reward", "mask",
                                                                     "done", "bbc", "env_done", "tcpa", "dcpa",
                                                                     "conf_cur", "conf_pre")}
            seen |= int(np.bitwise_or.reduce(out["mask"].reshape(-1)))
            envs = np.sort(pick.choice(E, S, replace=False))
            chunks = np.array_split(envs, 8)
            futs = [pool.submit(uam_oracle_steps, {key: v[c] for key, v in pre.items()}, act[c], N) for c in chunks]
            res = [r for f in futs for r in f.result()]
            for e, (obs, r, d, cg, bbc, mk, over, ref, td) in zip(envs, res):
                own, p2, rad, p3 = obs
                w = f"step {k} env {e}"
                np.testing.assert_allclose(out["own"][e], own, rtol=0, atol=TOL, err_msg=w)
                np.testing.assert_allclose(out["radar"][e], rad, rtol=0, atol=TOL, err_msg=w)
                np.testing.assert_allclose(out["nei"][e].reshape(N, -1), p2, rtol=0, atol=TOL, err_msg=w)
                np.testing.assert_allclose(out["nei6"][e], p3, rtol=0, atol=TOL, err_msg=w)
                np.testing.assert_allclose(out["reward"][e], r, rtol=0, atol=TOL, err_msg=w)
                assert np.array_equal(out["mask"][e], mk), w
                assert np.array_equal(out["done"][e].astype(bool), d), w
                assert np.array_equal(out["bbc"][e].astype(bool), bbc), w
                assert bool(out["env_done"][e]) == bool(over), w
                for key in ("pos", "vel", "pre_pos", "pre_vel", "heading", "clouds"):
                    np.testing.assert_allclose(post[key][e], ref[key], rtol=0, atol=1e-12, err_msg=w + key)
                assert np.array_equal(post["reach"][e], ref["reach"]) and np.array_equal(post["top2"][e], ref["top2"])
                # the live tdCPA outputs (UAM/util:916-938 at UAM/env:1738-1745 / :4001-4010)
                np.testing.assert_allclose(out["tcpa"][e], td[0], rtol=0, atol=TOL, err_msg=w + " tcpa")
                np.testing.assert_allclose(out["dcpa"][e], td[1], rtol=0, atol=TOL, err_msg=w + " dcpa")
                assert np.array_equal(out["conf_cur"][e], td[2]) and np.array_equal(out["conf_pre"][e], td[3]), w
                conf += int(td[2].sum())
                checked += 1
            env.auto_reset(b.env_done)
    assert checked == 20 * S
    assert conf > 0                             # potential tdCPA conflicts were counted and compared
    assert seen & 0b110 == 0b110, bin(seen)     # cloud / runway conflicts and drone collisions occurred


def test_uam_learner_b512(native_lib):
    """Config 5's learner shape: the fused float64 learner at B = 512, two updates on identical rows
    against oracle/uam_learner_ref.py: losses and all four networks within 1e-10."""
    from multi_agent_aac_amd import uam_learner as L
    m = L.MADDPG([7, 75, 18, 6], [7, 75, 18, 6], 2, n_agents=16, device=DEV, seed=12, batch_size=512,
                 memory_length=8192)
    rep = m.attach_replay(8192, seed=4)
    g = torch.Generator().manual_seed(12)
    E, N = 64, 16
    for _ in range(4):
        rnd = lambda *s: torch.rand(*s, generator=g, dtype=torch.float64) * 2 - 1   # noqa: E731
        rep.push_batch(rnd(E, N, 7).to(DEV), rnd(E, N, 18).abs().mul(5).to(DEV), rnd(E, N, 2).to(DEV),
                       rnd(E, N).mul(50).to(DEV), (rnd(E, N) > 0.8).double().to(DEV), rnd(E, N, 7).to(DEV),
                       rnd(E, N, 18).abs().mul(5).to(DEV))
    import copy
    a, c = UR.RefActor().double(), UR.RefCritic().double()
    a.load_state_dict({k: v.cpu() for k, v in m.actors.state_dict().items()})
    c.load_state_dict({k: v.cpu() for k, v in m.critics.state_dict().items()})
    at, ct = copy.deepcopy(a), copy.deepcopy(c)
    oa = torch.optim.Adam(a.parameters(), lr=1e-4)
    oc = torch.optim.Adam(c.parameters(), lr=1e-4)
    fu = m.fused(512, rep)
    rng = np.random.default_rng(3)
    for it in range(2):
        idx = torch.as_tensor(rng.choice(len(rep), 512, replace=False), dtype=torch.int32, device=DEV)
        lq, la = fu.run(idx)
        rows = rep.ring[idx.long()].cpu()
        b = {k: rows[:, s:e] for k, (s, e) in L.SLICES.items()}
        b["rew"], b["done"] = b["rew"][:, 0], b["done"][:, 0]
        rq, ra = UR.ref_update(a, c, at, ct, oa, oc, b)
        assert abs(float(lq) - rq) < 1e-10 * max(1.0, abs(rq)) and abs(float(la) - ra) < 1e-10 * max(1.0, abs(ra)), \
            (float(lq), rq, float(la), ra)
    for mine, ref in ((m.actors, a), (m.critics, c), (m.actors_target, at), (m.critics_target, ct)):
        for (k, p), (_, q) in zip(mine.state_dict().items(), ref.state_dict().items()):
            np.testing.assert_allclose(p.cpu().numpy(), q.numpy(), rtol=0, atol=1e-10, err_msg=k)
