"""torch-CPU fp32 restatement of the ``one_model_att`` learner (TEST INFRASTRUCTURE ONLY).

Follows, as text:
  ActorNetwork_ATT_TwoPortion   ATT/nets:177-213 (bmm scores, -inf masking, softmax over K / 8,
                                masked weights zeroed, sum of v * alpha)
  critic (canonical N-agent)    ATT/nets:672-724 pattern: separate Linear(D0+2, 128) per agent
                                index, concat in agent order, Linear(128N, 256), Linear(256, 1)
  update_myown                  ATT/maddpg:219-440 (per agent iteration: target with actors_target /
                                critics_target, MSE, critic Adam step, -Q(s, pi(s)).mean() actor Adam
                                step; then soft_update ATT/maddpg:18-22 with tau)
with canonical contract R1-R4.  The device learner is compared against this
on identical weights and identical sampled batches.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class RefActor(nn.Module):
    def __init__(self, actor_dim, n_actions):
        super().__init__()
        self.own_fc = nn.Sequential(nn.Linear(actor_dim[0], 64), nn.ReLU())
        self.own_grid = nn.Sequential(nn.Linear(actor_dim[1], 64), nn.ReLU())
        self.neigh_fc = nn.Sequential(nn.Linear(actor_dim[2], 64), nn.ReLU())
        self.merge_feature = nn.Sequential(nn.Linear(192, 256), nn.ReLU())
        self.act_out = nn.Sequential(nn.Linear(256, n_actions), nn.Tanh())
        self.k = nn.Linear(64, 64, bias=False)
        self.q = nn.Linear(64, 64, bias=False)
        self.v = nn.Linear(64, 64, bias=False)

    def forward(self, cur_state):
        own_obs = self.own_fc(cur_state[0])
        own_grid = self.own_grid(cur_state[1])
        x_e = self.neigh_fc(cur_state[2])
        q = self.q(own_obs)
        k = self.k(x_e)
        v = self.v(x_e)
        mask = cur_state[2].mean(axis=2, keepdim=True).bool()
        score = torch.bmm(k, q.unsqueeze(2))
        score_mask = score.clone()
        score_mask[~mask] = float("-inf")
        alpha = F.softmax(score_mask / np.sqrt(k.size(-1)), dim=1)
        alpha_mask = alpha.clone()
        alpha_mask[~mask] = 0
        v_att = torch.sum(v * alpha_mask, axis=1)
        merged = torch.cat((own_obs, own_grid, v_att), dim=1)
        return self.act_out(self.merge_feature(merged))


class RefCritic(nn.Module):
    def __init__(self, critic_obs, n_agents, n_actions):
        super().__init__()
        self.n_agents = n_agents
        for i in range(n_agents):
            setattr(self, f"o{i + 1}a{i + 1}", nn.Sequential(nn.Linear(critic_obs[0] + n_actions, 128), nn.ReLU()))
        self.combine_agents_fea = nn.Sequential(nn.Linear(128 * n_agents, 256), nn.ReLU())
        self.out_feature_q = nn.Sequential(nn.Linear(256, 1))

    def forward(self, combine_state, combine_action):
        feats = []
        for i in range(self.n_agents):
            obs_w_act = torch.cat((combine_state[0][:, i, :], combine_action[:, i, :]), dim=1)
            feats.append(getattr(self, f"o{i + 1}a{i + 1}")(obs_w_act))
        return self.out_feature_q(self.combine_agents_fea(torch.cat(feats, dim=1)))


def actor_rows(actor, own, grid, nei):
    """Apply the (row-wise) reference actor to (B, N, .) inputs, one agent slot per row."""
    B, N = own.shape[:2]
    out = actor([own.reshape(B * N, -1), grid.reshape(B * N, -1), nei.reshape(B * N, nei.shape[2], 6)])
    return out.reshape(B, N, -1)


def soft_update(target, source, t):
    for tp, sp in zip(target.parameters(), source.parameters()):
        tp.data.copy_((1 - t) * tp.data + t * sp.data)


def ref_update(actor, critic, actor_t, critic_t, batches, gamma=0.95, tau=0.01, lr=1e-3, opts=None, soft=True,
               records=None):
    """One update_myown on explicit batches (list of N dicts of CPU tensors).  ``soft``: the
    ``i_episode % UPDATE_EVERY == 0`` soft update (ATT/maddpg:436-438).  ``records`` (a list): the
    8-field single_eps_critic_cal_record entry of each iteration is appended (ATT/maddpg:372-379)."""
    if opts is None:
        opts = (torch.optim.Adam(actor.parameters(), lr=lr), torch.optim.Adam(critic.parameters(), lr=lr))
    a_opt, c_opt = opts
    stats = []
    for agent, b in enumerate(batches):
        na = actor_rows(actor_t, b["n_own"], b["n_radar"], b["n_nei"])
        q = critic([b["s_own"], b["s_radar"]], b["act"])
        with torch.no_grad():
            qn = critic_t([b["n_own"], b["n_radar"]], na).squeeze()
            done_comb = torch.from_numpy(np.array([1 if any(torch.eq(d, 1)) else 0 for d in b["done"]]))
            tar_before = gamma * qn * (1 - done_comb)
            reward_cal = b["rew"].clone()
            target = b["rew"][:, agent] + gamma * qn * (1 - done_comb)
            target = target.unsqueeze(1)
        loss_q = nn.MSELoss()(q, target.detach())
        if records is not None:
            tb, rc, ta, lq = (x.detach().cpu().numpy() for x in (tar_before, reward_cal, target, loss_q))
            records.append([tb, rc, ta, lq, (tb.min(), tb.max()), (rc.min(), rc.max()), (ta.min(), ta.max()),
                            (lq.min(), lq.max())])
        c_opt.zero_grad()
        loss_q.backward()
        c_opt.step()
        a_i = actor_rows(actor, b["s_own"], b["s_radar"], b["s_nei"])
        loss_a = -critic([b["s_own"], b["s_radar"]], a_i).mean()
        a_opt.zero_grad()
        loss_a.backward()
        a_opt.step()
        stats.append((loss_q.item(), loss_a.item(), q.detach().clone(), target.squeeze(1).clone()))
    if soft:
        soft_update(critic_t, critic, tau)
        soft_update(actor_t, actor, tau)
    return stats, opts


def ref_update_dp(actor, critic, actor_t, critic_t, rank_batches, gamma=0.95, tau=0.01, lr=1e-3, opts=None):
    """One data-parallel update_myown: every rank holds its own replay
    shard and samples its own batch i for iteration i; before each Adam step the ranks average
    their gradients (all_reduce(SUM) / world, ATT/maddpg:375-425 per rank).  Restated literally:
    each rank's loss on its own batch, backward of loss / world accumulated into the one set of
    gradients, then the Adam step.  rank_batches[r] = the N batch dicts of rank r.  Returns
    stats[r] = [(loss_q, loss_a, q, target)] per iteration on rank r's batch."""
    ws = len(rank_batches)
    N = len(rank_batches[0])
    if opts is None:
        opts = (torch.optim.Adam(actor.parameters(), lr=lr), torch.optim.Adam(critic.parameters(), lr=lr))
    a_opt, c_opt = opts
    stats = [[] for _ in range(ws)]
    for agent in range(N):
        targets = []
        for r in range(ws):
            b = rank_batches[r][agent]
            with torch.no_grad():
                na = actor_rows(actor_t, b["n_own"], b["n_radar"], b["n_nei"])
                qn = critic_t([b["n_own"], b["n_radar"]], na).squeeze()
                done_comb = torch.from_numpy(np.array([1 if any(torch.eq(d, 1)) else 0 for d in b["done"]]))
                targets.append((b["rew"][:, agent] + gamma * qn * (1 - done_comb)).unsqueeze(1))
        c_opt.zero_grad()
        lq, qs = [], []
        for r in range(ws):
            b = rank_batches[r][agent]
            q = critic([b["s_own"], b["s_radar"]], b["act"])
            loss_q = nn.MSELoss()(q, targets[r])
            (loss_q / ws).backward()
            lq.append(loss_q.item())
            qs.append(q.detach().clone())
        c_opt.step()
        a_opt.zero_grad()
        la = []
        for r in range(ws):
            b = rank_batches[r][agent]
            a_i = actor_rows(actor, b["s_own"], b["s_radar"], b["s_nei"])
            loss_a = -critic([b["s_own"], b["s_radar"]], a_i).mean()
            (loss_a / ws).backward()
            la.append(loss_a.item())
        a_opt.step()
        for r in range(ws):
            stats[r].append((lq[r], la[r], qs[r], targets[r].squeeze(1).clone()))
    soft_update(critic_t, critic, tau)
    soft_update(actor_t, actor, tau)
    return stats, opts


def random_transitions(E, N, seed, zero_nei_frac=0.1):
    g = torch.Generator().manual_seed(seed)
    D0, K = 6 + 4 * (N - 1), N - 1

    def r(*s):
        return torch.randn(*s, generator=g)
    s_nei = r(E, N, K, 6) * 0.5
    n_nei = r(E, N, K, 6) * 0.5
    zmask = torch.rand(E, N, K, generator=g) < zero_nei_frac
    s_nei[zmask] = 0.0
    n_nei[zmask] = 0.0
    s_nei[0, 0] = 0.0        # one all-masked attention row
    act = torch.rand(E, N, 2, generator=g) * 2 - 1
    rew = r(E, 1).repeat(1, N) * 5
    done = (torch.rand(E, N, generator=g) < 0.1).to(torch.uint8)
    return dict(s_own=r(E, N, D0), s_radar=torch.rand(E, N, 18, generator=g) * 15, s_nei=s_nei, act=act,
                rew=rew, done=done, n_own=r(E, N, D0), n_radar=torch.rand(E, N, 18, generator=g) * 15, n_nei=n_nei)


def check_one_update(MADDPG_cls, device="cuda", N=3, B=64, E=32, tol=1e-5, seed=0, iters=1, eps=1e-8,
                     param_tol=None, update_every=1, check_records=False):
    """Device learner vs this restatement on identical weights and batches; raises on mismatch.
    Q, targets and losses are compared at ``tol``; parameters at ``param_tol`` (default ``tol``).
    ``eps`` is Adam's epsilon on both sides: where a gradient is rounding noise (|g| << eps) Adam's
    step is ~lr g / eps instead of +-lr, so a larger eps makes the parameters compare the gradients.
    ``update_every``: update ``it`` (i_episode = it + 1) soft-updates the targets only when
    i_episode % update_every == 0.  ``check_records``: the device's 8-field critic records
    (``critic_records``) against the restatement's at ``tol``."""
    m = MADDPG_cls([6 + 4 * (N - 1), 18, 6], [6 + 4 * (N - 1), 18, 6], 2, n_agents=N, device=device, seed=seed,
                   memory_length=4 * E, batch_size=B)
    rep = m.attach_replay(4 * E)
    m.actor_optimizer.eps = m.critic_optimizer.eps = eps
    D0 = 6 + 4 * (N - 1)
    actor, critic = RefActor([D0, 18, 6], 2), RefCritic([D0, 18, 6], N, 2)
    actor.load_state_dict(m.actors.reference_state_dict())
    critic.load_state_dict(m.critics.reference_state_dict())
    actor_t, critic_t = RefActor([D0, 18, 6], 2), RefCritic([D0, 18, 6], N, 2)
    actor_t.load_state_dict(actor.state_dict())
    critic_t.load_state_dict(critic.state_dict())
    host = {k: [] for k in ("s_own", "s_radar", "s_nei", "act", "rew", "done", "n_own", "n_radar", "n_nei")}
    for p in range(4):
        tr = random_transitions(E, N, seed * 100 + p)
        dev = {k: v.to(device).contiguous() for k, v in tr.items()}
        rep.push_batch(*[dev[k] for k in host])
        for k in host:
            host[k].append(tr[k])
    host = {k: torch.cat(v) for k, v in host.items()}
    gen = np.random.default_rng(seed)
    opts = None
    for it in range(iters):
        idx = [torch.from_numpy(gen.choice(len(rep), size=B, replace=False).astype(np.int32)) for _ in range(N)]
        soft = (it + 1) % update_every == 0
        stats = m.update(B, use_graph=False, idx_list=[i.to(device) for i in idx], soft_update=soft)
        recs = m.critic_records(stats) if check_records else None
        batches = []
        for i in idx:
            b = {k: v[i.long()].clone() for k, v in host.items()}
            b["done"] = b["done"].to(torch.float32)
            batches.append(b)
        if opts is None:
            opts = (torch.optim.Adam(actor.parameters(), lr=1e-3, eps=eps),
                    torch.optim.Adam(critic.parameters(), lr=1e-3, eps=eps))
        rrecs = [] if check_records else None
        rstats, opts = ref_update(actor, critic, actor_t, critic_t, batches, opts=opts, soft=soft, records=rrecs)
        if check_records:
            for mine, ref in zip(recs, rrecs):
                if len(mine) != 8:
                    raise AssertionError("critic record: 8 fields")
                for k in range(4):
                    a, b = np.asarray(mine[k]), np.asarray(ref[k])
                    if a.shape != b.shape or not np.allclose(a, b, atol=tol, rtol=tol):
                        raise AssertionError(f"critic record field {k}: {a.shape} vs {b.shape}")
                for k in range(4, 8):
                    if not np.allclose(np.asarray(mine[k]), np.asarray(ref[k]), atol=tol, rtol=tol):
                        raise AssertionError(f"critic record field {k}: {mine[k]} vs {ref[k]}")
        for (lq, la, q, tg), (rlq, rla, rq, rtg) in zip(stats, rstats):
            if not torch.allclose(q.cpu().squeeze(1), rq.squeeze(1), atol=tol, rtol=tol):
                raise AssertionError(f"Q mismatch {float((q.cpu().squeeze(1) - rq.squeeze(1)).abs().max())}")
            if not torch.allclose(tg.cpu(), rtg, atol=tol, rtol=tol):
                raise AssertionError(f"target mismatch {float((tg.cpu() - rtg).abs().max())}")
            if abs(float(lq) - rlq) > tol * max(1.0, abs(rlq)) or abs(float(la) - rla) > tol * max(1.0, abs(rla)):
                raise AssertionError(f"loss mismatch {float(lq)} {rlq} {float(la)} {rla}")
    for mine, ref in ((m.actors.reference_state_dict(), actor.state_dict()),
                      (m.critics.reference_state_dict(), critic.state_dict()),
                      (m.actors_target.reference_state_dict(), actor_t.state_dict()),
                      (m.critics_target.reference_state_dict(), critic_t.state_dict())):
        for k in ref:
            d = float((mine[k] - ref[k]).abs().max())
            if d > (tol if param_tol is None else param_tol):
                raise AssertionError(f"param {k} differs by {d}")
    for opt in (m.actor_optimizer, m.critic_optimizer):      # Adam steps: N per update, soft or not
        if int(opt.step_t) != N * iters:
            raise AssertionError(f"Adam step counter {int(opt.step_t)} != {N * iters}")
    return True
