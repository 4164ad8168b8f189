"""CPU float64 restatement of the UAM learner's ``update_myown`` (default flags).
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

UAM/ = MADDPG_ownENV_randomOD_radar_N_model_use_tdCPA_forV2_changeskin_UAM.  Follows, as text:
  ActorNetwork_TwoPortion      UAM/nets:167-190   (second encoder reads the 18-wide radar: R1)
  critic_single_TwoPortion     UAM/nets:692-720
  update_myown                 UAM/maddpg:304-595 (var_iteration = 1, individual rewards / dones)
  soft_update                  UAM/maddpg:21-25
Written independently of multi_agent_aac_amd.uam_learner; modules are float64 like UAM/maddpg:148-180.
"""
import torch
import torch.nn as nn


class RefActor(nn.Module):
    def __init__(self, d_own=7, d_radar=18, n_act=2):
        super().__init__()
        self.own_fc = nn.Sequential(nn.Linear(d_own, 64), nn.ReLU())
        self.own_grid = nn.Sequential(nn.Linear(d_radar, 64), nn.ReLU())
        self.merge_feature = nn.Sequential(nn.Linear(128, 128), nn.ReLU())
        self.act_out = nn.Sequential(nn.Linear(128, n_act), nn.Tanh())

    def forward(self, s):
        own_obs = self.own_fc(s[0])
        own_grid = self.own_grid(s[1])
        return self.act_out(self.merge_feature(torch.cat((own_obs, own_grid), dim=1)))


class RefCritic(nn.Module):
    def __init__(self, d_own=7, d_radar=18, n_act=2):
        super().__init__()
        self.SA_fc = nn.Sequential(nn.Linear(d_own + n_act, 64), nn.ReLU())
        self.SA_grid = nn.Sequential(nn.Linear(d_radar, 64), nn.ReLU())
        self.merge_fc_grid = nn.Sequential(nn.Linear(128, 256), nn.ReLU())
        self.out_feature_q = nn.Sequential(nn.Linear(256, 1))

    def forward(self, s, a):
        own = self.SA_fc(torch.cat((s[0], a), dim=1))
        grid = self.SA_grid(s[1])
        return self.out_feature_q(self.merge_fc_grid(torch.cat((own, grid), dim=1)))


def soft_update(target, source, t):
    for tp, sp in zip(target.parameters(), source.parameters()):
        tp.data.copy_(tp.data * (1.0 - t) + sp.data * t)


def ref_update(actor, critic, actor_t, critic_t, opt_a, opt_c, b, gamma=0.95, tau=0.01):
    """One update_myown on the batch dict b (own, radar, act, rew (B,), done (B,), n_own, n_radar)."""
    s0, s2 = b["own"], b["radar"]
    n0, n2 = b["n_own"], b["n_radar"]
    next_actions = actor_t([n0, n2])
    current_Q = critic([s0, s2], b["act"])
    with torch.no_grad():
        next_q = critic_t([n0, n2], next_actions).squeeze()
        target_Q = (b["rew"] + gamma * next_q * (1 - b["done"])).unsqueeze(1)
    loss_Q = nn.MSELoss()(current_Q, target_Q.detach())
    opt_c.zero_grad()
    loss_Q.backward()
    opt_c.step()
    ac = actor([s0, s2])
    actor_loss = -critic([s0, s2], ac).mean()
    opt_a.zero_grad()
    actor_loss.backward()
    opt_a.step()
    soft_update(critic_t, critic, tau)
    soft_update(actor_t, actor, tau)
    return float(loss_Q.detach()), float(actor_loss.detach())


def ref_update_dp(actor, critic, actor_t, critic_t, opt_a, opt_c, rank_b, gamma=0.95, tau=0.01):
    """Data-parallel update_myown: rank r's loss of UAM/maddpg:346-512 on
    its own batch rank_b[r]; each Adam step uses the mean of the ranks' gradients (backward of
    loss / world accumulated).  Returns [(loss_q, loss_a)] per rank."""
    ws = len(rank_b)
    targets = []
    for b in rank_b:
        with torch.no_grad():
            n0, n2 = b["n_own"], b["n_radar"]
            next_q = critic_t([n0, n2], actor_t([n0, n2])).squeeze()
            targets.append((b["rew"] + gamma * next_q * (1 - b["done"])).unsqueeze(1))
    opt_c.zero_grad()
    lq = []
    for b, y in zip(rank_b, targets):
        loss_Q = nn.MSELoss()(critic([b["own"], b["radar"]], b["act"]), y)
        (loss_Q / ws).backward()
        lq.append(float(loss_Q.detach()))
    opt_c.step()
    opt_a.zero_grad()
    la = []
    for b in rank_b:
        s = [b["own"], b["radar"]]
        actor_loss = -critic(s, actor(s)).mean()
        (actor_loss / ws).backward()
        la.append(float(actor_loss.detach()))
    opt_a.step()
    soft_update(critic_t, critic, tau)
    soft_update(actor_t, actor, tau)
    return list(zip(lq, la))
