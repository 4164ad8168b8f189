"""torch-CPU fp32 restatement of the GRU-actor MADDPG learner (TEST INFRASTRUCTURE ONLY).

SURVEY.md section 8(f) row f2 (config 4, ``randomOD_gru_radar``).  Follows, as text,
MADDPG_ownENV_randomOD_Wgru_radar (``WGRU/`` below):
  GRUCELL_actor_TwoPortion            WGRU/Nnetworks:181-198  own_fc (d_own -> 64, ReLU),
                                      own_grid (18 -> 64, ReLU), GRUCell(128 -> 64) on the
                                      carried hidden state, outlay (64 -> 2, Tanh); returns (a, h')
  critic_single_obs_wGRU_TwoPortion   WGRU/Nnetworks:428-446  SA_fc (d_own + 2 -> 64, ReLU) on
                                      [own, a], SA_grid (18 -> 64, ReLU), GRUCell(128 -> 64) on the
                                      actor's hidden state, own_fc_outlay (64 -> 1); returns (q, h')
  update_myown                        WGRU/maddpg:211-326  ONE sampled batch for all agents; per
                                      agent i: y = r_i + gamma Q'_i(s'_i, pi'_i(s'_i, h'_i), h'_i)(1 - d_i),
                                      MSE critic step, actor loss 3 - mean Q_i(s_i, pi_i(s_i, h_i), h_i),
                                      one Adam per network; soft update of every target after the
                                      loop (WGRU/maddpg:318-322, UPDATE_EVERY = 1, WGRU/main:374)
  choose_action                       WGRU/maddpg:336-428  (act, h') = actor_i(obs_i, h_i) per agent
The agents' networks are disjoint and the batch is read-only, so the per-agent loop of the
reference equals one step of all agents at once; this restatement keeps the loop.
"""
import torch
import torch.nn as nn


class RefGRUActor(nn.Module):
    def __init__(self, actor_dim, n_actions, hidden=64):
        super().__init__()
        self.own_fc = nn.Sequential(nn.Linear(actor_dim[0], 64), nn.ReLU())
        self.own_grid = nn.Sequential(nn.Linear(actor_dim[1], 64), nn.ReLU())
        self.rnn_hidden_dim = hidden
        self.gru_cell = nn.GRUCell(64 + 64, hidden)
        self.outlay = nn.Sequential(nn.Linear(64, n_actions), nn.Tanh())

    def forward(self, cur_state, history_hidden_state):
        own_obs = self.own_fc(cur_state[0])
        own_grid = self.own_grid(cur_state[1])
        merge_obs_grid = torch.cat((own_obs, own_grid), dim=1)
        h_in = history_hidden_state.reshape(-1, self.rnn_hidden_dim)
        h = self.gru_cell(merge_obs_grid, h_in)
        return self.outlay(h), h


class RefGRUCritic(nn.Module):
    def __init__(self, critic_obs, n_actions, hidden=64):
        super().__init__()
        self.SA_fc = nn.Sequential(nn.Linear(critic_obs[0] + n_actions, 64), nn.ReLU())
        self.SA_grid = nn.Sequential(nn.Linear(critic_obs[1], 64), nn.ReLU())
        self.rnn_hidden_dim = hidden
        self.gru_cell = nn.GRUCell(64 + 64, hidden)
        self.own_fc_outlay = nn.Linear(64, 1)

    def forward(self, single_state, single_action, history_hidden_state):
        obs_w_action = torch.cat((single_state[0], single_action), dim=1)
        own = self.SA_fc(obs_w_action)
        grid = self.SA_grid(single_state[1])
        merge = torch.cat((own, grid), dim=1)
        h_in = history_hidden_state.reshape(-1, self.rnn_hidden_dim)
        h = self.gru_cell(merge, h_in)
        return self.own_fc_outlay(h), h


def soft_update(target, source, t):
    for tp, sp in zip(target.parameters(), source.parameters()):
        tp.data.copy_((1 - t) * tp.data + t * sp.data)


def ref_gru_update(actors, critics, actors_t, critics_t, b, d_own, gamma=0.95, tau=0.01, lr=1e-3, opts=None,
                   soft=True):
    """One update_myown on one batch dict of CPU tensors (B, N, .); own rows are cut to d_own.
    ``soft``: the ``i_episode % UPDATE_EVERY == 0`` soft update of WGRU/maddpg:320-324."""
    N = len(actors)
    if opts is None:
        opts = ([torch.optim.Adam(a.parameters(), lr=lr) for a in actors],
                [torch.optim.Adam(c.parameters(), lr=lr) for c in critics])
    a_opts, c_opts = opts
    own, nown = b["s_own"][..., :d_own], b["n_own"][..., :d_own]
    stats = []
    for i in range(N):
        with torch.no_grad():
            na = actors_t[i]([nown[:, i], b["n_radar"][:, i]], b["h_next"][:, i])[0]
        q = critics[i]([own[:, i], b["s_radar"][:, i]], b["act"][:, i], b["h_cur"][:, i])[0]
        with torch.no_grad():
            qn = critics_t[i]([nown[:, i], b["n_radar"][:, i]], na, b["h_next"][:, i])[0].squeeze()
            target = (b["rew"][:, i] + gamma * qn * (1 - b["done"][:, i])).unsqueeze(1)
        loss_q = nn.MSELoss()(q, target.detach())
        c_opts[i].zero_grad()
        loss_q.backward()
        c_opts[i].step()
        a_i = actors[i]([own[:, i], b["s_radar"][:, i]], b["h_cur"][:, i])[0]
        loss_a = 3 - critics[i]([own[:, i], b["s_radar"][:, i]], a_i, b["h_cur"][:, i])[0].mean()
        a_opts[i].zero_grad()
        loss_a.backward()
        a_opts[i].step()
        stats.append((loss_q.item(), loss_a.item(), q.detach().clone(), target.squeeze(1).clone()))
    for i in range(N if soft else 0):
        soft_update(critics_t[i], critics[i], tau)
        soft_update(actors_t[i], actors[i], tau)
    return stats, opts


def ref_gru_update_dp(actors, critics, actors_t, critics_t, rank_b, d_own, gamma=0.95, tau=0.01, lr=1e-3,
                      opts=None):
    """Data-parallel update_myown: rank r holds batch rank_b[r] of its own
    replay shard; every Adam step uses the mean over the ranks of their gradients (each rank's loss
    of WGRU/maddpg:242-310 on its own batch, backward of loss / world accumulated).  Returns
    stats[r] = [(loss_q, loss_a, q, target)] per agent on rank r's batch."""
    N, ws = len(actors), len(rank_b)
    if opts is None:
        opts = ([torch.optim.Adam(a.parameters(), lr=lr) for a in actors],
                [torch.optim.Adam(c.parameters(), lr=lr) for c in critics])
    a_opts, c_opts = opts
    stats = [[] for _ in range(ws)]
    for i in range(N):
        rows = []
        for b in rank_b:
            own, nown = b["s_own"][..., :d_own], b["n_own"][..., :d_own]
            with torch.no_grad():
                na = actors_t[i]([nown[:, i], b["n_radar"][:, i]], b["h_next"][:, i])[0]
                qn = critics_t[i]([nown[:, i], b["n_radar"][:, i]], na, b["h_next"][:, i])[0].squeeze()
                target = (b["rew"][:, i] + gamma * qn * (1 - b["done"][:, i])).unsqueeze(1)
            rows.append((own, target))
        c_opts[i].zero_grad()
        lq, qs = [], []
        for (own, target), b in zip(rows, rank_b):
            q = critics[i]([own[:, i], b["s_radar"][:, i]], b["act"][:, i], b["h_cur"][:, i])[0]
            loss_q = nn.MSELoss()(q, target)
            (loss_q / ws).backward()
            lq.append(loss_q.item())
            qs.append(q.detach().clone())
        c_opts[i].step()
        a_opts[i].zero_grad()
        la = []
        for (own, _), b in zip(rows, rank_b):
            a_i = actors[i]([own[:, i], b["s_radar"][:, i]], b["h_cur"][:, i])[0]
            loss_a = 3 - critics[i]([own[:, i], b["s_radar"][:, i]], a_i, b["h_cur"][:, i])[0].mean()
            (loss_a / ws).backward()
            la.append(loss_a.item())
        a_opts[i].step()
        for r in range(ws):
            stats[r].append((lq[r], la[r], qs[r], rows[r][1].squeeze(1).clone()))
    for i in range(N):
        soft_update(critics_t[i], critics[i], tau)
        soft_update(actors_t[i], actors[i], tau)
    return stats, opts


def ref_gru_act(actors, own, radar, h, d_own):
    """Deterministic actions and next hidden states of all agents: own (E, N, >= d_own)."""
    outs, hs = [], []
    with torch.no_grad():
        for i, a in enumerate(actors):
            act, hn = a([own[:, i, :d_own], radar[:, i]], h[:, i])
            outs.append(act)
            hs.append(hn)
    return torch.stack(outs, 1), torch.stack(hs, 1)


def random_gru_transitions(E, N, seed, H=64, D0=None):
    """Synthetic transitions of the GRU learner: the ATT env's fields plus the actor hidden
    states before (h_cur) and after (h_next) the step.  D0: own-row width (default the ATT env's
    6 + 4 (N - 1); 6 for the WGRU env variant)."""
    g = torch.Generator().manual_seed(seed)
    D0, K = D0 or 6 + 4 * (N - 1), N - 1

    def r(*s):
        return torch.randn(*s, generator=g)
    act = torch.rand(E, N, 2, generator=g) * 2 - 1
    return dict(s_own=r(E, N, D0), s_radar=torch.rand(E, N, 18, generator=g) * 15, s_nei=r(E, N, K, 6) * 0.5,
                act=act, rew=r(E, N) * 5, done=(torch.rand(E, N, generator=g) < 0.1).to(torch.uint8),
                n_own=r(E, N, D0), n_radar=torch.rand(E, N, 18, generator=g) * 15, n_nei=r(E, N, K, 6) * 0.5,
                h_cur=torch.tanh(r(E, N, H)), h_next=torch.tanh(r(E, N, H)))
