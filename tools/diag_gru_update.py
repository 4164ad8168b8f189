"""Diagnostic: per-parameter differences between the GRU learner and oracle/gru_ref.py after one
update_myown at several B (run on the GPU box: python tools/diag_gru_update.py 256 512)."""
import copy
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gru_ref  # noqa: E402

KEYS = ("s_own", "s_radar", "s_nei", "act", "rew", "done", "n_own", "n_radar", "n_nei", "h_cur", "h_next")


def run(B, N=8, E=256, eps=1e-3):
    from multi_agent_aac_amd.gru import MADDPG
    m = MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, device="cuda", seed=8, batch_size=B)
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
        rep.push_batch(*[tr[k].to("cuda").contiguous() for k in KEYS])
        for k in KEYS:
            host[k].append(tr[k])
    host = {k: torch.cat(v) for k, v in host.items()}
    m.actor_optimizer.eps = m.critic_optimizer.eps = eps
    opts = ([torch.optim.Adam(a.parameters(), lr=1e-3, eps=eps) for a in actors],
            [torch.optim.Adam(c.parameters(), lr=1e-3, eps=eps) for c in critics])
    gen = np.random.default_rng(17)
    idx = torch.from_numpy(gen.choice(len(rep), size=B, replace=False).astype(np.int32))
    m.update(B, use_graph=False, idx=idx.to("cuda"))
    b = {k: v[idx.long()].clone() for k, v in host.items()}
    b["done"] = b["done"].float()
    gru_ref.ref_gru_update(actors, critics, actors_t, critics_t, b, m.d_own, opts=opts)
    torch.cuda.synchronize()
    worst = []
    for i in range(N):
        for tag, mine, ref in (("actor", m.actors[i], actors[i]), ("critic", m.critics[i], critics[i])):
            for (k, v), (_, rv) in zip(mine.state_dict().items(), ref.state_dict().items()):
                d = (v.cpu() - rv).abs()
                worst.append((float(d.max()), i, tag, k, tuple(d.shape), int((d > 1e-5).sum())))
    worst.sort(reverse=True)
    print(f"B={B}")
    for w in worst[:12]:
        print("  %.3e agent %d %s %s %s n>1e-5=%d" % w)




def intermediates(B, N=8, E=256):
    """Run the plan up to the critic Adam step and check dcat_c and the SA_grid / SA_fc weight
    gradients against float64 recomputes from the device's own buffers."""
    from multi_agent_aac_amd.gru import MADDPG
    m = MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, device="cuda", seed=8, batch_size=B)
    rep = m.attach_replay(4 * E, seed=11)
    for p in range(3):
        tr = gru_ref.random_gru_transitions(E, N, 500 + p)
        rep.push_batch(*[tr[k].to("cuda").contiguous() for k in KEYS])
    fu = m._plan(B)
    idx = torch.from_numpy(np.random.default_rng(17).choice(len(rep), size=B, replace=False).astype(np.int32))
    fu.bidx.copy_(idx.cuda())
    stop = next(k for k, op in enumerate(fu.L) if "adam_at" in getattr(getattr(op, "__code__", None), "co_names", ()))
    for op in fu.L[1:stop]:
        op()
    torch.cuda.synchronize()
    d = lambda t: t.double().cpu()   # noqa: E731
    b = fu.batch
    print(f"B={B} ops before critic adam: {stop}")
    for i in range(N):
        Wih = d(m.critics[i].gru_cell.weight_ih)
        want = (d(fu.dgi_c[:, i]) @ Wih) * (d(fu.cat_c[:, i]) > 0)
        e1 = float((d(fu.dcat_c[:, i]) - want).abs().max())
        g = dict((k, d(v.grad)) for k, v in m.critics[i].named_parameters())
        wg = d(fu.dcat_c[:, i, 64:]).t() @ d(b["s_radar"][:, i])
        e2 = float((g["SA_grid.0.weight"] - wg).abs().max())
        bg = d(fu.dcat_c[:, i, 64:]).sum(0)
        e3 = float((g["SA_grid.0.bias"] - bg).abs().max())
        wf = d(fu.dcat_c[:, i, :64]).t() @ d(fu.Xsa[:, i])
        e4 = float((g["SA_fc.0.weight"] - wf).abs().max())
        print("  agent %d  dcat %.2e  dW_grid %.2e  db_grid %.2e  dW_fc %.2e" % (i, e1, e2, e3, e4))
        if e2 > 1e-4:
            bad = (g["SA_grid.0.weight"] - wg).abs()
            r, c = divmod(int(bad.argmax()), bad.shape[1])
            print("    worst at row", r, "col", c, "got", float(g["SA_grid.0.weight"][r, c]), "want", float(wg[r, c]),
                  "rows>1e-4:", sorted(set((bad > 1e-4).nonzero()[:, 0].tolist())))


def critic_chain(B, N=8, E=256, agent=0):
    """Float64 autograd of agent ``agent``'s critic step against the device buffers, stage by stage."""
    from multi_agent_aac_amd.gru import MADDPG
    m = MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, device="cuda", seed=8, batch_size=B)
    rep = m.attach_replay(4 * E, seed=11)
    for p in range(3):
        tr = gru_ref.random_gru_transitions(E, N, 500 + p)
        rep.push_batch(*[tr[k].to("cuda").contiguous() for k in KEYS])
    fu = m._plan(B)
    idx = torch.from_numpy(np.random.default_rng(17).choice(len(rep), size=B, replace=False).astype(np.int32))
    fu.bidx.copy_(idx.cuda())
    stop = next(k for k, op in enumerate(fu.L) if "adam_at" in getattr(getattr(op, "__code__", None), "co_names", ()))
    for op in fu.L[1:stop]:
        op()
    torch.cuda.synchronize()
    i = agent
    b = {k: v.double().cpu() for k, v in fu.batch.items()}
    c = gru_ref.RefGRUCritic([6, 18, 6], 2).double()
    c.load_state_dict({k: v.double().cpu() for k, v in m.critics[i].state_dict().items()})
    ct = gru_ref.RefGRUCritic([6, 18, 6], 2).double()
    ct.load_state_dict({k: v.double().cpu() for k, v in m.critics_target[i].state_dict().items()})
    d = lambda t: t.detach().double().cpu()   # noqa: E731
    own, radar, act, h = b["s_own"][:, i, :6], b["s_radar"][:, i], b["act"][:, i], b["h_cur"][:, i]
    sa = torch.relu(torch.cat([own, act], 1) @ c.SA_fc[0].weight.t() + c.SA_fc[0].bias)
    gr = torch.relu(radar @ c.SA_grid[0].weight.t() + c.SA_grid[0].bias)
    cat = torch.cat([sa, gr], 1).detach().requires_grad_(True)
    q, hh = c([own, radar], act, h)
    q2 = c.own_fc_outlay(c.gru_cell(cat, h))
    y = d(fu.y[:, i])
    loss = ((q2[:, 0] - y) ** 2).mean()
    loss.backward()
    def rep_(name, got, want):
        e = (d(got) - want).abs()
        print("  %-10s max %.3e  at %s" % (name, float(e.max()), np.unravel_index(int(e.argmax()), e.shape)))
    print(f"B={B} agent {i}")
    rep_("Xsa", fu.Xsa[:, i], torch.cat([own, act], 1))
    rep_("cat_c", fu.cat_c[:, i], cat.detach())
    rep_("q_c", fu.q_c[:, i], q2[:, 0].detach())
    rep_("dcat_c", fu.dcat_c[:, i], cat.grad * (cat.detach() > 0))
    g = dict((k, d(v.grad)) for k, v in m.critics[i].named_parameters())
    dgr = cat.grad[:, 64:] * (gr > 0)
    rep_("dW_grid", g["SA_grid.0.weight"], dgr.t() @ radar)
    rep_("db_grid", g["SA_grid.0.bias"], dgr.sum(0))


if __name__ == "__main__":
    for B in [int(x) for x in sys.argv[1:]] or [256, 512]:
        critic_chain(B)
