"""world_size 2 / 4 / 8 gloo tests of the data-parallel gradient exchange (CPU, no GPU), on the product's
own flat-buffer layout: the learners' gradient buffers and the collectives they issue between
graph segments (maddpg.MADDPG._share_grads / _allreduce_grads, gru.MADDPG._allreduce,
uam_learner.MADDPG._allreduce_flat over parallel.allreduce_sum_: the collectives SUM, and the
Adam launch after each divides by the world size); plus the data-parallel restatements of the
oracle (``*_dp``) against the update on the union of the shards."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gru_ref, learner_ref
from oracle import uam_learner_ref as UR


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fill_grads(module, rank, salt):
    """Rank-specific gradient values written through each parameter's own ``.grad`` view."""
    g = torch.Generator().manual_seed(1000 * rank + salt)
    for p in module.parameters():
        p.grad.copy_(torch.randn(p.shape, generator=g, dtype=p.grad.dtype))


def _grads(module):
    return torch.cat([p.grad.reshape(-1).clone() for p in module.parameters()])


def _worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from multi_agent_aac_amd import gru, uam_learner
    from multi_agent_aac_amd.maddpg import MADDPG
    pg = dist.group.WORLD
    res = {}
    # ATT: [critic | actor] halves of one buffer, one collective for one or both networks
    m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=5, device="cpu", seed=1, process_group=pg)
    nc = m.fc.numel
    res["att_alias"] = (m.fc.grad.data_ptr() == m.grads.data_ptr() and
                        m.fa.grad.data_ptr() == m.grads[nc:].data_ptr() and
                        all(p.grad.data_ptr() == m.grads[off:].data_ptr() for p, off, _ in m.fc.slices) and
                        all(p.grad.data_ptr() == m.grads[nc + off:].data_ptr() for p, off, _ in m.fa.slices))
    res["att_params"] = (m.fc.data.clone(), m.fa.data.clone())
    for tag, crit, act in (("c", True, False), ("a", False, True), ("ca", True, True)):
        _fill_grads(m.critics, rank, 1)
        _fill_grads(m.actors, rank, 2)
        res[f"att_{tag}_local"] = (_grads(m.critics), _grads(m.actors))
        m._allreduce_grads(critic=crit, actor=act)
        res[f"att_{tag}"] = (_grads(m.critics), _grads(m.actors))
    # GRU: one flat gradient per network kind (all agents), one collective each
    g = gru.MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=4, device="cpu", seed=1, process_group=pg)
    res["gru_params"] = (g.fc.data.clone(), g.fa.data.clone())
    for net in g.critics:
        _fill_grads(net, rank, 3)
    res["gru_local"] = g.fc.grad.clone()
    g._allreduce(g.fc)
    res["gru"] = (g.fc.grad.clone(), torch.cat([_grads(net) for net in g.critics]))
    # UAM: the fused learner's summed gradient [critic | actor], float64, one collective
    u = uam_learner.MADDPG([7, 20, 18, 6], [7, 20, 18, 6], 2, n_agents=5, device="cpu", seed=1, process_group=pg)
    st = u._flat_state()
    res["uam_params"] = st["flat"].clone()
    gflat = torch.randn(st["nC"] + st["nA"], dtype=torch.float64, generator=torch.Generator().manual_seed(rank))
    res["uam_local"] = gflat.clone()
    u._allreduce_flat(gflat)
    res["uam"] = gflat
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 4, 8])
def test_product_grad_exchange(ws):
    """Every rank ends with the sum of all ranks' gradients (bit-identical on every rank), the other
    network's half untouched; the Adam launch then applies 1 / ws (exact for these power-of-two worlds,
    aac_learn.hip)."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(ws, port, out), nprocs=ws, join=True)
    rs = [out[r] for r in range(ws)]
    r0 = rs[0]
    assert all(r["att_alias"] for r in rs)            # param.grad views live in the shared [critic | actor] buffer
    for r in rs[1:]:                                  # identical init on every rank (same seed)
        for k in ("att_params", "gru_params"):
            assert all(torch.equal(a, b) for a, b in zip(r0[k], r[k]))
        assert torch.equal(r0["uam_params"], r["uam_params"])
    for tag, crit, act in (("c", True, False), ("a", False, True), ("ca", True, True)):
        for j, reduced in enumerate((crit, act)):
            locs = [r[f"att_{tag}_local"][j] for r in rs]
            assert not torch.equal(locs[0], locs[1])
            # the mean-gradient restatement: (sum of the ranks' gradients) / ws, summed in rank order
            want = sum(locs[1:], locs[0].clone())
            for r in rs:
                got = r[f"att_{tag}"][j]
                if reduced:
                    torch.testing.assert_close(got, want, rtol=0, atol=1e-5)
                    torch.testing.assert_close(got / ws, want / ws, rtol=0, atol=1e-6)
                else:                                      # the other network's half is not touched
                    assert torch.equal(got, r[f"att_{tag}_local"][j])
            if reduced:
                assert all(torch.equal(r0[f"att_{tag}"][j], r[f"att_{tag}"][j]) for r in rs)
    gsum = sum((r["gru_local"] for r in rs[1:]), rs[0]["gru_local"].clone())
    usum = sum((r["uam_local"] for r in rs[1:]), rs[0]["uam_local"].clone())
    for r in rs:
        torch.testing.assert_close(r["gru"][0], gsum, rtol=0, atol=1e-5)
        assert torch.equal(r["gru"][0], r["gru"][1])      # the per-parameter views see the sum
        torch.testing.assert_close(r["uam"], usum, rtol=0, atol=1e-13)
        assert torch.equal(r0["gru"][0], r["gru"][0]) and torch.equal(r0["uam"], r["uam"])


def _split(b, B, n=2):
    return [{k: v[i * B:(i + 1) * B] for k, v in b.items()} for i in range(n)]


@pytest.mark.parametrize("ns", [2, 4, 8])
def test_dp_restatements_equal_union_batch(ns):
    """The mean over ns equal-size shards of the per-shard gradients of a mean loss is the gradient
    of the loss on their union: ``*_dp`` with ns shards (the ranks of a world of ns) matches the
    single-process restatement on the concatenated batch (a check of the data-parallel oracles
    themselves)."""
    torch.manual_seed(0)
    N, D0, B = 3, 14, 64 // ns
    tr = learner_ref.random_transitions(ns * B, N, 5)
    tr["done"] = tr["done"].float()
    nets = [learner_ref.RefActor([D0, 18, 6], 2), learner_ref.RefCritic([D0, 18, 6], N, 2)]
    a1 = [copy.deepcopy(n) for n in nets] + [copy.deepcopy(n) for n in nets]
    a2 = [copy.deepcopy(n) for n in a1]
    learner_ref.ref_update(*a1, [tr] * N)
    learner_ref.ref_update_dp(*a2, [[s] * N for s in _split(tr, B, ns)])
    for x, y in zip(a1, a2):
        for p, q in zip(x.parameters(), y.parameters()):
            torch.testing.assert_close(p, q, rtol=0, atol=2e-6)
    g = gru_ref.random_gru_transitions(ns * B, N, 6, D0=6)
    g["done"] = g["done"].float()
    acts = [gru_ref.RefGRUActor([6, 18, 6], 2) for _ in range(N)]
    crits = [gru_ref.RefGRUCritic([6, 18, 6], 2) for _ in range(N)]
    s1 = [copy.deepcopy(acts), copy.deepcopy(crits), copy.deepcopy(acts), copy.deepcopy(crits)]
    s2 = copy.deepcopy(s1)
    gru_ref.ref_gru_update(*s1, g, 6)
    gru_ref.ref_gru_update_dp(*s2, _split(g, B, ns), 6)
    for x, y in zip(s1, s2):
        for nx, ny in zip(x, y):
            for p, q in zip(nx.parameters(), ny.parameters()):
                torch.testing.assert_close(p, q, rtol=0, atol=2e-6)
    gen = torch.Generator().manual_seed(7)
    r = lambda *s: torch.rand(*s, generator=gen, dtype=torch.float64) * 2 - 1   # noqa: E731
    ub = dict(own=r(ns * B, 7), radar=r(ns * B, 18).abs() * 5, act=r(ns * B, 2), rew=r(ns * B) * 50,
              done=(r(ns * B) > 0.8).double(), n_own=r(ns * B, 7), n_radar=r(ns * B, 18).abs() * 5)
    a, c = UR.RefActor().double(), UR.RefCritic().double()
    u1 = [copy.deepcopy(a), copy.deepcopy(c), copy.deepcopy(a), copy.deepcopy(c)]
    u2 = copy.deepcopy(u1)
    o1 = (torch.optim.Adam(u1[0].parameters(), lr=1e-4), torch.optim.Adam(u1[1].parameters(), lr=1e-4))
    o2 = (torch.optim.Adam(u2[0].parameters(), lr=1e-4), torch.optim.Adam(u2[1].parameters(), lr=1e-4))
    UR.ref_update(*u1, *o1, ub)
    UR.ref_update_dp(*u2, *o2, _split(ub, B, ns))
    for x, y in zip(u1, u2):
        for p, q in zip(x.parameters(), y.parameters()):
            torch.testing.assert_close(p, q, rtol=0, atol=1e-12)


def test_rank_seeds_distinct():
    from multi_agent_aac_amd import parallel
    seeds = {parallel.rank_seed(7, r) for r in range(8)}
    assert len(seeds) == 8
