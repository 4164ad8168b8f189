"""world_size-2 gloo tests of the data-parallel gradient exchange (CPU, no GPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import learner_ref


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from multi_agent_aac_amd import parallel
    torch.manual_seed(0)
    N, D0, B = 3, 14, 32
    actor = learner_ref.RefActor([D0, 18, 6], 2)
    critic = learner_ref.RefCritic([D0, 18, 6], N, 2)
    params = list(actor.parameters()) + list(critic.parameters())
    flat = torch.zeros(sum(p.numel() for p in params))
    tr = learner_ref.random_transitions(B, N, 100 + rank)     # each rank has its own shard
    tr["done"] = tr["done"].float()
    q = critic([tr["s_own"], tr["s_radar"]], tr["act"])
    a = learner_ref.actor_rows(actor, tr["s_own"], tr["s_radar"], tr["s_nei"])
    loss = (q ** 2).mean() + (a ** 2).mean()
    loss.backward()
    off = 0
    for p in params:
        flat[off:off + p.numel()] = p.grad.reshape(-1)
        off += p.numel()
    local = flat.clone()
    parallel.allreduce_mean_(flat)
    out[rank] = (local, flat)
    dist.destroy_process_group()


def test_allreduce_mean_matches_global_batch():
    ws, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(ws, port, out), nprocs=ws, join=True)
    (l0, f0), (l1, f1) = out[0], out[1]
    assert torch.equal(f0, f1)                       # identical averaged gradient on every rank
    torch.testing.assert_close(f0, (l0 + l1) / 2, rtol=1e-6, atol=1e-7)
    assert not torch.equal(l0, l1)                   # shards really differ


def test_rank_seeds_distinct():
    from multi_agent_aac_amd import parallel
    seeds = {parallel.rank_seed(7, r) for r in range(8)}
    assert len(seeds) == 8
