"""Two ranks on the one GPU of the test box (gloo backend, world_size 2): the multi-rank fused
update -- one captured graph per segment between the gradient all-reduces, the critic step of iteration i+1 beside the actor step of i -- must give exactly
the single-process result when both ranks hold the same data (the mean of two identical
gradients is the gradient)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import learner_ref

pytestmark = pytest.mark.gpu
KEYS = ("s_own", "s_radar", "s_nei", "act", "rew", "done", "n_own", "n_radar", "n_nei")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(pg, N, B, E):
    from multi_agent_aac_amd.maddpg import MADDPG
    m = MADDPG([6 + 4 * (N - 1), 18, 6], [6 + 4 * (N - 1), 18, 6], 2, n_agents=N, device="cuda:0", seed=1,
               batch_size=B, process_group=pg)
    rep = m.attach_replay(4 * E, seed=9)
    for p in range(3):
        tr = learner_ref.random_transitions(E, N, 50 + p)
        rep.push_batch(*[tr[k].to("cuda:0").contiguous() for k in KEYS])
    return m


def _worker(rank, ws, port, q):
    try:
        _work(rank, ws, port, q)
    except BaseException as e:      # report instead of leaving the peer blocked in a collective
        q.put((rank, {"error": repr(e)}))
        raise


def _work(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    N, B, E = 5, 128, 256
    par = _model(dist.group.WORLD, N, B, E)
    solo = _model(None, N, B, E)
    for _ in range(3):
        par.update(B, use_graph=True, want_stats=False)
        solo.update(B, use_graph=True, want_stats=False)
    torch.cuda.synchronize()
    res = {"segmented": isinstance(par._graph, tuple),
           "n_segments": len(par._graph[0]) if isinstance(par._graph, tuple) else 0,
           "actor_equal": bool(torch.equal(par.fa.data, solo.fa.data)),
           "critic_equal": bool(torch.equal(par.fc.data, solo.fc.data)),
           "target_equal": bool(torch.equal(par.fc_t.data, solo.fc_t.data))}
    q.put((rank, res))
    dist.destroy_process_group()


def test_segmented_graph_update_two_ranks(native_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=150) for _ in procs)
    for r in range(2):
        assert "error" not in out[r], out[r]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        res = out[r]
        assert res["segmented"] and res["n_segments"] == 7        # N + 1 all-reduces per update, N = 5
        assert res["actor_equal"] and res["critic_equal"] and res["target_equal"], res
