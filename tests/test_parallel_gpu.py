"""Two ranks on the one GPU of the test box (gloo backend, world_size 2): the multi-rank fused
updates of the three learners -- one captured graph per segment between the gradient all-reduces
(ATT: the critic step of iteration i+1 beside the actor step of i; GRU; UAM) -- must give exactly
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
GRU_KEYS = KEYS + ("h_cur", "h_next")


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


def _gru_model(pg, N, B, E):
    from multi_agent_aac_amd.gru import MADDPG
    from oracle import gru_ref
    m = MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, device="cuda:0", seed=1, batch_size=B,
               process_group=pg)
    rep = m.attach_replay(4 * E, seed=9)
    for p in range(3):
        tr = gru_ref.random_gru_transitions(E, N, 50 + p)
        rep.push_batch(*[tr[k].to("cuda:0").contiguous() for k in GRU_KEYS])
    return m


def _uam_model(pg, N, B, E):
    from multi_agent_aac_amd import uam_learner as L
    m = L.MADDPG([7, 20, 18, 6], [7, 20, 18, 6], 2, n_agents=N, device="cuda:0", seed=1, batch_size=B,
                 memory_length=4 * E * N, process_group=pg)
    rep = m.attach_replay(4 * E * N, seed=3)
    g = torch.Generator().manual_seed(5)
    rnd = lambda *s: (torch.rand(*s, generator=g, dtype=torch.float64) * 2 - 1).to("cuda:0")   # noqa: E731
    for _ in range(3):
        rep.push_batch(rnd(E, N, 7), rnd(E, N, 18).abs().mul(5), rnd(E, N, 2), rnd(E, N).mul(50),
                       (rnd(E, N) > 0.8).double(), rnd(E, N, 7), rnd(E, N, 18).abs().mul(5))
    return m


def _worker(rank, ws, port, q, kind="att"):
    try:
        {"att": _work, "gru": _work_gru, "uam": _work_uam}[kind](rank, ws, port, q)
    except BaseException as e:      # report instead of leaving the peer blocked in a collective
        q.put((rank, {"error": repr(e)}))
        raise


def _work(rank, ws, port, q):
    dist = _init(rank, ws, port)
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


def _init(rank, ws, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    return dist


def _work_gru(rank, ws, port, q):
    dist = _init(rank, ws, port)
    N, B, E = 4, 128, 256
    par = _gru_model(dist.group.WORLD, N, B, E)
    solo = _gru_model(None, N, B, E)
    for _ in range(3):
        par.update(B, use_graph=True, want_stats=False)
        solo.update(B, use_graph=True, want_stats=False)
    par.update(B, use_graph=False, want_stats=False)       # eager: the same launch list, collectives inline
    solo.update(B, use_graph=False, want_stats=False)
    torch.cuda.synchronize()
    res = {"n_segments": len(par._graph[0]),
           "actor_equal": bool(torch.equal(par.fa.data, solo.fa.data)),
           "critic_equal": bool(torch.equal(par.fc.data, solo.fc.data)),
           "target_equal": bool(torch.equal(par.fc_t.data, solo.fc_t.data) and torch.equal(par.fa_t.data,
                                                                                           solo.fa_t.data))}
    q.put((rank, res))
    dist.destroy_process_group()


def _work_uam(rank, ws, port, q):
    dist = _init(rank, ws, port)
    N, B, E = 5, 128, 256
    par = _uam_model(dist.group.WORLD, N, B, E)
    solo = _uam_model(None, N, B, E)
    for _ in range(3):
        par.update(B, use_graph=True)
        solo.update(B, use_graph=True)
    par.update(B, use_graph=False)                        # eager fused run, collectives inline
    solo.fused(B, solo.replay).run()                      # (one rank's eager update is the torch path)
    torch.cuda.synchronize()
    fp, fs = par._fstate, solo._fstate
    res = {"n_segments": len(par._fu.graphs), "fused": par._fu is not None,
           "actor_equal": bool(torch.equal(fp["flat"][fp["nC"]:], fs["flat"][fs["nC"]:])),
           "critic_equal": bool(torch.equal(fp["flat"][:fp["nC"]], fs["flat"][:fs["nC"]])),
           "target_equal": bool(torch.equal(fp["tflat"], fs["tflat"]) and torch.equal(fp["m2"], fs["m2"]))}
    q.put((rank, res))
    dist.destroy_process_group()


def _run_two(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, kind)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=150) for _ in procs)
    for r in range(2):
        assert "error" not in out[r], out[r]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("kind,n_segments", [("gru", None), ("uam", 3)])
def test_segmented_graph_update_two_ranks_gru_uam(native_lib, kind, n_segments):
    out = _run_two(kind)
    for r in range(2):
        res = out[r]
        assert res["n_segments"] > 1 and (n_segments is None or res["n_segments"] == n_segments), res
        assert res["actor_equal"] and res["critic_equal"] and res["target_equal"], res


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
