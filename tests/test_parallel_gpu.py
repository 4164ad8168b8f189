"""Two ranks on the one GPU of the test box (gloo backend, world_size 2), each holding a DIFFERENT
replay shard (env shards per rank, the gradient mean before every Adam
step).  For the three learners (ATT ``fused.FusedUpdate._merged`` with its N + 1 collectives, GRU, UAM):

* two update_myown calls on explicitly sampled rows are checked against the CPU restatement that
  applies the MEAN of the two ranks' gradients (``learner_ref.ref_update_dp``,
  ``gru_ref.ref_gru_update_dp``, ``uam_learner_ref.ref_update_dp``) at the tolerances of the
  single-rank config-size tests, and both ranks must hold bit-identical parameters afterwards.  A
  skipped, wrong-slice or double-applied all-reduce fails both checks: the shards differ, so each
  rank's own gradient is not the mean;
* the segmented graph (one captured graph per segment between the all-reduces) is bit-equal to the
  eager launch list with its collectives inline, from the device sampler on the same shard.
"""
import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import gru_ref, learner_ref
from oracle import uam_learner_ref as UR

pytestmark = pytest.mark.gpu
KEYS = ("s_own", "s_radar", "s_nei", "act", "rew", "done", "n_own", "n_radar", "n_nei")
GRU_KEYS = KEYS + ("h_cur", "h_next")
EPS = 1e-3       # Adam eps on both sides: the parameters then compare the gradients (test_config_size_gpu)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, ws, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    # AAC_TEST_BACKEND=nccl: one GPU per rank (each process sees only its own, set before the first
    # HIP call by _worker), the collectives captured in the update graph (parallel.capturable)
    dist.init_process_group(os.environ.get("AAC_TEST_BACKEND", "gloo"), rank=rank, world_size=ws)
    return dist


def _cpu(sd):
    return {k: v.detach().cpu().clone() for k, v in sd.items()}


# --------------------------------------------------------------------------- ATT (config 3 learner)
def _att_model(pg, N, B, E, rank, seed=1):
    from multi_agent_aac_amd.maddpg import MADDPG
    m = MADDPG([6 + 4 * (N - 1), 18, 6], [6 + 4 * (N - 1), 18, 6], 2, n_agents=N, device="cuda:0", seed=seed,
               batch_size=B, process_group=pg)
    rep = m.attach_replay(4 * E, seed=9 + rank)
    host = {k: [] for k in KEYS}
    for p in range(3):
        tr = learner_ref.random_transitions(E, N, 50 + p + 1000 * rank)      # rank-distinct shard
        rep.push_batch(*[tr[k].to("cuda:0").contiguous() for k in KEYS])
        for k in KEYS:
            host[k].append(tr[k])
    return m, rep, {k: torch.cat(v) for k, v in host.items()}


def _att_state(m):
    return [_cpu(m.actors.reference_state_dict()), _cpu(m.critics.reference_state_dict()),
            _cpu(m.actors_target.reference_state_dict()), _cpu(m.critics_target.reference_state_dict())]


def _work_att(rank, ws, port):
    dist = _init(rank, ws, port)
    N, B, E = 5, 128, 256
    m, rep, host = _att_model(dist.group.WORLD, N, B, E, rank)
    m.actor_optimizer.eps = m.critic_optimizer.eps = EPS
    res = {"init": _att_state(m), "batches": [], "stats": []}
    gen = np.random.default_rng(77 + rank)
    for _ in range(2):
        idx = [torch.from_numpy(gen.choice(len(rep), size=B, replace=False).astype(np.int32)) for _ in range(N)]
        stats = m.update(B, use_graph=False, idx_list=[i.to("cuda:0") for i in idx])
        res["stats"].append([(float(lq), float(la), q.cpu().squeeze(1), y.cpu()) for lq, la, q, y in stats])
        bs = []
        for i in idx:
            b = {k: v[i.long()].clone() for k, v in host.items()}
            b["done"] = b["done"].to(torch.float32)
            bs.append(b)
        res["batches"].append(bs)
    torch.cuda.synchronize()
    res["final"] = _att_state(m)
    res["flat"] = [m.fa.data.cpu(), m.fc.data.cpu(), m.fa_t.data.cpu(), m.fc_t.data.cpu()]
    # the segmented graph vs the eager launch list (device sampler, this rank's shard)
    ge, _, _ = _att_model(dist.group.WORLD, N, B, E, rank, seed=3)
    gg, _, _ = _att_model(dist.group.WORLD, N, B, E, rank, seed=3)
    for _ in range(3):
        ge.update(B, use_graph=False, want_stats=False)
        gg.update(B, use_graph=True, want_stats=False)
    torch.cuda.synchronize()
    res["n_segments"] = len(gg._graph[0]) if isinstance(gg._graph, tuple) else 0
    res["graph_equal"] = all(torch.equal(a, b) for a, b in ((ge.fa.data, gg.fa.data), (ge.fc.data, gg.fc.data),
                                                            (ge.fa_t.data, gg.fa_t.data), (ge.fc_t.data, gg.fc_t.data)))
    dist.destroy_process_group()
    return res


def _check_att(out):
    N, D0 = 5, 22
    actor, critic = learner_ref.RefActor([D0, 18, 6], 2), learner_ref.RefCritic([D0, 18, 6], N, 2)
    actor.load_state_dict(out[0]["init"][0])
    critic.load_state_dict(out[0]["init"][1])
    actor_t, critic_t = copy.deepcopy(actor), copy.deepcopy(critic)
    opts = (torch.optim.Adam(actor.parameters(), lr=1e-3, eps=EPS), torch.optim.Adam(critic.parameters(), lr=1e-3,
                                                                                     eps=EPS))
    tol = 1e-5
    for it in range(2):
        rstats, opts = learner_ref.ref_update_dp(actor, critic, actor_t, critic_t,
                                                 [out[r]["batches"][it] for r in range(2)], opts=opts)
        for r in range(2):
            for ag, ((lq, la, q, y), (rlq, rla, rq, ry)) in enumerate(zip(out[r]["stats"][it], rstats[r])):
                torch.testing.assert_close(q, rq.squeeze(1), rtol=tol, atol=tol, msg=f"Q it{it} rank{r} agent{ag}")
                torch.testing.assert_close(y, ry, rtol=tol, atol=tol, msg=f"target it{it} rank{r} agent{ag}")
                assert abs(lq - rlq) <= tol * max(1.0, abs(rlq)) and abs(la - rla) <= tol * max(1.0, abs(rla)), \
                    (it, r, ag, lq, rlq, la, rla)
    for mine, ref in zip(out[0]["final"], (actor.state_dict(), critic.state_dict(), actor_t.state_dict(),
                                           critic_t.state_dict())):
        for k in ref:
            d = float((mine[k] - ref[k]).abs().max())
            assert d <= tol, (k, d)


# --------------------------------------------------------------------------- GRU (config 4 learner)
def _gru_model(pg, N, B, E, rank, seed=1):
    from multi_agent_aac_amd.gru import MADDPG
    m = MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, device="cuda:0", seed=seed, batch_size=B,
               process_group=pg)
    rep = m.attach_replay(4 * E, seed=9 + rank)
    host = {k: [] for k in GRU_KEYS}
    for p in range(3):
        tr = gru_ref.random_gru_transitions(E, N, 50 + p + 1000 * rank)
        rep.push_batch(*[tr[k].to("cuda:0").contiguous() for k in GRU_KEYS])
        for k in GRU_KEYS:
            host[k].append(tr[k])
    return m, rep, {k: torch.cat(v) for k, v in host.items()}


def _gru_state(m):
    return [[_cpu(net[i].state_dict()) for i in range(m.n_agents)]
            for net in (m.actors, m.critics, m.actors_target, m.critics_target)]


def _work_gru(rank, ws, port):
    dist = _init(rank, ws, port)
    N, B, E = 4, 128, 256
    m, rep, host = _gru_model(dist.group.WORLD, N, B, E, rank)
    m.actor_optimizer.eps = m.critic_optimizer.eps = EPS
    res = {"init": _gru_state(m), "batches": [], "stats": [], "d_own": m.d_own}
    gen = np.random.default_rng(77 + rank)
    for _ in range(2):
        idx = torch.from_numpy(gen.choice(len(rep), size=B, replace=False).astype(np.int32))
        stats = m.update(B, use_graph=False, idx=idx.to("cuda:0"))
        res["stats"].append([(float(lq), float(la), q.cpu(), y.cpu()) for lq, la, q, y in stats])
        b = {k: v[idx.long()].clone() for k, v in host.items()}
        b["done"] = b["done"].float()
        res["batches"].append(b)
    torch.cuda.synchronize()
    res["final"] = _gru_state(m)
    res["flat"] = [m.fa.data.cpu(), m.fc.data.cpu(), m.fa_t.data.cpu(), m.fc_t.data.cpu()]
    ge, _, _ = _gru_model(dist.group.WORLD, N, B, E, rank, seed=3)
    gg, _, _ = _gru_model(dist.group.WORLD, N, B, E, rank, seed=3)
    for _ in range(3):
        ge.update(B, use_graph=False, want_stats=False)
        gg.update(B, use_graph=True, want_stats=False)
    torch.cuda.synchronize()
    res["n_segments"] = len(gg._graph[0])
    res["graph_equal"] = all(torch.equal(a, b) for a, b in ((ge.fa.data, gg.fa.data), (ge.fc.data, gg.fc.data),
                                                            (ge.fa_t.data, gg.fa_t.data), (ge.fc_t.data, gg.fc_t.data)))
    dist.destroy_process_group()
    return res


def _check_gru(out):
    N, d = 4, out[0]["d_own"]
    nets = []
    for k, cls in enumerate((gru_ref.RefGRUActor, gru_ref.RefGRUCritic)):
        ns = [cls([d, 18, 6], 2) for _ in range(N)]
        for i in range(N):
            ns[i].load_state_dict(out[0]["init"][k][i])
        nets.append(ns)
    actors, critics = nets
    actors_t, critics_t = copy.deepcopy(actors), copy.deepcopy(critics)
    opts = ([torch.optim.Adam(a.parameters(), lr=1e-3, eps=EPS) for a in actors],
            [torch.optim.Adam(c.parameters(), lr=1e-3, eps=EPS) for c in critics])
    for it in range(2):
        rstats, opts = gru_ref.ref_gru_update_dp(actors, critics, actors_t, critics_t,
                                                 [out[r]["batches"][it] for r in range(2)], d, opts=opts)
        for r in range(2):
            for ag, ((lq, la, q, y), (rlq, rla, rq, ry)) in enumerate(zip(out[r]["stats"][it], rstats[r])):
                assert float((y - ry).abs().max()) < 2e-5 * max(1.0, float(ry.abs().max())), ("target", it, r, ag)
                assert float((q - rq).abs().max()) < 2e-5 * max(1.0, float(rq.abs().max())), ("q", it, r, ag)
                assert abs(lq - rlq) <= 1e-4 * max(1.0, abs(rlq)) and abs(la - rla) <= 1e-4 * max(1.0, abs(rla)), \
                    (it, r, ag, lq, rlq, la, rla)
    for k, refs in enumerate((actors, critics, actors_t, critics_t)):
        for i in range(N):
            for name, rv in refs[i].state_dict().items():
                dv = float((out[0]["final"][k][i][name] - rv).abs().max())
                assert dv < 2e-5, (k, i, name, dv)


# --------------------------------------------------------------------------- UAM (config 5 learner)
def _uam_model(pg, N, B, E, rank, seed=1):
    from multi_agent_aac_amd import uam_learner as L
    m = L.MADDPG([7, 20, 18, 6], [7, 20, 18, 6], 2, n_agents=N, device="cuda:0", seed=seed, batch_size=B,
                 memory_length=4 * E * N, process_group=pg)
    rep = m.attach_replay(4 * E * N, seed=3 + rank)
    g = torch.Generator().manual_seed(5 + 1000 * rank)
    rnd = lambda *s: (torch.rand(*s, generator=g, dtype=torch.float64) * 2 - 1).to("cuda:0")   # noqa: E731
    for _ in range(3):
        rep.push_batch(rnd(E, N, 7), rnd(E, N, 18).abs().mul(5), rnd(E, N, 2), rnd(E, N).mul(50),
                       (rnd(E, N) > 0.8).double(), rnd(E, N, 7), rnd(E, N, 18).abs().mul(5))
    return m, rep


def _uam_state(m):
    return [_cpu(net.state_dict()) for net in (m.actors, m.critics, m.actors_target, m.critics_target)]


def _work_uam(rank, ws, port):
    from multi_agent_aac_amd import uam_learner as L
    dist = _init(rank, ws, port)
    N, B, E = 5, 128, 256
    m, rep = _uam_model(dist.group.WORLD, N, B, E, rank)
    res = {"init": _uam_state(m), "batches": [], "losses": []}
    gen = np.random.default_rng(77 + rank)
    for _ in range(2):
        idx = torch.as_tensor(gen.choice(len(rep), B, replace=False), dtype=torch.int32, device="cuda:0")
        lq, la = m.update(B, use_graph=False, idx=idx)
        res["losses"].append((float(lq), float(la)))
        rows = rep.ring[idx.long()].cpu()
        b = {k: rows[:, s:e].clone() for k, (s, e) in L.SLICES.items()}
        b["rew"], b["done"] = b["rew"][:, 0], b["done"][:, 0]
        res["batches"].append(b)
    torch.cuda.synchronize()
    res["final"] = _uam_state(m)
    fs = m._fstate
    res["flat"] = [fs["flat"].cpu(), fs["tflat"].cpu(), fs["m1"].cpu(), fs["m2"].cpu()]
    ge, _ = _uam_model(dist.group.WORLD, N, B, E, rank, seed=3)
    gg, _ = _uam_model(dist.group.WORLD, N, B, E, rank, seed=3)
    for _ in range(3):
        ge.update(B, use_graph=False)
        gg.update(B, use_graph=True)
    torch.cuda.synchronize()
    res["n_segments"] = len(gg._fu.graphs)
    a, b = ge._fstate, gg._fstate
    res["graph_equal"] = all(torch.equal(a[k], b[k]) for k in ("flat", "tflat", "m1", "m2"))
    dist.destroy_process_group()
    return res


def _check_uam(out):
    nets = [UR.RefActor().double(), UR.RefCritic().double()]
    for k in range(2):
        nets[k].load_state_dict(out[0]["init"][k])
    a, c = nets
    at, ct = copy.deepcopy(a), copy.deepcopy(c)
    oa, oc = torch.optim.Adam(a.parameters(), lr=1e-4), torch.optim.Adam(c.parameters(), lr=1e-4)
    for it in range(2):
        rl = UR.ref_update_dp(a, c, at, ct, oa, oc, [out[r]["batches"][it] for r in range(2)])
        for r in range(2):
            (lq, la), (rq, ra) = out[r]["losses"][it], rl[r]
            assert abs(lq - rq) < 1e-10 * max(1.0, abs(rq)) and abs(la - ra) < 1e-10 * max(1.0, abs(ra)), \
                (it, r, lq, rq, la, ra)
    for mine, ref in zip(out[0]["final"], (a.state_dict(), c.state_dict(), at.state_dict(), ct.state_dict())):
        for k in ref:
            np.testing.assert_allclose(mine[k].numpy(), ref[k].numpy(), rtol=0, atol=1e-10, err_msg=k)


# --------------------------------------------------------------------------- driver
WORK = {"att": _work_att, "gru": _work_gru, "uam": _work_uam}
CHECK = {"att": _check_att, "gru": _check_gru, "uam": _check_uam}
SEGMENTS = {"att": 7, "gru": None, "uam": 3}      # ATT: N + 1 all-reduces per update at N = 5


def _pack(res):
    """The result as bytes (torch.save): tensors put on a queue directly travel as shared file
    descriptors, which die with the worker process."""
    import io
    b = io.BytesIO()
    torch.save(res, b)
    return b.getvalue()


def _unpack(blob):
    import io
    return torch.load(io.BytesIO(blob), weights_only=True)


def _worker(rank, ws, port, q, kind, backend="gloo"):
    os.environ["AAC_TEST_BACKEND"] = backend
    if backend == "nccl":
        os.environ["HIP_VISIBLE_DEVICES"] = str(rank)      # before this process's first HIP call
    try:
        q.put((rank, _pack(WORK[kind](rank, ws, port))))
    except BaseException as e:      # report instead of leaving the peer blocked in a collective
        q.put((rank, _pack({"error": repr(e)})))
        raise


def _run_two(kind, backend="gloo"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, kind, backend)) for r in range(2)]
    for p in procs:
        p.start()
    out = {r: _unpack(b) for r, b in (q.get(timeout=240) for _ in procs)}
    for r in range(2):
        assert "error" not in out[r], out[r]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("kind", ["att", "gru", "uam"])
def test_two_rank_shards_match_mean_gradient_oracle(native_lib, kind):
    out = _run_two(kind)
    # the shards really differ (so a missing all-reduce could not pass) ...
    assert out[0]["batches"][0] is not None
    b0, b1 = out[0]["batches"][0], out[1]["batches"][0]
    first = (b0[0] if isinstance(b0, list) else b0)
    second = (b1[0] if isinstance(b1, list) else b1)
    key = "own" if kind == "uam" else "s_own"
    assert not torch.equal(first[key], second[key])
    # ... the ranks end bit-identical ...
    for x, y in zip(out[0]["flat"], out[1]["flat"]):
        assert torch.equal(x, y)
    # ... and equal to the restatement that applies the mean of the two ranks' gradients
    CHECK[kind](out)
    # the segmented graph replays exactly the eager launch list (collectives between segments)
    for r in range(2):
        assert out[r]["n_segments"] > 1 and (SEGMENTS[kind] is None or out[r]["n_segments"] == SEGMENTS[kind]), out[r][
            "n_segments"]
        assert out[r]["graph_equal"], r


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="two GPUs needed (one rank per GPU over RCCL)")
@pytest.mark.parametrize("kind", ["att", "gru", "uam"])
def test_two_rank_rccl_matches_mean_gradient_oracle(native_lib, kind):
    """the world > 1 default over RCCL -- two ranks on two GPUs, the all-reduces captured
    inside the update graph -- against the same mean-gradient restatement, ranks bit-identical, the
    one-graph replay equal to the eager launch list.  Skipped on one-GPU boxes (this pool's): there
    the captured-collective schedule is pinned by test_rccl_collectives_captured_in_graph (one rank)
    and the mean-gradient arithmetic by the gloo test above; AAC_GRAPH_COLL=0 is the fallback
    (segments with eager RCCL collectives)."""
    out = _run_two(kind, "nccl")
    for x, y in zip(out[0]["flat"], out[1]["flat"]):
        assert torch.equal(x, y)
    CHECK[kind](out)
    for r in range(2):
        assert out[r]["graph_equal"], r


def test_rccl_collectives_captured_in_graph(native_lib):
    """The default world > 1 path over RCCL (parallel.capturable): the update's all-reduces captured
    inside ONE graph end bit-identical to the 7 segments with eager RCCL all-reduces between them
    (a one-rank "nccl" group, world = 2 schedule; tools/seg_overhead.py), and the schedule's cost is
    reported."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "seg_overhead.py"), "--updates", "5"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["graph_rccl_graphs"] == 1 and out["graph_rccl_eager_collectives"] == 0, out
    assert out["seg_rccl_graphs"] == 7 and out["seg_rccl_eager_collectives"] == 6, out
    assert out["graph_equals_segmented"], out
