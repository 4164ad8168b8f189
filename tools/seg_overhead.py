"""Cost of the world > 1 update schedule, measured on one GPU.

At world > 1 the fused ATT update_myown has N + 1 = 6 gradient all-reduces (one per Adam boundary of
fused.FusedUpdate._merged).  One process, one GPU, the same update (N = 5, B = 1024, replay of
synthetic transitions) in five forms, each timed over K updates with HIP events on the launching
stream, every form through the product's own capture (MADDPG.update -> capture):
  one         world = 1: one graph (what bench.py runs at N = 1)
  graph_noop  world = 2 schedule, collectives no-ops, one graph (the schedule's own cost)
  graph_rccl  the same with a real RCCL all-reduce per boundary CAPTURED in the graph, on a one-rank
              "nccl" group (the collective's kernels; no xGMI traffic on one rank) -- the default
              world > 1 path (parallel.capturable)
  seg_noop    AAC_GRAPH_COLL=0: 7 graph segments, the collectives (no-ops) issued between replays
  seg_rccl    the same with real eager RCCL all-reduces
and check: graph_rccl and seg_rccl end bit-identical (parameters + optimiser state).
The differences x - one are per-update overheads; /6 is the per-boundary cost c_seg of DESIGN.md
section 6's model.  The 1 -> 8 GPU curve itself is the driver's round-end run.

python tools/seg_overhead.py [--updates 50]   (prints one JSON line)
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multi_agent_aac_amd import parallel  # noqa: E402
from multi_agent_aac_amd.maddpg import MADDPG  # noqa: E402


def fill(rep, N, D0, E=4096, pushes=4, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    K = N - 1
    for _ in range(pushes):
        r = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
        nei = r(E, N, K, 6) * 0.5
        rep.push_batch(r(E, N, D0), torch.rand(E, N, 18, device="cuda", generator=g) * 15, nei,
                       torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1, r(E, 1).repeat(1, N) * 5,
                       (torch.rand(E, N, device="cuda", generator=g) < 0.1).float(), r(E, N, D0),
                       torch.rand(E, N, 18, device="cuda", generator=g) * 15, r(E, N, K, 6) * 0.5)


def model(N, B, world, pg):
    D0 = 6 + 4 * (N - 1)
    m = MADDPG([D0, 18, 6], [D0, 18, 6], 2, n_agents=N, seed=777, batch_size=B, memory_length=100000)
    if world > 1:            # the world > 1 schedule on one process: gradients shared, segments captured
        m.world, m.pg = world, pg
        m._share_grads()
    rep = m.attach_replay(100000, seed=3)
    fill(rep, N, D0)
    return m


def time_updates(m, B, K):
    for _ in range(3):
        m.update(B, want_stats=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        m.update(B, want_stats=False)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


def state(m):
    return [t.clone() for t in [m.fa.data, m.fc.data, m.fa_t.data, m.fc_t.data]
            + m.actor_optimizer.state() + m.critic_optimizer.state()]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--updates", type=int, default=50)
    p.add_argument("--agents", type=int, default=5)
    p.add_argument("--batch", type=int, default=1024)
    a = p.parse_args()
    N, B, K = a.agents, a.batch, a.updates
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    pg = dist.new_group([0])
    out = {"agents": N, "batch": B, "updates": K}
    out["one_ms"] = time_updates(model(N, B, 1, None), B, K)
    noop = lambda t, group=None: t                                                          # noqa: E731
    rccl = lambda t, group=None: (dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg), t)[1]  # noqa: E731
    # (parallel.allreduce_sum_ skips a one-rank group: the forms below call RCCL themselves)
    real, graph_coll = parallel.allreduce_sum_, parallel.GRAPH_COLL
    final = {}
    for tag, cap, fn in (("graph_noop", True, noop), ("graph_rccl", True, rccl),
                         ("seg_noop", False, noop), ("seg_rccl", False, rccl)):
        parallel.allreduce_sum_, parallel.GRAPH_COLL = fn, cap
        m = model(N, B, 2, pg)
        out[tag + "_ms"] = time_updates(m, B, K)
        segs, colls = m._graph
        out[tag + "_graphs"], out[tag + "_eager_collectives"] = len(segs), len(colls)
        if tag.endswith("rccl"):
            torch.cuda.synchronize()
            final[tag] = state(m)
    parallel.allreduce_sum_, parallel.GRAPH_COLL = real, graph_coll
    out["graph_equals_segmented"] = all(torch.equal(x, y) for x, y in zip(final["graph_rccl"], final["seg_rccl"]))
    nb = N + 1
    for tag in ("graph_noop", "graph_rccl", "seg_noop", "seg_rccl"):
        out[tag + "_overhead_us"] = round(1e3 * (out[tag + "_ms"] - out["one_ms"]), 2)
    out["segmented_overhead_us"] = out["graph_rccl_overhead_us"]      # the default world > 1 path
    out["c_seg_us"] = round(out["graph_rccl_overhead_us"] / nb, 2)
    out["c_seg_eager_us"] = round(out["seg_rccl_overhead_us"] / nb, 2)
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
