"""Cost of the world > 1 update schedule, measured on one GPU.

At world > 1 the fused ATT update_myown runs as N + 2 = 7 captured graph segments with N + 1 = 6
gradient all-reduces between them (fused.FusedUpdate._pipelined).  One process, one GPU, three forms
of the same update (N = 5, B = 1024, replay of synthetic transitions), each timed over K updates with
HIP events on the launching stream:
  one      world = 1: the merged schedule, one graph (what bench.py runs at N = 1)
  seg_noop the pipelined schedule's 7 graph segments, the collectives replaced by no-ops
  seg_rccl the same with a real RCCL all-reduce per boundary on a one-rank "nccl" process group (the
           collective's launch and its kernel; no xGMI traffic on one rank)
  pipe_one the pipelined schedule's launches (no-op collectives) as ONE graph: separates the cost of the
           schedule itself from the cost of cutting it into segments
  pipe_rccl_one  the same with the RCCL all-reduces captured inside the one graph
The difference seg_* - one is the schedule's overhead per update (the 1 -> 8 GPU curve itself is the
driver's round-end run); /6 is the per-boundary cost c_seg of DESIGN.md section 6's model.

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
    real = parallel.allreduce_sum_
    parallel.allreduce_sum_ = lambda t, group=None: t                              # no-op collectives
    m = model(N, B, 2, pg)
    out["seg_noop_ms"] = time_updates(m, B, K)
    segs, colls = m._graph if isinstance(m._graph, tuple) else ([], [])
    out["segments"], out["collectives"] = len(segs), len(colls)
    parallel.allreduce_sum_ = lambda t, group=None: (dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg), t)[1]
    out["seg_rccl_ms"] = time_updates(model(N, B, 2, pg), B, K)
    for tag, fn in (("pipe_one_ms", lambda t, group=None: t),
                    ("pipe_rccl_one_ms", lambda t, group=None: (dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg), t)[1])):
        parallel.allreduce_sum_ = fn
        m = model(N, B, 2, pg)
        m.update(B, want_stats=False)        # builds the plan (eager warm-up of every launch)
        fu = m._fused_plan(B)
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for op in fu.ops():
                    op()
            torch.cuda.synchronize()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            out[tag] = e0.elapsed_time(e1) / K
        except Exception as ex:       # capture of the collective not supported
            out[tag] = f"failed: {type(ex).__name__}: {ex}"[:200]
    parallel.allreduce_sum_ = real
    nb = max(out["collectives"], 1)
    out["segmented_overhead_us"] = round(1e3 * (out["seg_noop_ms"] - out["one_ms"]), 2)
    out["segmented_rccl_overhead_us"] = round(1e3 * (out["seg_rccl_ms"] - out["one_ms"]), 2)
    out["c_seg_us"] = round(1e3 * (out["seg_noop_ms"] - out["one_ms"]) / nb, 2)
    out["c_seg_rccl_us"] = round(1e3 * (out["seg_rccl_ms"] - out["one_ms"]) / nb, 2)
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
