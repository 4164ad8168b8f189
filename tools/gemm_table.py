"""Per-launch table (graph-replayed) of the fused learner's grouped GEMM launches (config 3 by default): products,
FLOPs, isolated duration (each launch replayed 20x back to back after one full update), TF/s.

python tools/gemm_table.py [--agents 5] [--batch 1024] [--model att|gru]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--model", default="att")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--split", action="store_true", help="also time each product of a launch alone")
    a = ap.parse_args()
    from multi_agent_aac_amd.fused import GemmLaunch
    N, B = a.agents, a.batch
    D0 = 6 + 4 * (N - 1)
    if a.model == "gru":
        from multi_agent_aac_amd.gru import MADDPG
        m = MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, device="cuda", seed=1, batch_size=B)
        rep = m.attach_replay(8192, seed=1)
        for p in range(2):
            rep.push_batch(*synth.transitions(4096, N, p, D0=6, H=64))
        fu = m._plan(B)
        ops = fu.ops()
    else:
        from multi_agent_aac_amd.maddpg import MADDPG
        m = MADDPG([D0, 18, 6], [D0, 18, 6], 2, n_agents=N, device="cuda", seed=1, batch_size=B)
        rep = m.attach_replay(8192, seed=1)
        for p in range(2):
            rep.push_batch(*synth.transitions(4096, N, p))
        fu = m._fused_plan(B)
        ops = fu.ops()
    for op in ops:
        op()
    torch.cuda.synchronize()
    tot_t, tot_f = 0.0, 0.0
    rows = []

    def timed(op):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        op()
        g = torch.cuda.CUDAGraph()        # device time, no host launch cost (as in the bench's replay)
        with torch.cuda.graph(g):
            for _ in range(a.reps):
                op()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    def shape(p, cfg):
        mode = "" if not cfg else f"[L{(cfg - 1) >> 2}{(cfg - 1) & 3}]"
        return (f"{p.M}x{p.N - p.ones}{'+1' if p.ones else ''}x{p.K}{'/' + str(p.ksplit) if p.ksplit > 1 else ''}"
                f"{'T' if p.ta else ''}{'t' if p.tb else ''}{mode}")
    for k, op in enumerate(ops):
        if not isinstance(op, GemmLaunch):
            continue
        us = timed(op)
        cfgs, wg = op.plan()
        shapes = " ".join(shape(p, c) for p, c in zip(op.arr, cfgs))
        rows.append((us, op.flops, k, shapes + f"  ({wg} wg)"))
        tot_t += us
        tot_f += op.flops
        if a.split and op.n > 1:
            for p in op.arr:
                one = GemmLaunch([p])
                print(f"      {k:3d} alone {timed(one):7.1f} us {one.flops / 1e9:6.3f} GF  {shape(p, one.plan()[0][0])}")
    for us, fl, k, shapes in rows:
        print(f"{k:3d} {us:7.1f} us {fl / 1e9:6.3f} GF {fl / us / 1e6:6.1f} TF/s  {shapes}")
    print(f"total {tot_t:.1f} us over {len(rows)} launches, {tot_f / 1e9:.2f} GF, {tot_f / tot_t / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
