"""Per-product split-K counts of the actor step's weight-gradient launches (config 3, N = 5, B = 1024),
graph-replayed: each weight-gradient product alone at several split counts (<= the copies Adam sums:
a product with fewer splits leaves its other copies zero), then the launches with the best ones.

python tools/mb_split.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from multi_agent_aac_amd.fused import AttnBwd, GemmLaunch, GemmProb
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B = 5, 1024
    D0 = 6 + 4 * (N - 1)
    m = MADDPG([D0, 18, 6], [D0, 18, 6], 2, n_agents=N, device="cuda", seed=1, batch_size=B)
    rep = m.attach_replay(8192, seed=1)
    for p in range(2):
        rep.push_batch(*synth.transitions(4096, N, p))
    fu = m._fused_plan(B)
    ops = fu.ops()
    for op in ops:
        op()
    torch.cuda.synchronize()

    def timed(fn):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    def with_split(p, s):
        q = GemmProb.from_buffer_copy(p)
        q.ksplit = s
        return q

    def name(p):
        return f"{p.M}x{p.N}x{p.K}/{p.ksplit}"

    # the last full iteration's wgrad1 / wgrad2
    idx = [k for k, op in enumerate(ops) if isinstance(op, GemmLaunch) and
           any(p.M == 5120 and p.N == 64 and p.K == 256 for p in op.arr[:op.n])]
    k = idx[-2]
    w1 = ops[k]
    j = k + 1
    while not isinstance(ops[j], AttnBwd):
        j += 1
    w2 = ops[j + 1]
    p1, p2 = list(w1.arr[:w1.n]), list(w2.arr[:w2.n])
    for p in p1 + p2:
        if p.ksplit > 1:
            res = [(s, timed(GemmLaunch([with_split(p, s)]))) for s in (1, 2, 4, 5, 8, 10, 16, 20) if s <= p.ksplit]
            print(name(p), " ".join(f"{s}:{t:.1f}" for s, t in res), flush=True)
    dwm = [p for p in p1 if p.M == 256 and p.N == 193][0]
    dwa = [p for p in p1 if p.M == 2][0]
    data = [p for p in p1 if p.M == 5120]
    for s in (4, 5, 8, 10, 16, 20):
        for sa in (2, 4, 20):
            w = [with_split(dwm, s), with_split(dwa, sa)]
            print(f"dWm/{s} dWa/{sa}: wgrad1 {timed(GemmLaunch(w + data)):.1f}  weights {timed(GemmLaunch(w)):.1f}  "
                  f"wgrad2+weights {timed(GemmLaunch(p2 + w)):.1f} us", flush=True)
    print(f"wgrad1 {timed(w1):.1f}  wgrad2 {timed(w2):.1f}")


if __name__ == "__main__":
    main()
