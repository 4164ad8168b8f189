"""What moving the actor step's data gradients out of the first weight-gradient launch would buy
(config 3, N = 5, B = 1024): graph-replayed times of the wgrad1 launch (dWa | dWm weight gradients +
the three 5120 x 64 x 256 data gradients), of its two halves alone, of the wgrad2 launch, and of wgrad2
with dWa | dWm added, plus the attention backward.

python tools/mb_regroup.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from multi_agent_aac_amd.fused import AttnBwd, GemmLaunch
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

    k = 0
    while k < len(ops):
        op = ops[k]
        if isinstance(op, GemmLaunch) and any(p.M == 5120 and p.N == 64 and p.K == 256 for p in op.arr[:op.n]):
            w1 = op
            j = k + 1
            while not isinstance(ops[j], AttnBwd):
                j += 1
            bwd = ops[j]
            w2 = ops[j + 1]
            data = [p for p in w1.arr[:w1.n] if p.M == 5120 and p.N == 64]
            wts = [p for p in w1.arr[:w1.n] if not (p.M == 5120 and p.N == 64)]
            w2p = list(w2.arr[:w2.n])
            res = {"wgrad1": timed(w1), "wgrad1_data_only": timed(GemmLaunch(data)),
                   "wgrad1_weights_only": timed(GemmLaunch(wts)), "attn_bwd": timed(bwd), "wgrad2": timed(w2)}
            if len(w2p) + len(wts) <= 16:
                res["wgrad2_plus_weights"] = timed(GemmLaunch(w2p + wts))
            print(f"launch {k}: " + "  ".join(f"{a} {b:.1f} us" for a, b in res.items()), flush=True)
            k = j + 2
        else:
            k += 1


if __name__ == "__main__":
    main()
