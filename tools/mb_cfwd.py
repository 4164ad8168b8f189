"""Microbenchmark of aac_critic_fwd and aac_actor_dcomb_out_bwd at the config-3 shapes (N = 5,
B = 1024; the target critic over N B = 5120 samples): python tools/mb_cfwd.py [reps].  Graph-replayed
launches, HIP events.  Env AAC_CF_* knobs pass through to the library."""
import json
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import fused  # noqa: E402


def graph_us(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
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


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev, N, B = "cuda", 5, 1024
    D0 = 6 + 4 * (N - 1)
    Din = D0 + 2
    P = fused.ptr
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g) * 0.2  # noqa: E731
    keep = []

    def net():
        t = dict(wenc=r(N, 128, Din), benc=r(N, 128), wc=r(256, 128 * N), bc=r(256), wq=r(256))
        keep.append(t)
        return SimpleNamespace(enc_w=[P(t["wenc"], n * 128 * Din) for n in range(N)],
                               enc_b=[P(t["benc"], n * 128) for n in range(N)], Wc=P(t["wc"]), bc=P(t["bc"]),
                               Wq=P(t["wq"]))

    def cset(Bs, fold, dual):
        cp = net()
        X, f, h, dh = r(Bs, N, Din), r(Bs, 128 * N), r(Bs, 256), r(Bs, 256)
        keep.extend([X, f, h, dh])
        fo = None
        if fold:
            ha, wa, ba = torch.relu(r(Bs * N, 256)), r(2, 256), r(2)
            keep.extend([ha, wa, ba])
            fo = (P(ha), SimpleNamespace(Wa=P(wa), ba=P(ba)), D0)
        return fused.critic_fwd_set(cp, P(X), Bs, N, Din, f, h, fold=fo, dual=(cp.Wq, dh, -1.0 / Bs) if dual else None)

    out = []
    cases = [("critic fwd B=1024 plain", [cset(B, False, False)]),
             ("critic fwd B=1024 fold+dual (actor step)", [cset(B, True, True)]),
             ("critic fwd actor step + critic step (2 sets)", [cset(B, True, True), cset(B, False, False)]),
             ("critic fwd target 5120 fold", [cset(N * B, True, False)]),
             ("critic fwd target + critic step 0", [cset(N * B, True, False), cset(B, False, False)])]
    for name, sets in cases:
        op = fused.CriticFwd(*sets)
        us = graph_us(op, reps)
        out.append({"launch": name, "us": round(us, 2), "tflops": round(op.flops / us / 1e6, 1)})
    dh, Wc, f = r(B, 256), r(256, 128 * N), torch.relu(r(B, 128 * N))
    wenc, X, wa, ha = r(N, 128, Din), r(B, N, Din), r(2, 256), torch.relu(r(B * N, 256))
    dout, dha = torch.empty(B * N, 2, device=dev), torch.empty(B * N, 256, device=dev)
    keep.extend([dh, Wc, f, wenc, X, wa, ha, dout, dha])
    a = fused.DaobArgs(P(dh), P(Wc), P(f), P(wenc), P(X), P(wa), P(ha), P(dout), P(dha), 128 * N, Din, D0, N, B)
    op = fused.DcombAob(a)
    us = graph_us(op, reps)
    out.append({"launch": "dcomb + actor out bwd", "us": round(us, 2), "tflops": round(op.flops / us / 1e6, 1)})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
