"""Do independent branches of a captured HIP graph run concurrently on this stack?

Two chains of 12 latency-bound GEMM launches (the critic combine shape, M=1024 N=256 K=640) are
captured (a) back to back on one stream, (b) on two streams forked/joined with events; the replay
times are compared.  python tools/graph_branch_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import fused  # noqa: E402


def main():
    dev = "cuda"
    M, N, K, L = 1024, 256, 640, 12
    bufs = []
    for _ in range(2):
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        C = torch.empty(M, N, device=dev)
        bufs.append([fused.GemmLaunch([fused.prob(fused.ptr(A), fused.ptr(W), fused.ptr(C), M, N, K, K, K, N, tb=1,
                                                  act=1)]) for _ in range(L)] + [A, W, C])
    chains = [b[:L] for b in bufs]

    def run_serial():
        for ch in chains:
            for op in ch:
                op()

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run_forked():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            for op in chains[0]:
                op()
        with torch.cuda.stream(s2):
            for op in chains[1]:
                op()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    out = {}
    for name, fn in (("serial", run_serial), ("forked", run_forked)):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fn()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_graph_us"] = e0.elapsed_time(e1) / 20 * 1e3
        # eager (no graph) for reference
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_eager_us"] = e0.elapsed_time(e1) / 20 * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
