"""Microbenchmark: weight-gradient GEMM dW = G^T X for the learner's shapes, several strategies."""
import sys
import time

import torch

SHAPES = [  # (M rows, in, out) at B=1024, N=5, K=4
    (20480, 6, 64), (20480, 64, 128), (5120, 22, 64), (5120, 18, 64), (5120, 64, 64), (5120, 192, 256),
    (5120, 256, 2), (5120, 24, 128), (1024, 640, 256), (1024, 256, 1)]


def bench(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else "default"
    if lib != "default":
        torch.backends.cuda.preferred_blas_library(lib)
    print("blas", torch.backends.cuda.preferred_blas_library())
    tot = {}
    for M, I, O in SHAPES:
        x = torch.randn(M, I, device="cuda")
        g = torch.randn(M, O, device="cuda")
        out = torch.empty(O, I, device="cuda")
        r = {}
        r["mm_gT_x"] = bench(lambda: torch.mm(g.t(), x, out=out))
        for S in (8, 16, 32):
            if M % S == 0:
                gs = g.view(S, M // S, O)
                xs = x.view(S, M // S, I)
                part = torch.empty(S, O, I, device="cuda")
                r[f"bmm{S}+sum"] = bench(lambda: torch.sum(torch.bmm(gs.transpose(1, 2), xs, out=part), 0, out=out))
        r["mm_xT_g"] = bench(lambda: torch.mm(x.t(), g))
        print(f"M={M:6d} in={I:4d} out={O:4d} " + " ".join(f"{k}={v:7.1f}us" for k, v in r.items()))
        for k, v in r.items():
            tot[k] = tot.get(k, 0) + v
    print("totals", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
