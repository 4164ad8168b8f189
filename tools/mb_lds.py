"""Isolated timings (graph-replayed, device time) of the config-3 learner's large GEMM shapes, one
product per launch, with the plan each gets.  Knobs are read when the library loads, so compare
configurations in separate processes:
    AAC_GEMM_LDS=0 python tools/mb_lds.py      (register-fragment path)
    AAC_GEMM_LDS_MIN_WG=256 python tools/mb_lds.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # M, N, K, ta, tb, ones, ksplit
    (25600, 256, 192, 0, 1, 0, 1),
    (5120, 256, 640, 0, 1, 0, 1),
    (5120, 256, 192, 0, 1, 0, 1),
    (1024, 640, 256, 0, 0, 0, 1),
    (1024, 256, 640, 0, 1, 0, 1),
    (5120, 64, 256, 0, 0, 0, 1),
    (256, 192, 5120, 1, 0, 1, 32),
    (256, 640, 1024, 1, 0, 1, 8),
    (64, 64, 5120, 1, 0, 0, 32),
]


def main(reps=20):
    from multi_agent_aac_amd import fused
    only = int(sys.argv[1]) if len(sys.argv) > 1 else None       # python tools/mb_lds.py 0: shape 0 only
    tot = 0.0
    for idx, (M, N, K, ta, tb, ones, ks) in enumerate(SHAPES):
        if only is not None and idx != only:
            continue
        A = torch.randn(K, M, device="cuda") if ta else torch.randn(M, K, device="cuda")
        B = torch.randn(N, K, device="cuda") if tb else torch.randn(K, N, device="cuda")
        # [ks][stride] partial copies, each with its cextra column block after the M x N product
        stride = M * N + M
        C = torch.empty(ks * stride, device="cuda")
        p = fused.prob(fused.ptr(A), fused.ptr(B), fused.ptr(C), M, N, K, A.shape[1], B.shape[1], N, ta=ta, tb=tb,
                       ones=ones, cextra=fused.ptr(C, M * N) if ones else None, ksplit=ks,
                       split_stride=stride if ks > 1 else 0)
        op = fused.GemmLaunch([p])
        op()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                op()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        tot += us
        cfg, wg = op.plan()
        print(f"{M}x{N}{'+1' if ones else ''}x{K}/{ks}{'T' if ta else ''}{'t' if tb else ''}: {us:7.2f} us "
              f"{op.flops / us / 1e6:6.1f} TF/s  plan {cfg[0]} ({wg} wg)", flush=True)
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
