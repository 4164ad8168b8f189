"""Microbenchmark of aac_gemm_batch on the learner's product shapes vs torch (hipBLASLt / rocBLAS).

python tools/mb_gemm.py  ->  one JSON line per shape: our us/launch, torch us, TF/s
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import fused  # noqa: E402

SHAPES = [  # name, M, N, K, ta, tb, ones, ksplit, act
    ("kv_fwd", 20480, 128, 64, 0, 1, 0, 1, 0),
    ("merge_fwd", 5120, 256, 192, 0, 1, 0, 1, 1),
    ("merge_fwd_t", 25600, 256, 192, 0, 1, 0, 1, 1),
    ("combine_fwd", 1024, 256, 640, 0, 1, 0, 1, 1),
    ("combine_fwd_t", 5120, 256, 640, 0, 1, 0, 1, 1),
    ("dcat", 5120, 64, 256, 0, 0, 0, 1, 0),
    ("df", 1024, 640, 256, 0, 0, 0, 1, 0),
    ("dWm", 256, 192, 5120, 1, 0, 1, 32, 0),
    ("dWc", 256, 640, 1024, 1, 0, 1, 8, 0),
    ("dWkv", 128, 64, 20480, 1, 0, 0, 32, 0),
]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = "cuda"
    for name, M, N, K, ta, tb, ones, ks, act in SHAPES:
        A = torch.randn(K, M, device=dev) if ta else torch.randn(M, K, device=dev)
        B = torch.randn(N, K, device=dev) if tb else torch.randn(K, N, device=dev)
        C = torch.empty(ks, M * N + M, device=dev)
        P = fused.ptr
        p = fused.prob(P(A), P(B), P(C), M, N, K, A.shape[1], B.shape[1], N, ta=ta, tb=tb, act=act, ones=ones,
                       cextra=P(C, M * N) if ones else None, ksplit=ks, split_stride=M * N + M if ks > 1 else 0)
        launch = fused.GemmLaunch([p])
        ours = timeit(launch)
        a = A.t() if ta else A
        b = B.t() if tb else B
        theirs = timeit(lambda: torch.mm(a, b))
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "ours_us": round(ours, 2),
                          "torch_us": round(theirs, 2), "ours_TFs": round(fl / ours / 1e6, 1),
                          "torch_TFs": round(fl / theirs / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
