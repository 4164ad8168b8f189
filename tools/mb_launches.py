"""Microbenchmark of the learner's grouped-GEMM launches as they occur in one bench step at
N = 5, E = 4096, B = 1024 (product groups taken from an AAC_GEMM_DUMP run of bench.py).

python tools/mb_launches.py [reps]  ->  one line per distinct launch (us, TF/s) and the GEMM time
per bench step (each launch weighted by how often it runs per step).  Tuning knobs are the
AAC_GEMM_* environment variables read by libaac_env.so at load.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import fused  # noqa: E402

# (name, per-step count, [(M, N, K, ta, tb, ones, ksplit, act, mact, addend)])
ENC = (1024, 128, 24, 0, 1, 0, 1, 1, 0, 0)
LAUNCHES = [
    ("act_enc", 1, [(20480, 64, 22, 0, 1, 0, 1, 1, 0, 0), (20480, 64, 18, 0, 1, 0, 1, 1, 0, 0),
                    (64, 64, 64, 1, 0, 0, 1, 0, 0, 0)]),
    ("act_merge", 1, [(20480, 256, 192, 0, 1, 0, 1, 1, 0, 0)]),
    ("act_out", 1, [(20480, 2, 256, 0, 1, 0, 1, 2, 0, 0)]),
    ("tgt_enc", 1, [(25600, 64, 22, 0, 1, 0, 1, 1, 0, 0), (25600, 64, 18, 0, 1, 0, 1, 1, 0, 0),
                    (64, 64, 64, 1, 0, 0, 1, 0, 0, 0)]),
    ("tgt_merge", 1, [(25600, 256, 192, 0, 1, 0, 1, 1, 0, 0)]),
    ("tgt_out", 1, [(25600, 2, 256, 0, 1, 0, 1, 2, 0, 0)]),
    ("tgt_cenc", 1, [(5120, 128, 24, 0, 1, 0, 1, 1, 0, 0)] * 5),
    ("tgt_comb", 1, [(5120, 256, 640, 0, 1, 0, 1, 1, 0, 0)]),
    ("it_enc", 5, [ENC] * 5 + [(5120, 64, 22, 0, 1, 0, 1, 1, 0, 0), (5120, 64, 18, 0, 1, 0, 1, 1, 0, 0),
                               (20480, 64, 6, 0, 1, 0, 1, 1, 0, 0)]),
    ("it_comb", 10, [(1024, 256, 640, 0, 1, 0, 1, 1, 0, 0)]),
    ("it_cgrad", 5, [(1, 257, 1024, 1, 0, 1, 8, 0, 0, 0), (256, 641, 1024, 1, 0, 1, 8, 0, 0, 0),
                     (1024, 640, 256, 0, 0, 0, 1, 0, 1, 0), (5120, 256, 192, 0, 1, 0, 1, 1, 0, 0)]),
    ("it_encgrad", 5, [(128, 25, 1024, 1, 0, 1, 8, 0, 0, 0)] * 5 + [(5120, 2, 256, 0, 1, 0, 1, 2, 0, 0)]),
    ("it_cenc2", 5, [ENC] * 5),
    ("it_df", 5, [(1024, 640, 256, 0, 0, 0, 1, 0, 1, 0)]),
    ("it_agrad1", 5, [(2, 257, 5120, 1, 0, 1, 32, 0, 0, 0), (256, 193, 5120, 1, 0, 1, 32, 0, 0, 0),
                      (5120, 64, 256, 0, 0, 0, 1, 0, 0, 0), (5120, 64, 256, 0, 0, 0, 1, 0, 1, 0),
                      (5120, 64, 256, 0, 0, 0, 1, 0, 0, 0)]),
    ("it_agrad2", 5, [(64, 64, 5120, 1, 0, 0, 32, 0, 0, 0)] * 3 +
                     [(64, 7, 20480, 1, 0, 1, 32, 0, 0, 0), (64, 23, 5120, 1, 0, 1, 32, 0, 0, 0),
                      (64, 19, 5120, 1, 0, 1, 32, 0, 0, 0)]),
]


def build(spec, dev, keep):
    probs, fl = [], 0.0
    for M, N, K, ta, tb, ones, ks, act, mact, add in spec:
        nr = N - ones
        A = torch.randn(K * M, device=dev)
        B = torch.randn(K * max(nr, 1), device=dev)
        stride = M * nr + M
        C = torch.empty(ks * stride, device=dev)
        bias = torch.randn(max(nr, 1), device=dev) if act else None
        mask = torch.randn(M * max(nr, 1), device=dev) if mact else None
        addt = torch.randn(M * max(nr, 1), device=dev) if add else None
        keep += [A, B, C, bias, mask, addt]
        P = fused.ptr
        probs.append(fused.prob(P(A), P(B), P(C), M, nr, K, M if ta else K, K if tb else max(nr, 1), max(nr, 1),
                                ta=ta, tb=tb, act=act, bias=P(bias) if bias is not None else None,
                                mask=P(mask) if mask is not None else None, mact=mact, ldmask=max(nr, 1),
                                addend=P(addt) if addt is not None else None, ldadd=max(nr, 1), ones=ones,
                                cextra=P(C, M * nr) if ones else None, ksplit=ks,
                                split_stride=stride if ks > 1 else 0))
        fl += 2.0 * M * N * K
    return fused.GemmLaunch(probs), fl


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    dev = "cuda"
    keep, total, tot_fl = [], 0.0, 0.0
    knobs = {k: v for k, v in os.environ.items() if k.startswith("AAC_GEMM")}
    for name, count, spec in LAUNCHES:
        launch, fl = build(spec, dev, keep)
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        # replay a captured graph of `reps` launches: GPU time, not the host's launch rate
        graph, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                for _ in range(reps):
                    launch()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        total += us * count
        tot_fl += fl * count
        print(json.dumps({"launch": name, "us": round(us, 2), "MFLOP": round(fl / 1e6), "TFs": round(fl / us / 1e6, 1),
                          "per_step": count}), flush=True)
    print(json.dumps({"knobs": knobs, "gemm_us_per_step": round(total, 1), "GFLOP_per_step": round(tot_fl / 1e9, 2),
                      "TFs": round(tot_fl / total / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
