"""Microbenchmark of aac_attn_enc_fwd (actor encoders + attention, riding critic encoders) at the
config-3 shapes (N = 5, B = 1024, E = 4096): python tools/mb_attn_enc.py [reps].  Graph-replayed
launches, HIP events; AAC_LIB picks the library (A/B against a variant build)."""
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
    dev, N, K, B, D0 = "cuda", 5, 4, 1024, 22
    Din = D0 + 2
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g) * 0.2  # noqa: E731
    P = fused.ptr
    W = {"Wo": r(64, D0), "bo": r(64), "Wg": r(64, 18), "bg": r(64), "Wn": r(64, 6), "bn": r(64), "Wq": r(64, 64)}
    kv = r(128, 64)
    ap = SimpleNamespace(**{k: P(v) for k, v in W.items()}, Wkv=P(kv))
    cw, cb = r(N, 128, Din), r(N, 128)
    cp = SimpleNamespace(enc_w=[P(cw, n * 128 * Din) for n in range(N)], enc_b=[P(cb, n * 128) for n in range(N)])

    def actor_set(R, train, ride=None):
        own, radar, nei, cat = r(R, Din), r(R, 18), r(R, K, 6), torch.empty(R, 192, device=dev)
        acts = fused.ActorActs(R, K, dev) if train else None
        keep.append((own, radar, nei, cat, acts))
        return fused.attn_set(ap, P(own), Din, D0, P(radar), P(nei), R, K, P(cat), acts=acts, ride=ride)

    def ride(rows):
        X, f = r(rows, N, Din), torch.empty(rows, N * 128, device=dev)
        keep.append((X, f))
        return fused.critic_enc_ride(cp, P(X), rows, N, Din, f)

    def gemm_cenc(rows):
        X, f = r(rows, N, Din), torch.empty(rows, N * 128, device=dev)
        keep.append((X, f))
        return fused.GemmLaunch([fused.prob(P(X, n * Din), cp.enc_w[n], P(f, n * 128), rows, 128, Din, N * Din, Din,
                                            128 * N, tb=1, bias=cp.enc_b[n], act=fused.RELU) for n in range(N)])

    def ride_fold(rows):
        """the target critic's encoders with the target actor's output layer folded in (ha rows)"""
        X, f = r(rows, N, Din), torch.empty(rows, N * 128, device=dev)
        ha = torch.relu(r(rows * N, 256))
        wa, ba = r(2, 256), r(2)
        keep.append((X, f, ha, wa, ba))
        return fused.critic_enc_ride(cp, P(X), rows, N, Din, f, fold=(P(ha), SimpleNamespace(Wa=P(wa), ba=P(ba)), D0))

    keep = []
    cases = [("target+ride | train (pre)", 1, fused.AttnEnc(actor_set(25 * B, False, ride(B)), actor_set(N * B, True))),
             ("train+ride (iteration)", 4, fused.AttnEnc(actor_set(N * B, True, ride(B)))),
             ("train (last iteration)", 1, fused.AttnEnc(actor_set(N * B, True))),
             ("ride only (actor-step critic)", 4, fused.AttnEnc(fused.ride_only(ride(B)))),
             ("ride pair (iteration 0)", 1, fused.AttnEnc(fused.ride_only(ride(B)), fused.ride_only(ride(B)))),
             ("act inference E*N rows", 1, fused.AttnEnc(actor_set(4096 * N, False))),
             ("target critic ride + folded output layer", 1, fused.AttnEnc(fused.ride_only(ride_fold(5 * B))))]
    if os.environ.get("MB_SWEEP"):
        cases = [(f"ride only rows={rows}", 0, fused.AttnEnc(fused.ride_only(ride(rows)))) for rows in (16, 256, 1024, 4096)]
        cases += [(f"train R={R}", 0, fused.AttnEnc(actor_set(R, True))) for R in (16, 1024, 5120, 20480)]
        cases += [(f"gemm cenc rows={rows}", 0, gemm_cenc(rows)) for rows in (16, 1024)]
    tot = 0.0
    for name, cnt, fn in cases:
        us = graph_us(fn, reps)
        tot += us * cnt
        print(json.dumps({"launch": name, "us": round(us, 2), "per_step": cnt}), flush=True)
    print(json.dumps({"attn_enc_us_per_step": round(tot, 1), "lib": os.environ.get("AAC_LIB", "in-tree")}), flush=True)


if __name__ == "__main__":
    main()
