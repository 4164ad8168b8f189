"""Microbenchmark of the config-5 act launch (aac_uam_actor: 8192 envs x 16 aircraft, float64
weights-stationary actor + exploration noise), graph-replayed, with and without the noise:
python tools/mb_uam_actor.py [reps].  AAC_LIB picks the library (A/B against a variant build)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_us(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
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


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from multi_agent_aac_amd import uam_learner
    E, N = 8192, 16
    dims = [7, (N - 1) * 5, 18, 6]
    m = uam_learner.MADDPG(dims, dims, 2, n_agents=N, seed=777, batch_size=512, memory_length=1 << 16)
    g = torch.Generator(device="cuda").manual_seed(0)
    own = torch.rand(E, N, 7, device="cuda", dtype=torch.float64, generator=g) * 2 - 1
    radar = torch.rand(E, N, 18, device="cuda", dtype=torch.float64, generator=g)
    ep = torch.ones(E, dtype=torch.int32, device="cuda")
    res = {}
    for noisy in (True, False):
        res["noisy" if noisy else "plain"] = round(graph_us(lambda: m.act(own, radar, ep, noisy=noisy), reps), 2)
    print(json.dumps({"uam_actor_us": res, "lib": os.environ.get("AAC_LIB", "in-tree")}), flush=True)


if __name__ == "__main__":
    main()
