"""Timing probe of the fused env step tail (aac_env_step_tail) against the separate launches, per part:
step only, step + push + reset as separate launches, the tail with push + reset, push only, reset only.
HIP events around the env part of one trainer step (median over steps).

python tools/tail_probe.py [--variant att|wgru] [--envs 4096] [--steps 30]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multi_agent_aac_amd import world  # noqa: E402
from multi_agent_aac_amd.env import BatchedEnv  # noqa: E402
from multi_agent_aac_amd.memory import DeviceReplay  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", default="att")
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--steps", type=int, default=30)
    a = p.parse_args()
    wgru = a.variant == "wgru"
    E, N = a.envs, (8 if wgru else 5)
    occ = world.synthetic_map(2026)
    bank = world.ODBank(occ, n_pairs=65536, seed=5, max_wp=32)
    env = BatchedEnv(E, N, occ, radar_mode=None if wgru else "combined", max_wp=32, variant=a.variant)
    env.set_od_bank(bank, seed=3)
    H = 64 if wgru else 0
    rep = DeviceReplay(100000, N, env.D0, hidden=H)
    bufs = [env.alloc_buffers(), env.alloc_buffers()]
    env.auto_reset(None, out=bufs[0])
    hid = [torch.zeros(E, N, H or 1, device="cuda") for _ in range(2)]
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1 for _ in range(8)]
    state = {"k": 0}

    def one(mode):
        k = state["k"]
        c, n = bufs[k], bufs[1 - k]
        act = acts[k % 8]
        srcs = [c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei] + ([hid[k], hid[1 - k]] if H else [])
        if mode == "step":
            env.step(act, out=n)
        elif mode == "sep":
            env.step(act, out=n)
            rep.push_batch(*srcs)
            env.auto_reset(n.env_done, out=n)
        elif mode == "tail":
            env.step_tail(act, out=n, replay=rep, srcs=srcs, zero_rows=hid[1 - k] if H else None)
        elif mode == "tail_push":
            env.step_tail(act, out=n, replay=rep, srcs=srcs, auto_reset=False)
        elif mode == "tail_reset":
            env.step_tail(act, out=n, auto_reset=True)
        state["k"] = 1 - k

    for mode in ("step", "sep", "tail", "tail_push", "tail_reset", "sep", "tail"):
        for _ in range(5):
            one(mode)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        dn = []
        for i in range(a.steps):
            ev[i][0].record()
            one(mode)
            ev[i][1].record()
            dn.append(bufs[state["k"]].env_done.sum())
        torch.cuda.synchronize()
        ms = sorted(x.elapsed_time(y) for x, y in ev)
        print(json.dumps({"variant": a.variant, "envs": E, "mode": mode, "median_ms": ms[len(ms) // 2],
                          "min_ms": ms[0], "done_per_step": float(torch.stack(dn).float().mean())}), flush=True)


if __name__ == "__main__":
    main()
