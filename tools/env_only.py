"""Env-only driver (no learner): E x N envs stepping on pre-generated actions with GPU auto-reset.
Used for PMC (rocprofv3 --pmc) traffic runs and per-radar-mode timing of the fused env kernel.

python tools/env_only.py [--envs 4096] [--agents 5] [--radar combined] [--steps 20]
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


def run(E, N, radar, steps, reset=True):
    occ = world.synthetic_map(2026)
    bank = world.ODBank(occ, n_pairs=65536, seed=5, max_wp=32)
    env = BatchedEnv(E, N, occ, radar_mode=radar, max_wp=32)
    env.set_od_bank(bank, seed=3)
    env.auto_reset(None)
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1 for _ in range(8)]
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for i in range(steps):
        ev[i][0].record()
        env.step(acts[i % 8])
        ev[i][1].record()
        if reset:
            env.auto_reset(env.bufs.env_done)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev[2:])
    return {"envs": E, "agents": N, "radar": radar, "median_step_kernel_ms": ms[len(ms) // 2],
            "agent_env_steps_per_s": E * N / (ms[len(ms) // 2] * 1e-3)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--agents", type=int, default=5)
    p.add_argument("--radar", default="combined")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--sweep", action="store_true", help="time every radar mode at several E")
    a = p.parse_args()
    if a.sweep:
        for E in (4096, 65536, 262144):
            for radar in ("drones", "obstacles", "combined"):
                print(json.dumps(run(E, a.agents, radar, 12)), flush=True)
    else:
        print(json.dumps(run(a.envs, a.agents, a.radar, a.steps)), flush=True)


if __name__ == "__main__":
    main()
