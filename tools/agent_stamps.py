"""Sub-phase timeline of the env step kernel's agent phase (thread 0 = agent 0 of the workgroup's
first env) from a stamp build with agent stamps:
  bash tools/variant_lib.sh astamps aac_env.hip -DAAC_ENV_STAMPS -DAAC_ENV_AGENT_STAMPS
  AAC_LIB=tools/vlib/lib_astamps.so python tools/agent_stamps.py [E] [N] [att|wgru]
Phases (cycles): observe_agent (obs rows + tdCPA), neighbour loops (collisions, penalty), building
cells, goal + bound predicates, reward + writes (WGRU: wgru_reward); with the step phases around them."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from multi_agent_aac_amd import _native, world
    from multi_agent_aac_amd.env import BatchedEnv
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    variant = sys.argv[3] if len(sys.argv) > 3 else "att"
    occ = world.synthetic_map(2026)
    env = BatchedEnv(E, N, occ, radar_mode=None if variant == "wgru" else "combined", max_wp=32, variant=variant)
    env.set_od_bank(world.ODBank(occ, n_pairs=16384, seed=5, max_wp=32), seed=3)
    env.auto_reset(None)
    g = torch.Generator(device="cuda").manual_seed(0)
    L = _native.lib()
    L.aac_env_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.aac_env_reset_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    epb_for = lambda apw: 1 if N > apw else apw // N                      # noqa: E731  (aac_env.hip policy)
    if E // epb_for(50) >= 1024:
        epb = epb_for(50)
    else:
        epb = epb_for(24)
        while epb < epb_for(50) and (E + epb - 1) // epb > 1024:
            epb += 1
    nwg = (E + epb - 1) // epb
    acc = {k: [] for k in ("kin", "radar", "agent", "final", "a_obs", "a_nei", "a_bld", "a_goal_bnd", "a_rew",
                           "a_wait")}
    for k in range(12):
        env.step(torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1)
        torch.cuda.synchronize()
        if k < 6:
            env.auto_reset(env.bufs.env_done)
            continue
        sb = np.zeros((nwg, 7), dtype=np.uint64)
        ab = np.zeros((nwg, 7), dtype=np.uint64)
        assert L.aac_env_stamps(sb.ctypes.data, nwg) == 0
        assert L.aac_env_reset_stamps(ab.ctypes.data, nwg) == 0
        s, a = sb.astype(np.int64), ab.astype(np.int64)
        ph = np.diff(s[:, 1:6], axis=1)
        ok = (a[:, 0] >= s[:, 3]) & (a[:, 5] <= s[:, 4])
        for name, col in zip(("kin", "radar", "agent", "final"), ph.T):
            acc[name] += col.tolist()
        sub = np.diff(a[ok, 0:6], axis=1)
        if variant == "wgru":      # stamp 6: after the next-waypoint search inside wgru_reward
            acc.setdefault("r_search", []).extend((a[ok, 6] - a[ok, 4]).tolist())
            acc.setdefault("r_cross_rest", []).extend((a[ok, 5] - a[ok, 6]).tolist())
        for name, col in zip(("a_obs", "a_nei", "a_bld", "a_goal_bnd", "a_rew"), sub.T):
            acc[name] += col.tolist()
        acc["a_wait"] += (s[ok, 4] - a[ok, 5]).tolist()     # after thread 0's agent to the barrier
        env.auto_reset(env.bufs.env_done)
    print(f"E={E} N={N}: {nwg} wg x {epb} envs")
    for name, v in acc.items():
        v = np.asarray(v)
        if v.size:
            print(f"  {name:10s} cycles median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  max {v.max():8.0f}")


if __name__ == "__main__":
    main()
