"""Per-workgroup phase timeline of the fused env step tail (aac_env_step_tail: step + replay push +
auto-reset) in a steady training-like loop, from a stamp build (bash tools/variant_lib.sh estamps
aac_env.hip -DAAC_ENV_STAMPS; AAC_LIB=ablibs/lib_estamps.so).

python tools/tail_stamps.py [att|wgru]

Step phases (cycles): kinematics, radar, agent, then for the workgroups that reset an env: final +
zero rows + OD draw, waypoint copy + state writes, reset radar, reset observation; the rest: final."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from multi_agent_aac_amd import _native, world
    from multi_agent_aac_amd.env import BatchedEnv
    from multi_agent_aac_amd.memory import DeviceReplay
    kind = sys.argv[1] if len(sys.argv) > 1 else "att"
    wgru = kind == "wgru"
    E, N = (4096, 8) if wgru else (4096, 5)
    occ = world.synthetic_map(2026)
    env = BatchedEnv(E, N, occ, radar_mode=None if wgru else "combined", max_wp=32, variant=kind)
    env.set_od_bank(world.ODBank(occ, n_pairs=65536, seed=5, max_wp=32), seed=3)
    H = 64 if wgru else 0
    rep = DeviceReplay(100000, N, env.D0, hidden=H)
    bufs = [env.alloc_buffers(), env.alloc_buffers()]
    env.auto_reset(None, out=bufs[0])
    hid = [torch.zeros(E, N, H or 1, device="cuda") for _ in range(2)]
    g = torch.Generator(device="cuda").manual_seed(0)
    L = _native.lib()
    L.aac_env_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.aac_env_reset_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    epb_for = lambda apw: 1 if N > apw else apw // N                      # noqa: E731  (aac_env.hip policy)
    epb = epb_for(24)
    while epb < epb_for(50) and (E + epb - 1) // epb > 1024:
        epb += 1
    nwg = (E + epb - 1) // epb
    acc = {k: [] for k in ("kin", "radar", "agent", "final", "draw", "writes", "rradar", "robs", "life_r", "life_n")}
    ev = []
    for k in range(40):
        c, n = bufs[k % 2], bufs[1 - k % 2]
        act = torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1
        srcs = [c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei] + \
            ([hid[k % 2], hid[1 - k % 2]] if H else [])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.step_tail(act, out=n, replay=rep, srcs=srcs, zero_rows=hid[1 - k % 2] if H else None)
        e1.record()
        torch.cuda.synchronize()
        if k < 20:
            continue
        ev.append(e0.elapsed_time(e1) * 1e3)
        sb = np.zeros((nwg, 7), dtype=np.uint64)
        rb = np.zeros((nwg, 7), dtype=np.uint64)
        assert L.aac_env_stamps(sb.ctypes.data, nwg) == 0
        assert L.aac_env_reset_stamps(rb.ctypes.data, nwg) == 0
        s, r = sb.astype(np.int64), rb.astype(np.int64)
        ph = np.diff(s[:, 1:6], axis=1)
        res = (r[:, 2] > s[:, 4]) & (r[:, 2] < s[:, 5])          # reset stamps from this launch
        acc["kin"] += ph[:, 0].tolist()
        acc["radar"] += ph[:, 1].tolist()
        acc["agent"] += ph[:, 2].tolist()
        acc["final"] += ph[~res, 3].tolist()
        acc["draw"] += (r[res, 2] - s[res, 4]).tolist()
        acc["writes"] += (r[res, 3] - r[res, 2]).tolist()
        acc["rradar"] += (r[res, 4] - r[res, 3]).tolist()
        acc["robs"] += (r[res, 5] - r[res, 4]).tolist()
        acc["life_r"] += (s[res, 5] - s[res, 1]).tolist()
        acc["life_n"] += (s[~res, 5] - s[~res, 1]).tolist()
    print(f"[{kind}] E={E} N={N}: {nwg} wg x {epb} envs, event median {np.median(ev):.1f} us, "
          f"resetting wg per step {len(acc['draw']) / len(ev):.0f}")
    for name, v in acc.items():
        v = np.asarray(v)
        if v.size:
            print(f"  {name:7s} cycles median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  max {v.max():8.0f}")


if __name__ == "__main__":
    main()
