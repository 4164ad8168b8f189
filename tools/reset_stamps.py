"""Phase timeline of the env auto-reset kernel (reset_kernel) in the training loop's steady state,
from a stamp build (bash tools/variant_lib.sh estamps multi_agent_aac_amd/csrc/aac_env.hip
-DAAC_ENV_STAMPS; AAC_LIB=tools/vlib/lib_estamps.so).  Default: config 4 (WGRU env, 8 agents x
4096 envs); ``att`` for config 3 (5 x 4096, combined radar).  Phases: OD draw, state writes, radar,
observation (cycles), per resetting workgroup."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from multi_agent_aac_amd import _native, world
    from multi_agent_aac_amd.env import BatchedEnv
    kind = sys.argv[1] if len(sys.argv) > 1 else "wgru"
    E, N = (4096, 8) if kind == "wgru" else (4096, 5)
    occ = world.synthetic_map(2026)
    env = BatchedEnv(E, N, occ, max_wp=32, variant=kind if kind == "wgru" else "att",
                     radar_mode=None if kind == "wgru" else "combined")
    env.set_od_bank(world.ODBank(occ, n_pairs=65536, seed=5, max_wp=32), seed=3)
    env.auto_reset(None)
    g = torch.Generator(device="cuda").manual_seed(0)
    L = _native.lib()
    L.aac_env_reset_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.aac_env_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    nwg = 65536
    epb_for = lambda apw: 1 if N > apw else apw // N                      # noqa: E731  (aac_env.hip policy)
    epb = epb_for(50) if E // epb_for(50) >= 1024 else epb_for(24)
    swg = (E + epb - 1) // epb
    for k in range(40):
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        env.step(torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1)
        s1.record()
        torch.cuda.synchronize()
        if k >= 30 and not k % 3:
            sb = np.zeros((swg, 7), dtype=np.uint64)
            assert L.aac_env_stamps(sb.ctypes.data, swg) == 0
            ss = sb.astype(np.int64)
            sp = np.diff(ss[:, 1:6], axis=1)
            print(f"[{kind}] step {k}: {swg} wg x {epb} envs, event {s0.elapsed_time(s1) * 1e3:.1f} us")
            for name, col in zip(("kinematics", "radar", "agent", "final"), sp.T):
                print(f"  {name:10s} cycles median {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}  "
                      f"max {col.max():8.0f}")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.auto_reset(env.bufs.env_done)
        e1.record()
        torch.cuda.synchronize()
        if k < 30 or k % 3:
            continue
        buf = np.zeros((nwg, 7), dtype=np.uint64)
        assert L.aac_env_reset_stamps(buf.ctypes.data, nwg) == 0
        st = buf.astype(np.int64)
        busy = st[:, 1] != 0
        st = st[busy]
        ph = np.diff(st[:, 1:6], axis=1)
        life = (st[:, 6] - st[:, 0]) / 100.0
        print(f"[{kind}] step {k}: {int(env.bufs.env_done.sum())} envs reset, {busy.sum()} busy wg, event "
              f"{e0.elapsed_time(e1) * 1e3:.1f} us, median life {np.median(life):.2f} us, max {life.max():.2f} us")
        for name, col in zip(("draw", "writes", "radar", "observe"), ph.T):
            print(f"  {name:8s} cycles median {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}  max {col.max():8.0f}")


if __name__ == "__main__":
    main()
