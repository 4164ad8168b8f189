"""Per-workgroup phase timeline of the env step kernel at config 3 (4096 x 5, combined radar) from a
stamp build (bash tools/variant_lib.sh estamps aac_env.hip -DAAC_ENV_STAMPS; AAC_LIB=...)."""
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
    occ = world.synthetic_map(2026)
    env = BatchedEnv(E, N, occ, radar_mode="combined", max_wp=32)
    env.set_od_bank(world.ODBank(occ, n_pairs=16384, seed=5, max_wp=32), seed=3)
    env.auto_reset(None)
    g = torch.Generator(device="cuda").manual_seed(0)
    L = _native.lib()
    L.aac_env_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    for k in range(8):
        env.step(torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1)
        env.auto_reset(env.bufs.env_done)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    env.step(torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1)
    e1.record()
    torch.cuda.synchronize()
    nwg = (E + (24 // N) - 1) // (24 // N)
    buf = np.zeros((nwg, 7), dtype=np.uint64)
    assert L.aac_env_stamps(buf.ctypes.data, nwg) == 0
    st = buf.astype(np.int64)
    t0 = st[:, 0].min()
    start, end = (st[:, 0] - t0) / 100.0, (st[:, 6] - t0) / 100.0     # us
    ph = np.diff(st[:, 1:6], axis=1)                                  # kin, radar, agent, final (cycles)
    print(f"E={E} N={N}: {nwg} wg, event {e0.elapsed_time(e1) * 1e3:.1f} us; start spread {start.max():.2f} us, "
          f"last end {end.max():.2f} us, median life {np.median(end - start):.2f} us")
    for name, col in zip(("kinematics", "radar", "agent", "final"), ph.T):
        print(f"  {name:10s} cycles median {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}  max {col.max():8.0f}")
    print("  starts per bin:", np.histogram(start, bins=8)[0].tolist())


if __name__ == "__main__":
    main()
