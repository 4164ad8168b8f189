"""Per-workgroup phase timeline of the env step kernel at config 3 (4096 x 5, combined radar) from a
stamp build (bash tools/variant_lib.sh estamps aac_env.hip -DAAC_ENV_STAMPS; AAC_LIB=tools/vlib/lib_estamps.so)."""
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
    radar = sys.argv[3] if len(sys.argv) > 3 else "combined"
    occ = world.synthetic_map(2026)
    env = BatchedEnv(E, N, occ, radar_mode=radar, max_wp=32)
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
    print(f"[{radar}] E={E} N={N}: {nwg} wg, event {e0.elapsed_time(e1) * 1e3:.1f} us; start spread {start.max():.2f} us, "
          f"last end {end.max():.2f} us, median life {np.median(end - start):.2f} us")
    for name, col in zip(("kinematics", "radar", "agent", "final"), ph.T):
        print(f"  {name:10s} cycles median {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}  max {col.max():8.0f}")
    print("  starts per bin:", np.histogram(start, bins=8)[0].tolist())
    # what slow radar workgroups hold: the closest agent pair of the workgroup's envs
    pos = env.get_state()["pos"].cpu().numpy()                      # (E, N, 2) after the step
    d = np.linalg.norm(pos[:, :, None, :] - pos[:, None, :, :], axis=-1)
    d[:, np.arange(N), np.arange(N)] = np.inf
    epb = 24 // N
    dmin = np.full(nwg, np.inf)
    for w in range(nwg):
        dmin[w] = d[w * epb:(w + 1) * epb].min()
    rad = ph[:, 1]
    # agent phase vs the full-path geometry cases: bound capsule in its uncertain band (fillet
    # vertices with fp64 cos/sin), goal in the 64-gon band
    stt = env.get_state()
    pp, gl = stt["pre_pos"].cpu().numpy(), stt["goal"].cpu().numpy()
    from multi_agent_aac_amd.world import BOUND
    r = 2.5                   # pB (ATT/env: the drone radius)
    lx, hx = np.minimum(pp[..., 0], pos[..., 0]), np.maximum(pp[..., 0], pos[..., 0])
    ly, hy = np.minimum(pp[..., 1], pos[..., 1]), np.maximum(pp[..., 1], pos[..., 1])
    lo, hi = r + 1e-9, r * np.cos(np.pi / 32) - 1e-9
    unc = np.zeros(pos.shape[:2], bool)
    for q, v in enumerate(BOUND):
        mn, mx = (lx, hx) if q < 2 else (ly, hy)
        inside = (v >= mn - hi) & (v <= mx + hi)
        outside = (v < mn - lo) | (v > mx + lo)
        unc |= ~inside & ~outside
    gd = np.linalg.norm(gl - pos, axis=-1)
    R = r + 1.0
    gband = (gd <= R * (1 + 1e-12) + 1e-12) & (gd >= R * np.cos(np.pi / 64) * (1 - 1e-12) - 1e-12)
    ag = ph[:, 2]
    for name, flag in (("capsule band", unc), ("goal band", gband)):
        fw = np.array([flag[w * epb:(w + 1) * epb].any() for w in range(nwg)])
        if fw.any():
            print(f"  {name}: {fw.sum()} wg, agent cycles median {np.median(ag[fw]):8.0f} max {ag[fw].max():8.0f}; "
                  f"others median {np.median(ag[~fw]):8.0f} max {ag[~fw].max():8.0f}")
        else:
            print(f"  {name}: none")
    slow = np.argsort(ag)[-5:]
    print("  slowest agent phases (cycles):", ag[slow].tolist())
    for lo, hi in ((0, 2.5), (2.5, 5), (5, 15), (15, 1e9)):
        sel = (dmin >= lo) & (dmin < hi)
        if sel.any():
            print(f"  closest pair in [{lo}, {hi}): {sel.sum():5d} wg, radar cycles median {np.median(rad[sel]):8.0f} "
                  f"max {rad[sel].max():8.0f}")


if __name__ == "__main__":
    main()
