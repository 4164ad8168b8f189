"""Per-workgroup timeline of selected grouped-GEMM launches of the config-3 update, from a stamp
build (bash tools/variant_lib.sh stamps aac_fused.hip -DAAC_GEMM_STAMPS; AAC_LIB=...):
python tools/gemm_stamps.py 9 4 13   (launch indices as printed by tools/gemm_table.py)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import synth  # noqa: E402


def main():
    from multi_agent_aac_amd import _native
    from multi_agent_aac_amd.fused import GemmLaunch
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B, D0 = 5, 1024, 22
    m = MADDPG([D0, 18, 6], [D0, 18, 6], 2, n_agents=N, device="cuda", seed=1, batch_size=B)
    rep = m.attach_replay(8192, seed=1)
    for p in range(2):
        rep.push_batch(*synth.transitions(4096, N, p))
    ops = m._fused_plan(B).ops()
    for op in ops:
        op()
    torch.cuda.synchronize()
    L = _native.lib()
    L.aac_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    for k in [int(x) for x in sys.argv[1:]]:
        op = ops[k]
        assert isinstance(op, GemmLaunch)
        for _ in range(3):
            ops[k - 1]()            # the producer ran just before, as in the update
            op()
        torch.cuda.synchronize()
        buf = np.zeros((16384, 5), dtype=np.uint64)
        L.aac_gemm_stamps(buf.ctypes.data, 16384)      # read + clear
        ops[k - 1]()
        op()
        torch.cuda.synchronize()
        assert L.aac_gemm_stamps(buf.ctypes.data, 16384) == 0
        nwg = int((buf[:, 0] > 0).sum())
        st = buf[:nwg].astype(np.int64)
        t0 = st[:, 0].min()
        start = (st[:, 0] - t0) * 10 / 1000.0       # us (100 MHz)
        end = (st[:, 4] - t0) * 10 / 1000.0
        body = st[:, 2] - st[:, 1]
        epi = st[:, 3] - st[:, 2]
        shapes = " ".join(f"{p.M}x{p.N}x{p.K}/{p.ksplit}" for p in op.arr)
        print(f"launch {k}: {nwg} wg  {shapes}")
        print(f"  start spread {start.max():.2f} us, last end {end.max():.2f} us, median wg life "
              f"{np.median(end - start):.2f} us (p10 {np.percentile(end - start, 10):.2f}, p90 {np.percentile(end - start, 90):.2f})")
        print(f"  cycles: select+mma median {np.median(body):.0f} (p90 {np.percentile(body, 90):.0f}), epilogue median "
              f"{np.median(epi):.0f} (p90 {np.percentile(epi, 90):.0f})")
        hist = np.histogram(start, bins=8)
        print("  starts per bin:", hist[0].tolist(), "edges", [round(x, 2) for x in hist[1]])


if __name__ == "__main__":
    main()
