"""Phase stamps of one aac_critic_fwd launch (variant library built with -DAAC_CF_STAMPS, loaded with
AAC_LIB): python tools/cf_stamps.py [case]  (case 0: B = 1024 plain, 1: fold + dual, 3: target 5120).
Prints median / max cycles per phase over the workgroups: 0->1 input rows, 1->2 folded output layer,
2->3 patch + barrier, 3->4 encoders, 4->5 barrier, 5->6 combine, 6->7 epilogue; plus the start skew."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tools.mb_cfwd as M  # noqa: E402
from multi_agent_aac_amd import fused  # noqa: E402


def main():
    case = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    ops = []
    orig = M.graph_us
    M.graph_us = lambda fn, reps: (ops.append(fn), 1.0)[1]
    M.main.__globals__["graph_us"] = M.graph_us
    M.main()
    op = ops[case]
    for _ in range(3):
        op()
    torch.cuda.synchronize()
    buf = np.zeros((4096, 8), dtype=np.uint64)
    lib = fused.lib()
    lib.aac_cf_stamps.argtypes = [ctypes.c_void_p]
    assert lib.aac_cf_stamps(buf.ctypes.data) == 0
    nwg = sum(4 * ((int(a.Bs) + 15) // 16) for a in op.arr)
    st = buf[:min(nwg, 4096)].astype(np.int64)
    d = np.diff(st, axis=1)
    names = ["rows", "fold", "patch+bar", "encoders", "barrier", "combine", "epilogue"]
    for k, n in enumerate(names):
        print(f"{n:10s} median {np.median(d[:, k]):8.0f}  p90 {np.percentile(d[:, k], 90):8.0f}  max {d[:, k].max():8.0f}")
    life = st[:, 7] - st[:, 0]
    print(f"life       median {np.median(life):8.0f}  max {life.max():8.0f}; start skew {st[:, 0].max() - st[:, 0].min()}")
    M.graph_us = orig


if __name__ == "__main__":
    main()
