"""Phase timestamps (s_memtime) of uam_step_kernel's first 64 workgroups at the config-5 size,
from a probe build with -DAAC_UAM_STAMPS (multi_agent_aac_amd/libaac_probe.so via AAC_LIB).
Phases: 1 clouds + kinematics, 2 distances, 3 neighbour order, radar (3a fixed boundaries +
candidate list, 3b clip jobs, 3c stores), 5 observation + goal touch, 6 ss_reward predicates, end:
the per-env pass and the writes."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import uam  # noqa: E402


def main():
    E, N = 8192, 16
    env = uam.BatchedUAM(E, N, neighbours=True)
    env.set_bank(uam.build_bank(16384, N, seed=1), seed=2)
    env.auto_reset()
    L = uam.lib()
    buf = (ctypes.c_ulonglong * (64 * 16))()
    g = torch.Generator(device="cuda").manual_seed(0)
    for it in range(6):
        act = torch.rand(E, N, 2, dtype=torch.float64, device="cuda", generator=g) * 2 - 1
        b = env.step(act)
        torch.cuda.synchronize()
        L.aac_uam_stamps(buf)
        a = np.array(buf, dtype=np.int64).reshape(64, 16)
        marks = [0, 1, 2, 3, 7, 8, 4, 5, 6, 15]     # radar = 3a (3 -> 7), 3b clips (7 -> 8), 3c stores (8 -> 4)
        d = np.diff(a[:, marks], axis=1)
        print("phase cycles (mean over 64 WGs):", [int(x) for x in d.mean(0)], "total", int((a[:, 15] - a[:, 0]).mean()))
        env.auto_reset(b.env_done)


if __name__ == "__main__":
    main()
