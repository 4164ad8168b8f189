"""Replay one grouped-GEMM launch of the config-3 update (index as printed by tools/gemm_table.py)
``reps`` times, for PMC runs: python tools/gemm_one.py 4 200."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import synth  # noqa: E402


def main():
    from multi_agent_aac_amd.maddpg import MADDPG
    k, reps = int(sys.argv[1]), int(sys.argv[2]) if len(sys.argv) > 2 else 100
    m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=5, device="cuda", seed=1, batch_size=1024)
    rep = m.attach_replay(8192, seed=1)
    for p in range(2):
        rep.push_batch(*synth.transitions(4096, 5, p))
    ops = m._fused_plan(1024).ops()
    for op in ops:
        op()
    for _ in range(reps):
        ops[k]()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
