"""Dump the whole-step pair graph of a small ATT / GRU trainer (hipGraphDebugDotPrint via
torch.cuda.CUDAGraph.debug_dump) and list its nodes in order: which non-kernel nodes (memcpy,
memset, event) sit between the kernels.  python tools/graph_dump.py [att|gru] -> gpurun_out/graph_<model>.dot
"""
import collections
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "gru"
    from multi_agent_aac_amd import trainer
    N = 8 if model == "gru" else 5
    tr = trainer.Trainer(512, N, 128, 4096, "combined", seed=0, model=model)
    while len(tr.replay) <= 3 * tr.B:
        tr.step(update=False)
    tr.step(update=True)
    p = 0 if tr.cur is tr.bufs[0] else 1
    orig = torch.cuda.CUDAGraph

    class Dbg(orig):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.enable_debug_mode()

    torch.cuda.CUDAGraph = Dbg
    try:
        g, _ = tr._capture_step(p, steps=2)
    finally:
        torch.cuda.CUDAGraph = orig
    os.makedirs("gpurun_out", exist_ok=True)
    path = f"gpurun_out/graph_{model}.dot"
    g.debug_dump(path)
    txt = open(path).read()
    kinds = collections.Counter()
    for m in re.finditer(r'label="([^"]*)"', txt):
        lab = m.group(1)
        kinds[lab.split("\\n")[0].split("|")[0][:40]] += 1
    print(len(txt), "bytes")
    for k, v in kinds.most_common(40):
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
