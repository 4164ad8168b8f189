"""Microbenchmark of the replay draw (aac_replay_sample: B distinct rows of the ring, one workgroup),
graph-replayed: python tools/mb_sample.py [reps].  Prints us per launch for the config-3 / 4 / 5
batch sizes at a few ring sizes.  AAC_LIB picks the library (A/B against a variant build)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    from multi_agent_aac_amd import ops
    res = {}
    for B in (512, 1024):
        for size in (20000, 200000, 1000000):
            meta = torch.tensor([0, size], dtype=torch.int64, device="cuda")
            counter = torch.zeros(1, dtype=torch.int64, device="cuda")
            idx = torch.zeros(B, dtype=torch.int32, device="cuda")
            fn = lambda: ops.replay_sample(meta, B, 7, counter, idx)   # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(reps):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[f"B{B}_size{size}"] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
    print(json.dumps({"sample_us": res, "lib": os.environ.get("AAC_LIB", "in-tree")}), flush=True)


if __name__ == "__main__":
    main()
