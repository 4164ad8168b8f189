"""Per-component device time of the UAM training step (bench.py --model uam's UamTrainer):
actor + noise, env step, replay push, auto-reset, update.  python tools/uam_breakdown.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    E, N, B = 8192, 16, 512
    tr = bench.UamTrainer(E, N, B, 1 << 20, seed=0)
    for _ in range(5):
        tr.step(update=True)
    torch.cuda.synchronize()
    names = ["act", "env", "push", "reset", "update"]
    ev = {k: [] for k in names}
    for _ in range(20):
        c, n = tr.cur, tr.nxt
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        marks[0].record()
        act = tr.model.act(c.own, c.radar, tr.episode, noisy=True)
        marks[1].record()
        tr.env.step(act, out=n)
        marks[2].record()
        tr.replay.push_batch(c.own, c.radar, act, n.reward, n.done, n.own, n.radar)
        marks[3].record()
        tr.env.auto_reset(n.env_done, out=n)
        tr.episode.add_(n.env_done.to(torch.int32))
        marks[4].record()
        tr.cur, tr.nxt = n, c
        tr.model.update(B)
        marks[5].record()
        for k, name in enumerate(names):
            ev[name].append((marks[k], marks[k + 1]))
    torch.cuda.synchronize()
    out = {k: sum(a.elapsed_time(b) for a, b in v) / len(v) for k, v in ev.items()}
    out["total"] = sum(out.values())
    print(json.dumps({k: round(v * 1e3, 1) for k, v in out.items()}))


if __name__ == "__main__":
    main()
