"""Microbenchmark of the training attention kernels (aac_attn_train_fwd / _bwd) at the bench's
shapes (R = B * N rows, K = N - 1 neighbours).  python tools/mb_attn.py [R] [K]; the rows per
workgroup come from AAC_ATTN_ROWS (read by libaac_env.so at load)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import fused  # noqa: E402


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 5120   # noqa
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    d = "cuda"
    g = torch.Generator(device=d).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=d, generator=g)  # noqa: E731
    eo, xn, nei = r(R, 192), torch.relu(r(R * K, 64)), r(R * K, 6)
    Wq, Wk, Wv = r(64, 64) / 8, r(64, 64) / 8, r(64, 64) / 8
    q, qk, xb, vout = (torch.empty(R, 64, device=d) for _ in range(4))
    alpha = torch.empty(R, K, device=d)
    dv, dcat = r(R, 128), r(R, 192)
    dxn, dqk, dq, deo = torch.empty(R * K, 64, device=d), *(torch.empty(R, 64, device=d) for _ in range(3))
    P = fused.ptr
    f = lambda: fused.attn_train_fwd(P(eo), 192, P(xn), P(nei), P(Wq), P(Wk), P(Wv), P(q), P(qk), P(alpha),  # noqa
                                     P(xb), P(vout), 128, R, K)
    bw = lambda: fused.attn_train_bwd(P(dv), 128, P(xn), P(alpha), P(qk), P(eo), 192, P(dcat), 192, P(Wq),  # noqa
                                      P(Wk), P(Wv), P(dxn), P(dqk), P(dq), P(deo), R, K)
    Wn, bn, wqk, out = r(64, 6) / 2, r(64) / 8, r(64, 64) / 8, torch.empty(R, 64, device=d)
    blk = lambda: fused.attn_block(P(eo), 192, P(nei), P(Wn), P(bn), P(wqk), P(Wv), P(out), 64, R, K)  # noqa: E731
    print(f"R={R} K={K} rows/wg={os.environ.get('AAC_ATTN_ROWS', 16)} fwd {timed(f):.2f} us  bwd {timed(bw):.2f} us"
          f"  block {timed(blk):.2f} us")


if __name__ == "__main__":
    main()
