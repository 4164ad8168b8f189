"""Phase timestamps (s_memtime, shader clocks) of workgroup 0 of the MFMA training-attention
forward, from a probe build (tools/attn_stamps.sh builds it with -DAAC_ATTN_STAMPS)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import fused  # noqa: E402
from multi_agent_aac_amd import _native  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    K = 4
    d = "cuda"
    r = lambda *s: torch.randn(*s, device=d)  # noqa: E731
    eo, xn, nei = r(R, 192), torch.relu(r(R * K, 64)), r(R * K, 6)
    Wq, Wk, Wv = r(64, 64) / 8, r(64, 64) / 8, r(64, 64) / 8
    q, qk, xb, vout = (torch.empty(R, 64, device=d) for _ in range(4))
    alpha = torch.empty(R, K, device=d)
    P = fused.ptr
    L = _native.lib()
    buf = (ctypes.c_ulonglong * 16)()
    for it in range(5):
        fused.attn_train_fwd(P(eo), 192, P(xn), P(nei), P(Wq), P(Wk), P(Wv), P(q), P(qk), P(alpha), P(xb),
                             P(vout), 128, R, K)
        torch.cuda.synchronize()
        L.aac_attn_stamps(buf)
        t = [buf[i] for i in range(6)]
        print("R", R, "phase cycles:", [t[i + 1] - t[i] for i in range(5)], "total", t[5] - t[0])


if __name__ == "__main__":
    main()
