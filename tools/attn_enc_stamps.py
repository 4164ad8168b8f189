"""Phase timestamps (s_memtime) of workgroup 0 of aac_attn_enc_fwd (training set, config-3 shapes),
from a probe build: bash tools/variant_lib.sh astamp aac_fused.hip -DAAC_ATTN_STAMPS, then
AAC_LIB=tools/vlib/lib_astamp.so python tools/attn_enc_stamps.py [R ...].  Phases: issue of the
staging + weight-fragment loads, staging barrier, encoders + stores, barrier, q, qk, softmax, v."""
import ctypes
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_agent_aac_amd import _native, fused  # noqa: E402

NAMES = ["issue", "stage-bar", "enc", "enc-bar", "q+bar", "qk+bar", "softmax+bar", "v"]


def main():
    dev, K, D0 = "cuda", 4, 22
    P = fused.ptr
    r = lambda *s: torch.randn(*s, device=dev) * 0.2  # noqa: E731
    W = {"Wo": r(64, D0), "bo": r(64), "Wg": r(64, 18), "bg": r(64), "Wn": r(64, 6), "bn": r(64), "Wq": r(64, 64)}
    kv = r(128, 64)
    ap = SimpleNamespace(**{k: P(v) for k, v in W.items()}, Wkv=P(kv))
    L = _native.lib()
    buf = (ctypes.c_ulonglong * 16)()
    for R in [int(x) for x in sys.argv[1:]] or [16, 5120]:
        own, radar, nei, cat = r(R, D0 + 2), r(R, 18), r(R, K, 6), torch.empty(R, 192, device=dev)
        acts = fused.ActorActs(R, K, dev)
        launch = fused.AttnEnc(fused.attn_set(ap, P(own), D0 + 2, D0, P(radar), P(nei), R, K, P(cat), acts=acts))
        for it in range(4):
            launch()
            torch.cuda.synchronize()
            L.aac_attn_stamps(buf)
            t = [buf[i] for i in range(9)]
            d = {NAMES[i]: int(t[i + 1] - t[i]) for i in range(8)}
            print(f"R {R} cycles total {t[8] - t[0]}:", d, flush=True)


if __name__ == "__main__":
    main()
