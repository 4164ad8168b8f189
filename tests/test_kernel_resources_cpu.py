"""Compile-time guards (hipcc, no GPU): the hot kernels keep their registers -- no scratch.

Two regressions this catches were measured on the GPU: the env step kernel's 32 hoisted
building-hit limits spilled 66 VGPRs (240 B of scratch per lane, 23.5 MB of extra HBM writes per
launch), and a larger head-job code path made the compiler keep the grouped GEMM's by-value
GBatch argument in scratch (3.2 KB per lane: 0.6 -> 4.9 ms of GEMM per update)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _usage(src):
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                          "--offload-device-only", "-c", "-o", os.devnull, "-I", os.path.join(ROOT, "include"),
                          "-Rpass-analysis=kernel-resource-usage", os.path.join(ROOT, "multi_agent_aac_amd", "csrc", src)],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    kernels, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", line)
        if m and cur:
            kernels[cur][m.group(1).strip()] = int(m.group(2))
    return kernels


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,pattern", [("aac_fused.hip", "gemm_kernel"), ("aac_env.hip", "step_kernel"),
                                         ("aac_uam.hip", "uam_step_kernel"), ("aac_fused.hip", "actor_dcomb_out_bwd"),
                                         ("aac_fused.hip", "attn_mfma_bwd_kernel"),
                                         ("aac_fused.hip", "attn_enc_kernel")])
def test_hot_kernels_have_no_scratch(src, pattern):
    ks = {k: v for k, v in _usage(src).items() if pattern in k}
    assert ks, f"no {pattern} in {src}"
    for name, u in ks.items():
        assert u.get("ScratchSize", 0) == 0, (name, u)
