"""In-tree build of the native libraries (hipcc, gfx950).

``python -m multi_agent_aac_amd.build`` (or ``__graft_entry__.build()``) compiles
``csrc/*.hip`` + ``csrc/aac_host.cpp`` into ``libaac_env.so`` next to this file.  The library
links the HIP runtime by SONAME (libamdhip64.so.7), so inside a process that imported torch
it binds to torch's runtime and shares its streams.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("AAC_OFFLOAD_ARCH", "gfx950")

SOURCES = ["csrc/aac_env.hip", "csrc/aac_learn.hip", "csrc/aac_fused.hip", "csrc/aac_gru.hip", "csrc/aac_mpe.hip",
           "csrc/aac_uam.hip", "csrc/aac_uam_actor.hip", "csrc/aac_uam_learn.hip", "csrc/aac_host.cpp"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
         f"--offload-arch={ARCH}"]
LIB = os.path.join(HERE, "libaac_env.so")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    srcs = [os.path.join(HERE, s) for s in SOURCES if os.path.exists(os.path.join(HERE, s))]
    deps = srcs + [os.path.join(ROOT, "include", h) for h in ("aac_env.h", "aac_learn.h", "aac_fused.h", "aac_gru.h", "aac_mpe.h", "aac_uam.h", "aac_uam_learn.h")]
    deps += [os.path.join(HERE, "csrc", h) for h in ("aac_wave.h", "aac_geom.h")]
    deps = [d for d in deps if os.path.exists(d)]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = [HIPCC] + FLAGS + ["-I", os.path.join(ROOT, "include"), "-o", LIB] + srcs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=HERE)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
