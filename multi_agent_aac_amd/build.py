"""In-tree build of the native libraries (hipcc, gfx950).

``python -m multi_agent_aac_amd.build`` (or ``__graft_entry__.build()``) compiles each of
``csrc/*.hip`` + ``csrc/aac_host.cpp`` to an object under ``build/`` (in parallel, only the stale
ones) and links them into ``libaac_env.so`` next to this file.  The library links the HIP runtime
by SONAME (libamdhip64.so.7), so inside a process that imported torch it binds to torch's runtime
and shares its streams.
"""
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("AAC_OFFLOAD_ARCH", "gfx950")

SOURCES = ["csrc/aac_env.hip", "csrc/aac_learn.hip", "csrc/aac_fused.hip", "csrc/aac_gru.hip", "csrc/aac_mpe.hip",
           "csrc/aac_uam.hip", "csrc/aac_uam_actor.hip", "csrc/aac_uam_learn.hip", "csrc/aac_host.cpp",
           "csrc/aac_trace.cpp"]
HEADERS = ["include/aac_env.h", "include/aac_learn.h", "include/aac_fused.h", "include/aac_gru.h", "include/aac_mpe.h",
           "include/aac_uam.h", "include/aac_uam_learn.h", "include/aac_trace.h", "multi_agent_aac_amd/csrc/aac_wave.h",
           "multi_agent_aac_amd/csrc/aac_geom.h"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function", f"--offload-arch={ARCH}"]
# roctx ranges (include/aac_trace.h) come from rocprofiler-sdk's roctx library, found at run time by rpath
LINK = ["-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
LIB = os.path.join(HERE, "libaac_env.so")
OBJ = os.path.join(ROOT, "build", "obj")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, obj, verbose):
    cmd = [HIPCC] + FLAGS + ["-I", os.path.join(ROOT, "include"), "-c", "-o", obj, src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=HERE)
    return obj


def build(force=False, verbose=False, jobs=None):
    srcs = [os.path.join(HERE, s) for s in SOURCES if os.path.exists(os.path.join(HERE, s))]
    hdrs = [p for p in (os.path.join(ROOT, h) for h in HEADERS) if os.path.exists(p)]
    if not force and not _stale(LIB, srcs + hdrs):
        return LIB              # up to date (the GPU box gets the library without the objects)
    os.makedirs(OBJ, exist_ok=True)
    objs = [os.path.join(OBJ, os.path.basename(s) + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if force or _stale(o, [s] + hdrs)]
    if todo:
        with cf.ThreadPoolExecutor(jobs or min(len(todo), os.cpu_count() or 4, 8)) as ex:
            for f in [ex.submit(_compile, s, o, verbose) for s, o in todo]:
                f.result()
    if force or todo or _stale(LIB, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + LINK
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=HERE)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
