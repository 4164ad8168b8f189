"""ctypes binding of libaac_env.so (the C ABI declared in include/aac_env.h).

The library must be the in-tree build (``multi_agent_aac_amd/libaac_env.so``, made by
``__graft_entry__.build()``).  There is no fallback: if it is missing or a call fails,
a RuntimeError is raised.  torch is imported first so that the HIP runtime torch ships
(SONAME libamdhip64.so.7) is the one the library binds to, which lets the kernels run on
torch's streams and write into torch tensors.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
# AAC_LIB: load another build of the same library (kernel experiments); default = the in-tree build
LIB_PATH = os.environ.get("AAC_LIB") or os.path.join(_HERE, "libaac_env.so")

EXPORTS = (
    "aac_env_create", "aac_env_destroy", "aac_last_error", "aac_env_reset", "aac_env_step", "aac_env_step_tail",
    "aac_env_set_od_bank", "aac_env_set_od_banks", "aac_env_auto_reset", "aac_env_set_reset_compact", "aac_env_use_episode_buffer", "aac_env_get_state", "aac_env_set_state",
    "aac_env_band_max", "aac_astar", "aac_od_bank_build",
)

vp = ctypes.c_void_p
i32 = ctypes.c_int32


class EnvCfg(ctypes.Structure):
    _fields_ = [("E", i32), ("N", i32), ("R", i32), ("radar_mode", i32), ("compat", i32), ("team_reward", i32),
                ("max_wp", i32),
                ("episode_length", i32), ("grid_w", i32), ("grid_h", i32), ("n_maps", i32),
                ("dt", ctypes.c_double), ("acc_max", ctypes.c_double), ("vmax", ctypes.c_double),
                ("pB", ctypes.c_double), ("radar_len", ctypes.c_double), ("bound", ctypes.c_double * 4),
                ("cell", ctypes.c_double), ("occ", vp), ("variant", i32)]


class StepOut(ctypes.Structure):
    _fields_ = [(n, vp) for n in ("own", "radar", "nei", "reward", "done", "mask", "env_done", "bbc",
                                  "tcpa", "dcpa", "conf_cur", "conf_pre")]


class StepTail(ctypes.Structure):
    _fields_ = [("ring", vp), ("row_width", i32), ("capacity", ctypes.c_int64), ("pos", ctypes.c_int64),
                ("size", ctypes.c_int64), ("meta", vp), ("n_fields", i32), ("srcs", ctypes.POINTER(vp)),
                ("widths", ctypes.POINTER(i32)), ("dtypes", ctypes.POINTER(i32)), ("zero_rows", vp),
                ("zero_width", i32), ("auto_reset", i32), ("pos_in", vp), ("pos_out", vp)]


_lib = None


def lib():
    """Load libaac_env.so (in-tree) and declare signatures.  Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    L.aac_last_error.restype = ctypes.c_char_p
    L.aac_env_create.argtypes = [ctypes.POINTER(EnvCfg), ctypes.c_int, ctypes.POINTER(vp)]
    L.aac_env_destroy.argtypes = [vp]
    L.aac_env_destroy.restype = None
    L.aac_env_reset.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.POINTER(StepOut), vp]
    L.aac_env_step.argtypes = [vp, vp, ctypes.POINTER(StepOut), vp]
    L.aac_env_step_tail.argtypes = [vp, vp, ctypes.POINTER(StepOut), ctypes.POINTER(StepTail), vp]
    L.aac_env_set_od_bank.argtypes = [vp, vp, vp, vp, i32, ctypes.c_uint64]
    L.aac_env_set_od_banks.argtypes = [vp, i32, vp, vp, vp, vp, ctypes.c_uint64]
    L.aac_env_auto_reset.argtypes = [vp, vp, ctypes.POINTER(StepOut), vp]
    L.aac_env_set_reset_compact.argtypes = [ctypes.c_int32]
    L.aac_env_set_reset_compact.restype = None
    L.aac_env_use_episode_buffer.argtypes = [vp, vp, vp]
    if hasattr(L, "aac_env_band_max") or not os.environ.get("AAC_LIB"):   # (older A/B builds lack it)
        L.aac_env_band_max.argtypes = [vp, vp, vp, vp]
    L.aac_env_get_state.argtypes = [vp] + [vp] * 13 + [vp]
    L.aac_env_set_state.argtypes = [vp] + [vp] * 13 + [vp]
    L.aac_astar.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, i32]
    L.aac_od_bank_build.argtypes = [vp, i32, i32, vp, ctypes.c_double, i32, ctypes.c_uint64, i32, vp, vp, vp]
    for name in EXPORTS:
        if os.environ.get("AAC_LIB") and not hasattr(L, name):
            continue          # an A/B experiment build of an earlier revision
        getattr(L, name)
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        msg = lib().aac_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")
    return rc
