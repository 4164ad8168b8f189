"""The C-ABI library loads on a CPU-only host and exports every function include/*.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(aac_\w+)\s*\(", src, flags=re.M)))


@pytest.mark.parametrize("header", sorted(h for h in os.listdir(os.path.join(ROOT, "include")) if h.endswith(".h")))
def test_exports(native_lib, header):
    names = _declared(header)
    assert names, header
    lib = ctypes.CDLL(os.path.join(ROOT, "multi_agent_aac_amd", "libaac_env.so"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_error_reporting(native_lib):
    from multi_agent_aac_amd import _native
    cfg = _native.EnvCfg()
    cfg.E, cfg.N, cfg.R = 0, 5, 18
    h = ctypes.c_void_p()
    rc = _native.lib().aac_env_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc == -1
    assert b"E > 0" in _native.lib().aac_last_error()
