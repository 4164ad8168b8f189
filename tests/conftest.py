"""Test configuration: ``-m gpu`` tests need a ROCm GPU and the in-tree libaac_env.so."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def native_lib():
    from multi_agent_aac_amd import build
    build.build()
    from multi_agent_aac_amd import _native
    return _native.lib()


@pytest.fixture(scope="session")
def occ():
    from multi_agent_aac_amd import world
    return world.synthetic_map(2026)


@pytest.fixture(autouse=True, scope="module")
def _drain_device_between_modules():
    """After each GPU test module: finish the device's queued work, then collect the module's
    native handles and captured graphs, so that no finaliser (env destroy, graph release) runs at
    an arbitrary garbage-collection point while launches that use their memory are in flight."""
    yield
    import gc
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        gc.collect()
        torch.cuda.synchronize()
