import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP kernels")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def single_call_worker_clean():
    """Session-end check: no single call of the whole run was
    handed from the persistent worker kernel to the launch path -- a missed
    1 s deadline, a stream error, more than three restarts, a failed start or
    a lone-block staging wait that gave up (lz4m_host.hip g_worker_failures).
    A worker that stalls cannot hide behind the fallback's correct bytes."""
    yield
    nat = sys.modules.get("lz4._native")
    if nat is None or getattr(nat, "_lib", None) is None:
        return   # the library never loaded (CPU-only run)
    import ctypes
    st = (ctypes.c_uint32 * 16)()
    failures = nat.lib().lz4m_single_call_worker_state(st)
    assert failures == 0, f"{failures} single call(s) fell back from the worker to the launch path"


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    return O.Oracle()


@pytest.fixture(scope="session")
def reference():
    import oracle as O
    if not os.path.exists(O.REF_SO) and not os.path.isdir("/root/reference/lz4libs"):
        pytest.skip("reference lz4libs build not available")
    return O.Reference()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import lz4._native as N
    N.lib()
    return torch.device("cuda", 0)
