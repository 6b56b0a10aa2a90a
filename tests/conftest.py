import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


def pytest_sessionstart(session):
    # GPU sessions: initialise PyTorch's HIP runtime up front.  The library
    # shares it (torch's libamdhip64.so and /opt/rocm's have one soname, and
    # _capi.lib() imports torch before it loads libsgm_hip.so: INTEGRATION.md
    # "One HIP runtime per process"); this only makes the device
    # initialisation happen once, before the first test.
    expr = session.config.getoption("markexpr", "") or ""
    if "gpu" in expr and "not gpu" not in expr:
        try:
            import torch
            if torch.cuda.device_count() > 0:
                torch.cuda.init()
        except Exception:
            pass
