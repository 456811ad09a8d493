import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libgrape.so)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()


# Achieved parity errors, recorded by the GPU parity tests (tests/parity_log.py) and written to
# gpurun_out/parity_errors_<pid>.json at the end of the session when that directory exists.
def pytest_sessionfinish(session, exitstatus):
    from tests import parity_log
    parity_log.dump(os.path.join(ROOT, "gpurun_out"))
