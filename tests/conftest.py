import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from tests import report  # noqa: E402

try:  # torch's bundled HIP runtime must load before the engine's: the GPU tests
    import torch  # noqa: F401,E402  use torch tensors after engine contexts exist
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """One line per BASELINE config checked (tests/report.py), so the tail of
    a -q run names every config and its parity errors."""
    if report.LINES:
        terminalreporter.write_sep("=", "config parity (max relative errors)")
        for line in report.LINES:
            terminalreporter.write_line(line)


@pytest.fixture(scope="session")
def ref_examples():
    path = "/root/reference/examples"
    if not os.path.isdir(path):
        pytest.skip("reference examples not mounted (GPU box)")
    return path
