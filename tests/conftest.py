import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def reference_src():
    """The read-only reference package, used only as a test oracle (skips if absent)."""
    if not os.path.isdir(os.path.join(REFERENCE, "src")):
        pytest.skip("reference checkout not available on this machine")
    if REFERENCE not in sys.path:
        sys.path.append(REFERENCE)
    import importlib
    return importlib.import_module("src")
