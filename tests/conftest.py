import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"
SHIPPED_DATA = os.path.join(REFERENCE, "data", "synthetic_data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


def _load_reference_package():
    """Import the read-only reference ``src`` package under the name ``ref_src`` (this repo has
    its own top-level ``src`` compatibility package, so the name must not collide)."""
    if "ref_src" in sys.modules:
        return sys.modules["ref_src"]
    sys.dont_write_bytecode = True       # never write .pyc files into the read-only checkout
    init = os.path.join(REFERENCE, "src", "__init__.py")
    spec = importlib.util.spec_from_file_location("ref_src", init,
                                                  submodule_search_locations=[os.path.dirname(init)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ref_src"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def reference_src():
    """The reference package as a test oracle (skips where the checkout is absent, e.g. on the
    GPU box). Only its Python sources are imported; nothing prebuilt is loaded."""
    if not os.path.isfile(os.path.join(REFERENCE, "src", "__init__.py")):
        pytest.skip("reference checkout not available on this machine")
    return _load_reference_package()


@pytest.fixture(scope="session")
def shipped_data():
    if not os.path.isdir(os.path.join(SHIPPED_DATA, "char")):
        pytest.skip("reference synthetic data not available")
    return SHIPPED_DATA


@pytest.fixture(autouse=True)
def _trace_live_engines(request):
    """DLAP_TRACE_LIVE=1: print the number of native engines alive after each test (leaks)."""
    yield
    if os.environ.get("DLAP_TRACE_LIVE") == "1" and "deeplearninginassetpricing_paperreplication_amd._dlap_hip" in sys.modules:
        import gc
        gc.collect()
        mod = sys.modules["deeplearninginassetpricing_paperreplication_amd._dlap_hip"]
        print(f"\n[live-engines] {request.node.name}: {mod.Engine.live_engines()}", flush=True)
