"""Run pytest inside the host-ASan harness (``engine.build --asan-harness``):

    ASAN_OPTIONS=detect_leaks=0 DLAP_CRASH_TRACE=0 PYTHONHOME=/usr \\
        deeplearninginassetpricing_paperreplication_amd/asan/dlap_asan_python tools/asan_pytest.py tests -m gpu -q

The engine module is the instrumented built-in one the harness registers; any heap / stack /
global error in the runtime, the launchers or the bindings aborts with an ASan report."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":     # (multiprocessing's spawned children re-import this file)
    import pytest

    mod = sys.modules.get("deeplearninginassetpricing_paperreplication_amd._dlap_hip")
    print(f"[asan] engine module: {getattr(mod, '__file__', 'built-in (instrumented)')}", flush=True)
    sys.exit(pytest.main(sys.argv[1:]))
