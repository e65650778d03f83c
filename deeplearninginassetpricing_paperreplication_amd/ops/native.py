"""Loader of the in-tree native HIP extension (``_dlap_hip``).

GPU code paths must run on the hand-written gfx950 kernels: if the extension is missing or
fails to load on a machine with a GPU we raise instead of silently falling back to eager
PyTorch. ``DLAP_AUTOBUILD=1`` (default) compiles it in-tree on first use.

``DLAP_NATIVE=debug`` (device bounds assertions) or ``DLAP_NATIVE=ubsan`` (host UBSan, trap
mode) loads the variant built by ``engine.build --debug`` / ``--ubsan`` instead.
"""
from __future__ import annotations

import importlib
import os

_mod = None
_err = None


def load(required: bool = True):
    global _mod, _err
    if _mod is not None:
        return _mod
    variant = os.environ.get("DLAP_NATIVE", "")
    if variant:
        _mod = _load_variant(variant)
        return _mod
    try:
        _mod = importlib.import_module("deeplearninginassetpricing_paperreplication_amd._dlap_hip")
        return _mod
    except ImportError as e:  # pragma: no cover - exercised on fresh checkouts
        _err = e
    if os.environ.get("DLAP_AUTOBUILD", "1") == "1":
        from ..engine.build import build
        build(verbose=False)
        _mod = importlib.import_module("deeplearninginassetpricing_paperreplication_amd._dlap_hip")
        return _mod
    if required:
        raise RuntimeError(f"native HIP extension _dlap_hip is not available ({_err}); "
                           "run `python -m deeplearninginassetpricing_paperreplication_amd.engine.build`")
    return None


def _load_variant(variant: str):
    import importlib.util
    import sys
    from ..engine.build import build, variant_path
    path = variant_path(variant)
    if not path.exists():
        if os.environ.get("DLAP_AUTOBUILD", "1") != "1":
            raise RuntimeError(f"native variant {variant!r} not built ({path})")
        build(verbose=False, ubsan=variant == "ubsan", debug=variant == "debug")
    name = "deeplearninginassetpricing_paperreplication_amd._dlap_hip"
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules[name] = mod
    return mod


def available() -> bool:
    try:
        return load(required=False) is not None
    except Exception:
        return False
