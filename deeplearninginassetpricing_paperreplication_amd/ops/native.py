"""Loader of the in-tree native HIP extension (``_dlap_hip``).

GPU code paths must run on the hand-written gfx950 kernels: if the extension is missing or
fails to load on a machine with a GPU we raise instead of silently falling back to eager
PyTorch. ``DLAP_AUTOBUILD=1`` (default) compiles it in-tree on first use.
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


def available() -> bool:
    try:
        return load(required=False) is not None
    except Exception:
        return False
