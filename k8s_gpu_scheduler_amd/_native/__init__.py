"""Loader for the in-tree native modules (_core, _smi, _hip).

Policy: on a machine with a visible GPU the HIP module is REQUIRED -- `hip()` raises if
it is missing instead of silently falling back to PyTorch, so a GPU run can never pass
on a non-native path.  `_core` (host scoring core) and `_smi` are optional on CPU-only
hosts; callers fall back to the Python implementations there.
"""
from __future__ import annotations

import importlib
import os
from typing import Any, Optional

_cache: dict = {}


class NativeMissing(ImportError):
    pass


def _load(name: str) -> Optional[Any]:
    if name in _cache:
        return _cache[name]
    try:
        mod = importlib.import_module(f"{__name__}.{name}")
    except ImportError:
        mod = None
    _cache[name] = mod
    return mod


def core() -> Optional[Any]:
    return _load("_core")


def smi() -> Optional[Any]:
    return _load("_smi")


def hip(required: bool = True) -> Optional[Any]:
    m = _load("_hip")
    if m is None and required:
        raise NativeMissing("k8s_gpu_scheduler_amd._native._hip is not built: run "
                            "`python -m k8s_gpu_scheduler_amd._native.build` (hipcc --offload-arch=gfx950)")
    return m


def ensure_built() -> None:
    """Build stale/missing modules (no-op when up to date)."""
    from .build import build
    build()
    _cache.clear()


def loaded_paths() -> dict:
    return {k: getattr(v, "__file__", None) for k, v in _cache.items() if v is not None}
