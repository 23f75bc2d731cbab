"""Compiled control-plane modules: the scheduling hot path (framework runtime, queue, cache,
GPU plugin, object helpers, fake apiserver + informers, bench control plane) compiled with
Cython into extension modules that sit NEXT TO their .py sources.

The scheduler is a Python re-implementation of the kube-scheduler framework (the reference
links the Go one, reference cmd/scheduler/main.go:20-22); on the bench's 8-GPU node the
control plane schedules 32 pods per epoch inside one GPU epoch, so its per-pod cost bounds
multi-GPU scaling (profiles/archive/r02_control_plane_timing_box.txt).  Compiling the unchanged
sources removes the interpreter's dispatch overhead (~15-18 % per epoch measured).

Safety: an extension module shadows its .py (CPython's path finder prefers extension
modules), so a source edited after the build would silently run stale code.  `install()`
puts a finder first on sys.meta_path that checks each compiled module's recorded source
hash (manifest written by `build()`) against the current source and imports the .py when
they differ.  `GPUSCHED_PURE_PYTHON=1` disables the compiled modules entirely.
"""
from __future__ import annotations

import hashlib
import importlib.abc
import importlib.machinery
import importlib.util
import json
import os
import subprocess
import sys
import sysconfig
import tempfile
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(HERE)
PKG = os.path.basename(PKG_DIR)
MANIFEST = os.path.join(HERE, "cy_manifest.json")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

# dotted names below the package
MODULES = (
    "api.objects",
    "framework.interface", "framework.runtime", "framework.scheduler", "framework.queue",
    "framework.cache", "framework.changes", "framework.default_plugins", "framework.placement_plugins",
    "kube.client", "kube.informer",
    "plugins.gpu.plugin", "plugins.gpu.devices", "plugins.gpu.scoring", "plugins.gpu.planner",
    "plugins.gpu.timeline",
    "telemetry.cache", "telemetry.workcost",
    "parallel.podbench",
)


def _source(mod: str) -> str:
    return os.path.join(PKG_DIR, *mod.split(".")) + ".py"


def _ext_path(mod: str) -> str:
    return os.path.join(PKG_DIR, *mod.split(".")) + EXT


def _sha(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha1(f.read()).hexdigest()


def _read_manifest() -> Dict[str, str]:
    try:
        with open(MANIFEST) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def available() -> bool:
    try:
        import Cython  # noqa: F401
    except ImportError:
        return False
    return True


def build(force: bool = False, verbose: bool = False) -> List[str]:
    """Compile stale modules (source hash differs from the manifest, or no extension)."""
    if not available():
        return []
    man = _read_manifest()
    todo = [m for m in MODULES if force or man.get(m) != _sha(_source(m)) or not os.path.exists(_ext_path(m))]
    if not todo:
        return []
    inc = sysconfig.get_paths()["include"]
    tmp = tempfile.mkdtemp(prefix="gpusched_cy_")

    def one(mod: str) -> str:
        full = f"{PKG}.{mod}"
        src, c_file, out = _source(mod), os.path.join(tmp, full + ".c"), _ext_path(mod)
        sha = _sha(src)
        cmd = [sys.executable, "-m", "cython", "-3", "-X", "binding=True", "-X", "embedsignature=False", "-X", "annotation_typing=False",
               "--module-name", full, "-o", c_file, src]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"cython {mod} failed:\n{p.stderr[-3000:]}")
        cc = ["gcc", "-O2", "-shared", "-fPIC", "-fno-strict-aliasing", "-Wno-unused-result",
              f"-I{inc}", c_file, "-o", out + ".tmp"]
        if verbose:
            print(" ".join(cc), file=sys.stderr)
        p = subprocess.run(cc, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"compiling {mod} failed:\n{p.stderr[-3000:]}")
        os.replace(out + ".tmp", out)
        return sha

    with ThreadPoolExecutor(min(8, len(todo))) as ex:
        shas = list(ex.map(one, todo))
    for m, s in zip(todo, shas):
        man[m] = s
    with open(MANIFEST + ".tmp", "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    os.replace(MANIFEST + ".tmp", MANIFEST)
    return [_ext_path(m) for m in todo]


class _Finder(importlib.abc.MetaPathFinder):
    """For compiled modules: the extension when its recorded source hash matches the
    current source, else the .py (never a stale extension)."""

    def __init__(self, manifest: Dict[str, str], pure: bool = False, skip: frozenset = frozenset()):
        self.manifest = manifest
        self.pure = pure
        self.skip = skip
        self.compiled: Dict[str, bool] = {}

    def find_spec(self, fullname: str, path=None, target=None) -> Optional[importlib.machinery.ModuleSpec]:
        if not fullname.startswith(PKG + "."):
            return None
        mod = fullname[len(PKG) + 1:]
        if mod not in MODULES:
            return None
        src, ext = _source(mod), _ext_path(mod)
        use_ext = (not self.pure and mod not in self.skip and os.path.exists(ext) and os.path.exists(src)
                   and self.manifest.get(mod) == _sha(src))
        self.compiled[fullname] = use_ext
        if use_ext:
            return importlib.util.spec_from_file_location(
                fullname, ext, loader=importlib.machinery.ExtensionFileLoader(fullname, ext))
        return importlib.util.spec_from_file_location(
            fullname, src, loader=importlib.machinery.SourceFileLoader(fullname, src))


_finder: Optional[_Finder] = None


def install() -> Optional[_Finder]:
    """Idempotent.  With GPUSCHED_PURE_PYTHON=1 the finder still runs -- and imports every
    listed module from its .py, which an extension next to it would otherwise shadow;
    GPUSCHED_CY_SKIP=mod[,mod] (dotted names below the package) does so for those modules
    only (A/Bs of one module's compilation)."""
    global _finder
    if _finder is None:
        skip = frozenset(x.strip() for x in os.environ.get("GPUSCHED_CY_SKIP", "").split(",") if x.strip())
        _finder = _Finder(_read_manifest(), pure=os.environ.get("GPUSCHED_PURE_PYTHON", "") not in ("", "0"),
                          skip=skip)
        sys.meta_path.insert(0, _finder)
    return _finder


def status() -> Dict[str, bool]:
    """fullname -> True when the compiled extension was imported."""
    return dict(_finder.compiled) if _finder is not None else {}
