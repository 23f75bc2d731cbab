"""Compiled control-plane modules (_native.cyaccel): an extension is imported only while its
recorded source hash matches the current source, never stale; pure mode imports the .py."""
import os

import pytest

from k8s_gpu_scheduler_amd._native import cyaccel


def test_finder_never_returns_a_stale_extension(tmp_path):
    mod = "api.objects"
    full = f"{cyaccel.PKG}.{mod}"
    fresh = cyaccel._Finder({mod: cyaccel._sha(cyaccel._source(mod))})
    stale = cyaccel._Finder({mod: "0" * 40})
    pure = cyaccel._Finder({mod: cyaccel._sha(cyaccel._source(mod))}, pure=True)
    assert stale.find_spec(full).origin.endswith(".py")
    assert pure.find_spec(full).origin.endswith(".py")
    spec = fresh.find_spec(full)
    if os.path.exists(cyaccel._ext_path(mod)):
        assert spec.origin == cyaccel._ext_path(mod)
    else:
        assert spec.origin.endswith(".py")
    assert fresh.find_spec("json") is None
    assert fresh.find_spec(f"{cyaccel.PKG}.cli.main") is None       # not a compiled module


def test_compiled_modules_loaded_when_built():
    if not all(os.path.exists(cyaccel._ext_path(m)) for m in cyaccel.MODULES):
        pytest.skip("compiled modules not built (python -m k8s_gpu_scheduler_amd._native.build)")
    if os.environ.get("GPUSCHED_PURE_PYTHON", "") not in ("", "0"):
        pytest.skip("pure-Python mode requested")
    import k8s_gpu_scheduler_amd.framework.scheduler as sched
    man = cyaccel._read_manifest()
    if man.get("framework.scheduler") != cyaccel._sha(cyaccel._source("framework.scheduler")):
        pytest.skip("compiled modules are stale (sources edited since the build)")
    assert sched.__file__.endswith(cyaccel.EXT)
    assert cyaccel.status().get(f"{cyaccel.PKG}.framework.scheduler") is True
