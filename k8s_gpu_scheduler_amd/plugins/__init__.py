"""Plugin registry: in-tree defaults + the out-of-tree "GPU" plugin
(the reference registers it with app.WithPlugin(gpuPlugin.Name, gpuPlugin.New),
reference cmd/scheduler/main.go:20-22)."""
from __future__ import annotations

from ..framework.default_plugins import default_registry
from ..framework.runtime import Registry


def full_registry() -> Registry:
    from .gpu.plugin import register
    r = default_registry()
    register(r)
    return r
