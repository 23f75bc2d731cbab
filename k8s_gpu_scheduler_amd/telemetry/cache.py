"""Live per-device telemetry as the scheduler sees it.

The reference reads DCGM series through Prometheus inside Score (only on its fallback
path; reference gpu_plugins.go:162-300,508-527).  Here sources (the node agent's
amdsmi sampler, a Prometheus poller, or the bench's RCCL all-gather of per-rank
counters) *push* samples into this cache, and Score reads it with no I/O.  Samples
older than `stale_s` are ignored (telemetry outage -> the plugin degrades to
prediction/packing-only scoring).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Dict, Optional


@dataclass
class DeviceSample:
    gfx_activity: float = 0.0        # 0..1 (DCGM_FI_PROF_GR_ENGINE_ACTIVE analog)
    umc_activity: float = 0.0        # 0..1 (memory controller busy)
    vram_used_mb: float = 0.0
    vram_total_mb: float = 288 * 1024.0
    power_w: float = 0.0
    temp_c: float = 0.0
    xgmi_tx_bps: float = 0.0
    xgmi_rx_bps: float = 0.0
    ts: float = field(default_factory=time.monotonic)

    @property
    def vram_free_frac(self) -> float:
        return max(0.0, 1.0 - self.vram_used_mb / max(self.vram_total_mb, 1.0))


class TelemetryCache:
    def __init__(self, stale_s: float = 10.0):
        self._lock = threading.Lock()
        self._d: Dict[str, Dict[str, DeviceSample]] = {}      # node -> uuid -> latest sample
        self.stale_s = stale_s
        self.updates = 0
        self._node_ver: Dict[str, int] = {}
        from ..framework.changes import ChangeFanout
        self.changes = ChangeFanout()           # scheduling-cycle node-result caches

    def update(self, node: str, uuid: str, sample: DeviceSample) -> None:
        with self._lock:
            self._d.setdefault(node, {})[uuid] = sample
            self.updates += 1
            self._node_ver[node] = self._node_ver.get(node, 0) + 1
        self.changes.touch(node)

    def node_version(self, node: str) -> int:
        """Bumped on every sample for the node (0 = never sampled): lets Score memoise
        per-node results until the node's telemetry changes."""
        return self._node_ver.get(node, 0)

    def get(self, node: str, uuid: str) -> Optional[DeviceSample]:
        with self._lock:
            s = self._d.get(node, {}).get(uuid)
        if s is None or (self.stale_s and time.monotonic() - s.ts > self.stale_s):
            return None
        return s

    def node(self, node: str) -> Dict[str, DeviceSample]:
        """Fresh samples of one node, uuid -> sample (one lock, O(devices of the node))."""
        with self._lock:
            d = dict(self._d.get(node, {}))
        if not self.stale_s:
            return d
        now = time.monotonic()
        return {u: s for u, s in d.items() if now - s.ts <= self.stale_s}
