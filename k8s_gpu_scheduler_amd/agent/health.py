"""GPU health for the node agent (failure detection).

The reference has no health path: a failed GPU keeps its UUID in Redis and keeps getting
pods (its only recovery is deleting the profiler pod after a MIG change,
reference gpu_plugins.go:415-451).  Here the agent turns each amd-smi sample into a
per-device verdict -- the device-plugin model of Kubernetes, where an unhealthy device
stops being allocatable but running pods are left alone unless eviction is asked for:

* **uncorrectable ECC** -- the accumulated count (amdsmi_get_gpu_total_ecc_count) grew by
  more than `ecc_uncorrectable_max` since the agent first saw the device: sticky (HBM
  with uncorrectable errors needs an operator / GPU reset; a reset re-enumerates and the
  new UUID starts clean);
* **unresponsive** -- `miss_max` consecutive samples in which neither the activity nor the
  VRAM query answered (or no sample at all for the device): recovers when it answers;
* **thermal** -- hotspot >= `temp_crit_c`: recovers below `temp_crit_c - temp_hyst_c`.

`update()` returns whether any verdict changed, so the agent republishes the device
descriptors (field `healthy`) and the node annotation only on transitions.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple


@dataclass
class DeviceHealth:
    healthy: bool = True
    reason: str = ""
    ecc_base: Optional[float] = None
    misses: int = 0
    hot: bool = False
    ecc_failed: bool = False
    history: List[Tuple[bool, str]] = field(default_factory=list)


class HealthMonitor:
    def __init__(self, ecc_uncorrectable_max: float = 0.0, temp_crit_c: float = 105.0, temp_hyst_c: float = 10.0,
                 miss_max: int = 3):
        self.ecc_uncorrectable_max = ecc_uncorrectable_max
        self.temp_crit_c = temp_crit_c
        self.temp_hyst_c = temp_hyst_c
        self.miss_max = miss_max
        self.devices: Dict[str, DeviceHealth] = {}

    def healthy(self, uuid: str) -> bool:
        h = self.devices.get(uuid)
        return h is None or h.healthy

    def reason(self, uuid: str) -> str:
        h = self.devices.get(uuid)
        return h.reason if h else ""

    def unhealthy(self) -> Dict[str, str]:
        return {u: h.reason for u, h in self.devices.items() if not h.healthy}

    def update(self, samples: List[Dict[str, Any]], devices: List[Dict[str, Any]]) -> bool:
        """samples: amd-smi dicts with `index` (position in `devices`); returns True when
        any device changed state."""
        by_idx = {int(s.get("index", -1)): s for s in samples}
        changed = False
        seen = set()
        for i, d in enumerate(devices):
            uuid = d["uuid"]
            seen.add(uuid)
            h = self.devices.setdefault(uuid, DeviceHealth())
            s = by_idx.get(i)
            # partitions of one GPU share its ECC / thermal counters: all verdicts are per
            # sample index, which the sources report per enumerated device
            if s is None or not self._responsive(s):
                h.misses += 1
            else:
                h.misses = 0
                ue = float(s.get("ecc_uncorrectable", -1))
                if ue >= 0:
                    if h.ecc_base is None:
                        h.ecc_base = ue
                    elif ue - h.ecc_base > self.ecc_uncorrectable_max:
                        h.ecc_failed = True
                t = float(s.get("temp_c", -1))
                if t >= self.temp_crit_c:
                    h.hot = True
                elif h.hot and 0 <= t < self.temp_crit_c - self.temp_hyst_c:
                    h.hot = False
            if h.ecc_failed:
                ok, why = False, "uncorrectable ECC errors"
            elif h.misses >= self.miss_max:
                ok, why = False, f"unresponsive for {h.misses} samples"
            elif h.hot:
                ok, why = False, f"hotspot temperature >= {self.temp_crit_c:g} C"
            else:
                ok, why = True, ""
            if ok != h.healthy or why != h.reason:
                changed = changed or ok != h.healthy
                h.healthy, h.reason = ok, why
                h.history.append((ok, why))
        for u in list(self.devices):
            if u not in seen:             # re-enumerated (reset / repartition): forget
                del self.devices[u]
        return changed

    @staticmethod
    def _responsive(s: Dict[str, Any]) -> bool:
        if "responsive" in s:
            return bool(s["responsive"])
        return float(s.get("gfx_activity", -1)) >= 0 or float(s.get("vram_used_mb", -1)) >= 0
