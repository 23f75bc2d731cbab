"""amd-smi activity sampling for one process's GPUs (benchmark / executor side).

The native `_smi` module samples gfx/umc activity, VRAM and power of selected GPUs on a C++
thread into a ring (native/smi/smi.cpp `start_activity`); this wrapper maps HIP device
indices to amd-smi processors by PCI address (the two enumerations need not agree, and a
container may see fewer HIP devices than amd-smi processors), drains the ring
incrementally, and summarises any time window -- so the benchmark can report what amd-smi
(the `DCGM_FI_PROF_GR_ENGINE_ACTIVE` analog the reference's Prometheus path reads,
reference pkg/prom/fetch_prom_metrics/prom_metrics.go:64-70) saw during its timed
region, next to its own HIP-event accounting, and feed the same samples into the
scheduler's TelemetryCache.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

log = logging.getLogger(__name__)

Row = Tuple[float, int, float, float, float, float]     # ts, smi index, gfx %, umc %, vram MB, power W


def smi_index_for_hip_devices(smi, hip_devices: Sequence[int]) -> Dict[int, int]:
    """{hip device index: amd-smi processor index}, matched on PCI domain/bus/device."""
    import torch
    by_bdf: Dict[Tuple[int, int, int], int] = {}
    for i in range(smi.count()):
        e = smi.enumeration(i)
        if "pci_bus" in e:
            by_bdf[(int(e["pci_domain"]), int(e["pci_bus"]), int(e["pci_device"]))] = i
    out: Dict[int, int] = {}
    for h in hip_devices:
        p = torch.cuda.get_device_properties(h)
        k = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
        if k in by_bdf:
            out[h] = by_bdf[k]
    return out


class ActivitySampler:
    """Background amd-smi activity sampler for the given HIP devices.

    `start()` returns False (and the sampler stays inert) when amd-smi is unavailable --
    callers report the fields as null rather than failing the run."""

    def __init__(self, hip_devices: Sequence[int], period_s: float = 0.005):
        self.hip_devices = list(hip_devices)
        self.period_s = period_s
        self.rows: List[Row] = []
        self._smi = None
        self.map: Dict[int, int] = {}
        self.error = ""
        self._lock = threading.Lock()

    def start(self) -> bool:
        try:
            from .. import _native
            mod = _native.smi()
            if mod is None:
                self.error = "native _smi module not built"
                return False
            smi = mod.Smi()
            if not smi.init():
                self.error = smi.error()
                return False
            self.map = smi_index_for_hip_devices(smi, self.hip_devices)
            if not self.map:
                self.error = "no amd-smi processor matches the HIP devices' PCI addresses"
                smi.shutdown()
                return False
            smi.start_activity(self.period_s, 200000, sorted(set(self.map.values())))
            self._smi = smi
            return True
        except Exception as e:          # telemetry must never break the workload
            self.error = str(e)
            log.warning("amd-smi activity sampler unavailable: %s", e)
            return False

    @property
    def active(self) -> bool:
        return self._smi is not None

    def poll(self) -> List[Row]:
        """Drain new samples (also kept for window summaries); returns only the new ones."""
        if self._smi is None:
            return []
        new = [tuple(r) for r in self._smi.drain_activity()]
        with self._lock:
            self.rows.extend(new)       # type: ignore[arg-type]
        return new                      # type: ignore[return-value]

    def stop(self) -> None:
        if self._smi is not None:
            self._smi.stop_activity()
            self.poll()
            self._smi.shutdown()
            self._smi = None

    def summary(self, t0: Optional[float] = None, t1: Optional[float] = None,
                rows: Optional[List[Row]] = None) -> Dict[str, Optional[float]]:
        """Mean / max over samples with t0 <= ts <= t1 (wall-clock seconds, time.time())."""
        with self._lock:
            src = list(self.rows if rows is None else rows)
        sel = [r for r in src if (t0 is None or r[0] >= t0) and (t1 is None or r[0] <= t1)]
        gfx = [r[2] for r in sel if r[2] >= 0]
        umc = [r[3] for r in sel if r[3] >= 0]
        vram = [r[4] for r in sel if r[4] >= 0]
        pw = [r[5] for r in sel if r[5] >= 0]

        def mean(v):
            return sum(v) / len(v) if v else None
        return {"samples": float(len(sel)),
                "gfx_activity_pct_mean": mean(gfx), "gfx_activity_pct_max": max(gfx) if gfx else None,
                "umc_activity_pct_mean": mean(umc),
                "vram_used_mb_max": max(vram) if vram else None, "vram_used_mb_mean": mean(vram),
                "power_w_mean": mean(pw)}


def now() -> float:
    """The sampler's clock (system wall clock, as the native sampler stamps rows)."""
    return time.time()
