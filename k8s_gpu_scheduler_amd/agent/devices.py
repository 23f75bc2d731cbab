"""Device enumeration sources for the node agent.

Reference: `parse_smi_uuids.py` runs `nvidia-smi -L`, regex-extracts UUIDs and prints
`MIG-<uuid>` / `GPU-<uuid>` (reference pkg/profiler/parse_smi_uuids.py:6-18).  On
MI355X the UUIDs, partitions, NUMA node and HBM size come from amd-smi through the
native `_smi` module; when amd-smi cannot initialise (no driver access in a container)
the HIP runtime device query (`_hip.query_all`, the gpu_profiling.cpp equivalent) is
used; `StaticSource` serves tests and the simulator.  Every source returns the same
descriptor dicts as `plugins.gpu.devices.Device.to_json()`.
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional

from ..api import constants as C

UUID_RE = re.compile(r"[a-f0-9]{8}-?[a-f0-9]{4}-?[a-f0-9]{4}-?[a-f0-9]{4}-?[a-f0-9]{12}", re.I)


def parse_smi_list(text: str) -> List[str]:
    """Reference-compatible parser for an `*-smi -L` style listing: one device per line,
    partition lines ('MIG'/'Partition') prefixed MIG-, others GPU-."""
    out = []
    for line in text.splitlines():
        m = UUID_RE.search(line)
        if m:
            part = "MIG" in line or "Partition" in line
            out.append(("MIG-" if part else "GPU-") + m.group(0))
    return out


class DeviceSource:
    name = "base"

    def devices(self) -> List[Dict[str, Any]]:
        raise NotImplementedError

    def topology(self) -> Optional[Dict[str, Any]]:
        return None

    def samples(self) -> List[Dict[str, Any]]:
        return []

    def processes(self, index: int) -> List[Dict[str, Any]]:
        return []

    def set_compute_partition(self, index: int, mode: str) -> str:
        return "unsupported"


class StaticSource(DeviceSource):
    name = "static"

    def __init__(self, descriptors: List[Dict[str, Any]], topology: Optional[Dict[str, Any]] = None,
                 samples: Optional[List[Dict[str, Any]]] = None):
        self.desc = list(descriptors)
        self.topo = topology
        self._samples = samples or []
        self.partition_calls: List[tuple] = []

    def devices(self):
        return [dict(d) for d in self.desc]

    def topology(self):
        return self.topo

    def samples(self):
        return list(self._samples)

    def set_compute_partition(self, index, mode):
        self.partition_calls.append((index, mode))
        parts = C.COMPUTE_PARTITIONS[mode]
        gpu = self.desc[index]["gpu"] if index < len(self.desc) else index
        rest = [d for d in self.desc if d["gpu"] != gpu]
        new = [{"uuid": f"GPU-{gpu:02d}{p:02d}0000-0000-0000-0000-{gpu:012d}", "gpu": gpu, "partition": p,
                "partitions": parts, "cus": C.MI355X_CUS // parts, "hbm_gib": C.MI355X_HBM_GIB / parts,
                "numa": 0 if gpu < 4 else 1, "model": C.MI355X, "first_xcd": 0} for p in range(parts)]
        self.desc = sorted(rest + new, key=lambda d: (d["gpu"], d["partition"]))
        return ""


def synthetic_node(n_gpus: int = 8, partition: str = "SPX", node: str = "node") -> StaticSource:
    parts = C.COMPUTE_PARTITIONS[partition]
    desc = []
    for g in range(n_gpus):
        for p in range(parts):
            desc.append({"uuid": f"GPU-{g:02d}{p:02d}{abs(hash(node)) % 10**4:04d}-0000-0000-0000-{g:012d}",
                         "gpu": g, "partition": p, "partitions": parts, "cus": C.MI355X_CUS // parts,
                         "hbm_gib": C.MI355X_HBM_GIB / parts, "numa": 0 if g < n_gpus // 2 else 1,
                         "model": C.MI355X, "first_xcd": 0})
    from ..plugins.gpu.topology import Topology
    return StaticSource(desc, Topology.fully_connected(n_gpus).to_json())


class SmiSource(DeviceSource):
    """amd-smi via the native `_smi` module."""
    name = "amd-smi"

    def __init__(self):
        from .. import _native
        mod = _native.smi()
        if mod is None:
            raise RuntimeError("_smi native module not built")
        self.smi = mod.Smi()
        if not self.smi.init():
            raise RuntimeError(f"amd-smi init failed: {self.smi.error()}")

    @staticmethod
    def _rocr_ids() -> Dict[str, List[str]]:
        """PCI BDF -> ROCr device ids ("GPU-<16 hex>", what ROCR_VISIBLE_DEVICES accepts) from
        the HIP runtime, in enumeration order; empty when HIP is unavailable."""
        try:
            from .. import _native
            h = _native.hip(required=False)
            if h is None:
                return {}
            ids: Dict[str, List[str]] = {}
            for d in h.query_all():
                if d.get("rocr_uuid"):
                    ids.setdefault(d.get("pci", "").lower(), []).append(d["rocr_uuid"])
            return ids
        except Exception:
            return {}

    def devices(self):
        out = []
        raw = self.smi.devices()
        rocr = self._rocr_ids()
        # partitions of one physical GPU share a BDF bus/device; count them per bus
        for d in raw:
            mode = (d.get("compute_partition") or "SPX").upper()
            parts = C.COMPUTE_PARTITIONS.get(mode, 1)
            ids = rocr.get(str(d.get("bdf", "")).lower()) or []
            uuid = ids.pop(0) if ids else "GPU-" + d.get("uuid", f"idx{d['index']}")
            out.append({"uuid": uuid, "smi_uuid": d.get("uuid", ""), "gpu": d["index"] // parts,
                        "partition": d["index"] % parts, "partitions": parts,
                        "cus": int(d.get("num_cu") or C.MI355X_CUS // parts),
                        "hbm_gib": float(d.get("vram_total_mb", C.MI355X_HBM_GIB * 1024 / parts)) / 1024.0,
                        "numa": int(d.get("numa", 0)), "model": C.MI355X if "355" in d.get("market_name", "MI355X")
                        else d.get("market_name", ""), "first_xcd": 0, "bdf": d.get("bdf", "")})
        return out

    def topology(self):
        return self.smi.topology()

    def samples(self):
        return self.smi.sample()

    def processes(self, index):
        return self.smi.processes(index)

    def set_compute_partition(self, index, mode):
        return self.smi.set_compute_partition(index, mode)


class HipSource(DeviceSource):
    """HIP runtime device query (no amd-smi): UUIDs, CUs, HBM."""
    name = "hip"

    def __init__(self):
        from .. import _native
        self.hip = _native.hip(required=True)

    def devices(self):
        out = []
        for d in self.hip.query_all():
            uuid = d.get("rocr_uuid") or "GPU-" + (d.get("uuid") or f"idx{d['index']}")
            out.append({"uuid": uuid, "gpu": d["index"], "partition": 0,
                        "partitions": 1, "cus": d["cus"], "hbm_gib": d["total_mem"] / 2**30,
                        "numa": 0, "model": C.MI355X if d["arch"].startswith("gfx950") else d["arch"],
                        "first_xcd": 0, "bdf": d.get("pci", "")})
        return out


def best_source() -> DeviceSource:
    for cls in (SmiSource, HipSource):
        try:
            src = cls()
            if src.devices():
                return src
        except Exception:
            continue
    return StaticSource([])
