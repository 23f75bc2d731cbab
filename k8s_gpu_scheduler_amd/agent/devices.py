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
from dataclasses import dataclass, field
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


# What an MI355X offers when nothing could be probed (synthetic nodes, tests): the four
# compute modes, NPS1 with every one of them and NPS2 with the split modes.
MI355X_PROFILES = [{"mode": "SPX", "partitions": 1, "memory_caps": ["NPS1"]},
                   {"mode": "DPX", "partitions": 2, "memory_caps": ["NPS1", "NPS2"]},
                   {"mode": "QPX", "partitions": 4, "memory_caps": ["NPS1", "NPS2"]},
                   {"mode": "CPX", "partitions": 8, "memory_caps": ["NPS1", "NPS2"]}]


@dataclass
class PartitionCaps:
    """Partition modes one GPU supports, from the read-only amd-smi probe
    (`_smi.partition_info`: accelerator partition profiles + memory partition config)."""
    current_compute: str = "SPX"
    current_memory: str = "NPS1"
    compute_modes: List[str] = field(default_factory=list)          # probed; empty = unknown
    memory_by_compute: Dict[str, List[str]] = field(default_factory=dict)
    memory_modes: List[str] = field(default_factory=list)
    probed: bool = False

    def check(self, compute: str, memory: Optional[str] = None) -> Optional[str]:
        """None if (compute, memory) may be applied, else why not.  Nothing is assumed: a
        GPU whose profiles could not be read accepts no change."""
        if not self.probed or not self.compute_modes:
            return "partition capabilities unknown (amd-smi profile query failed)"
        if compute not in self.compute_modes:
            return f"compute partition {compute} not supported (supported: {','.join(self.compute_modes)})"
        if memory:
            allowed = self.memory_by_compute.get(compute) or self.memory_modes
            if allowed and memory not in allowed:
                return f"memory partition {memory} not allowed with {compute} (allowed: {','.join(allowed)})"
        return None

    def to_json(self) -> Dict[str, Any]:
        return {"current_compute": self.current_compute, "current_memory": self.current_memory,
                "compute_modes": self.compute_modes, "memory_by_compute": self.memory_by_compute,
                "memory_modes": self.memory_modes, "probed": self.probed}

    @classmethod
    def from_json(cls, d: Dict[str, Any]) -> "PartitionCaps":
        return cls(d.get("current_compute", "SPX"), d.get("current_memory", "NPS1"), list(d.get("compute_modes", [])),
                   {k: list(v) for k, v in (d.get("memory_by_compute") or {}).items()},
                   list(d.get("memory_modes", [])), bool(d.get("probed", False)))


def partition_capabilities(info: Dict[str, Any]) -> PartitionCaps:
    """PartitionCaps from one `partition_info` dict (amd-smi or synthetic)."""
    profiles = [p for p in info.get("profiles") or [] if p.get("mode") in C.COMPUTE_PARTITIONS]
    caps = PartitionCaps(current_compute=str(info.get("compute_partition") or info.get("current_profile") or "SPX"),
                         current_memory=str(info.get("memory_partition") or "NPS1"))
    seen = []
    for p in profiles:
        if p["mode"] not in seen:
            seen.append(p["mode"])
        caps.memory_by_compute.setdefault(p["mode"], [])
        for m in p.get("memory_caps") or []:
            if m not in caps.memory_by_compute[p["mode"]]:
                caps.memory_by_compute[p["mode"]].append(m)
    caps.compute_modes = sorted(seen, key=lambda m: C.COMPUTE_PARTITIONS[m])
    caps.memory_modes = list(info.get("memory_caps") or sorted({m for v in caps.memory_by_compute.values() for m in v}))
    caps.probed = bool(profiles)
    return caps


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

    def set_memory_partition(self, index: int, mode: str) -> str:
        return "unsupported"

    def partition_info(self, index: int) -> Dict[str, Any]:
        """Read-only probe (see `partition_capabilities`); {} when unknown."""
        return {}


class StaticSource(DeviceSource):
    name = "static"

    def __init__(self, descriptors: List[Dict[str, Any]], topology: Optional[Dict[str, Any]] = None,
                 samples: Optional[List[Dict[str, Any]]] = None,
                 profiles: Optional[List[Dict[str, Any]]] = None, memory_partition: str = "NPS1"):
        self.desc = list(descriptors)
        self.topo = topology
        self._samples = samples or []
        # a source built without a sample list (synthetic nodes) has no telemetry at all: the
        # health monitor then has nothing to judge -- its devices must not turn "unresponsive"
        self.has_telemetry = samples is not None
        self.partition_calls: List[tuple] = []
        self.profiles = MI355X_PROFILES if profiles is None else profiles
        self.memory_partition = memory_partition
        # scripted per-process usage: device index -> [{"pid", "vram_bytes", ...}] (tests)
        self.procs: Dict[int, List[Dict[str, Any]]] = {}

    def processes(self, index):
        return [dict(p) for p in self.procs.get(index, [])]

    def partition_info(self, index):
        d = self.desc[index] if 0 <= index < len(self.desc) else {}
        mode = C.PARTITIONS_TO_MODE.get(int(d.get("partitions", 1)), "SPX")
        return {"compute_partition": mode, "memory_partition": self.memory_partition,
                "memory_caps": sorted({m for p in self.profiles for m in p["memory_caps"]}),
                "profiles": [dict(p) for p in self.profiles], "errors": {}}

    def set_memory_partition(self, index, mode):
        self.partition_calls.append((index, mode))
        if mode not in C.MEMORY_PARTITIONS:
            return "unknown mode"
        self.memory_partition = mode
        return ""

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

    def set_memory_partition(self, index, mode):
        return self.smi.set_memory_partition(index, mode)

    def partition_info(self, index):
        return self.smi.partition_info(index)


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
