"""Device inventory and the per-device reservation ledger.

The reference knows a node's devices only as a JSON list of UUIDs in Redis
(reference pkg/profiler/cmd/client/client.go:70-76) and assumes one physical GPU per node
(`<nUUIDs>P_<model>`).  An MI355X node has 8 GPUs, each optionally
split into SPX/DPX/QPX/CPX compute partitions, so the inventory here is a list of
`Device`s (physical index, partition index, CUs, HBM, NUMA), and the ledger accounts
fractional use in **CU-slice units**: a GPU is 8 units of 32 CUs, where unit u is
word u of the 256-bit HIP CU mask.  Measured on MI355X (tools/diag_gpu.py,
profiles/archive/diag_r01.json): in SPX mode mask bit i selects CU i//8 of XCC i%8, and a mask
that leaves any XCC without CUs is ignored by the driver, so a unit is 4 CUs on *every*
XCD (XCD isolation needs a real compute partition, DPX/QPX/CPX, which the agent applies
through amd-smi).  A fractional pod gets a contiguous, naturally aligned run of units
(buddy style) and its CU mask is exactly those words.
"""
from __future__ import annotations

import hashlib
import json
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional, Tuple

from ...api import constants as C
from ...api import objects as O

Obj = Dict[str, Any]
CUS_PER_XCD = C.MI355X_CUS // C.MI355X_XCDS     # 32


def synth_uuid(node: str, gpu: int, part: int = -1) -> str:
    h = hashlib.md5(f"{node}/{gpu}/{part}".encode()).hexdigest()
    u = f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:32]}"
    return f"GPU-{u}" if part < 0 else f"GPU-{u}"


@dataclass
class Device:
    uuid: str
    node: str
    gpu: int                    # physical GPU index on the node (0..7)
    partition: int = 0          # partition index inside the GPU
    partitions: int = 1         # partitions per GPU (SPX=1 .. CPX=8)
    cus: int = C.MI355X_CUS
    hbm_gib: float = float(C.MI355X_HBM_GIB)
    numa: int = 0
    model: str = C.MI355X
    units: int = 0              # XCD units (32 CUs each)
    first_xcd: int = 0          # first CU-slice unit of the GPU owned by this device
    healthy: bool = True        # agent health verdict (agent/health.py); unhealthy = not allocatable

    def __post_init__(self) -> None:
        if not self.units:
            self.units = max(1, self.cus // CUS_PER_XCD)

    def to_json(self) -> Dict[str, Any]:
        return {"uuid": self.uuid, "gpu": self.gpu, "partition": self.partition, "partitions": self.partitions,
                "cus": self.cus, "hbm_gib": self.hbm_gib, "numa": self.numa, "model": self.model,
                "first_xcd": self.first_xcd, "healthy": self.healthy}

    @classmethod
    def from_json(cls, node: str, d: Dict[str, Any]) -> "Device":
        return cls(uuid=d["uuid"], node=node, gpu=int(d.get("gpu", 0)), partition=int(d.get("partition", 0)),
                   partitions=int(d.get("partitions", 1)), cus=int(d.get("cus", C.MI355X_CUS)),
                   hbm_gib=float(d.get("hbm_gib", C.MI355X_HBM_GIB)), numa=int(d.get("numa", 0)),
                   model=d.get("model", C.MI355X), first_xcd=int(d.get("first_xcd", 0)),
                   healthy=bool(d.get("healthy", True)))


def devices_for_node(node: Obj, uuids: Optional[List[str]] = None,
                     descriptors: Optional[List[Dict[str, Any]]] = None) -> List[Device]:
    """Inventory of a node: from the agent's descriptors if published, else from the
    node labels (GPU count + compute partition), with Redis UUIDs (reference schema)
    assigned in order when given."""
    nm = O.name(node)
    bad = O.node_unhealthy_devices(node)
    if descriptors:
        out = [Device.from_json(nm, d) for d in descriptors]
        for d in out:
            if d.uuid in bad:
                d.healthy = False
        return out
    gpus = O.node_gpu_count(node)
    parts = O.node_partitions_per_gpu(node)
    model = O.node_gpu_model(node) or C.MI355X
    mem_parts = C.MEMORY_PARTITIONS.get(O.labels(node).get(C.LABEL_MEMORY_PARTITION, "NPS1"), 1)
    out: List[Device] = []
    i = 0
    for g in range(gpus):
        for p in range(parts):
            u = uuids[i] if uuids and i < len(uuids) else synth_uuid(nm, g, p if parts > 1 else -1)
            # NPS1: all partitions share the GPU's HBM; account an equal split so the
            # ledger never over-commits it.
            hbm = C.MI355X_HBM_GIB / max(parts, mem_parts)
            out.append(Device(u, nm, g, p, parts, C.MI355X_CUS // parts, hbm,
                              numa=0 if g < max(gpus // 2, 1) else 1, model=model,
                              first_xcd=0))   # a partition is its own HIP device: units restart at 0
            i += 1
    if uuids and len(uuids) > len(out) and not gpus:
        # Unlabelled node with UUIDs (reference-style): one device per UUID.
        out = [Device(u, nm, k, 0, 1) for k, u in enumerate(uuids)]
    for d in out:
        if d.uuid in bad:
            d.healthy = False
    return out


def cu_slice_mask(first_unit: int, n_units: int, cus: int = C.MI355X_CUS) -> List[int]:
    """CU mask (list of 32-bit words, bit i = logical CU i) for units [first_unit,
    first_unit+n_units): word u is all ones.  Each word covers CUs 4u..4u+3 of every one
    of the 8 XCCs (bit i -> XCC i % 8, CU i // 8 inside it; verified by
    ops.cumask.probe_xcd_map)."""
    words = [0] * ((cus + 31) // 32)
    for u in range(first_unit, min(first_unit + n_units, len(words))):
        words[u] = 0xFFFFFFFF
    return words



def hsa_cu_mask_ranges(words: List[int]) -> str:
    """Set bits of a CU mask as ROCr's HSA_CU_MASK range list ("0-31,64-95")."""
    bits = [32 * wi + b for wi, w in enumerate(words) for b in range(32) if (w >> b) & 1]
    out, start, prev = [], None, None
    for b in bits:
        if start is None:
            start = prev = b
        elif b == prev + 1:
            prev = b
        else:
            out.append(f"{start}-{prev}" if prev > start else str(start))
            start = prev = b
    if start is not None:
        out.append(f"{start}-{prev}" if prev > start else str(start))
    return ",".join(out)


def mask_to_hex(words: List[int]) -> str:
    """HSA_CU_MASK style: 0x<hex> with word 0 least significant."""
    v = 0
    for i, w in enumerate(words):
        v |= (w & 0xFFFFFFFF) << (32 * i)
    return hex(v)


@dataclass
class PodUse:
    key: str
    name: str
    slo: float
    cu: int
    hbm_gib: float
    units: Tuple[int, int]       # (first unit, count) inside the device
    whole: bool = False
    work: float = 0.0            # predicted whole-GPU seconds of this pod on this device
    iters: float = 0.0           # iterations a batch pod runs (0 = a long-running service): co-run model


@dataclass
class DeviceState:
    device: Device
    used_units: List[bool] = field(default_factory=list)
    hbm_used: float = 0.0
    pods: Dict[str, PodUse] = field(default_factory=dict)
    work: float = 0.0            # sum of the residents' predicted GPU time (PodUse.work)

    def __post_init__(self) -> None:
        if not self.used_units:
            self.used_units = [False] * self.device.units

    @property
    def free_units(self) -> int:
        return self.used_units.count(False)

    @property
    def hbm_free(self) -> float:
        return self.device.hbm_gib - self.hbm_used

    def find_units(self, n: int) -> Optional[int]:
        """Best-fit aligned run of n free units (alignment = next pow2 >= n); memoised
        until the unit map changes.  The memo is tagged with the state's version, which the
        ledger bumps before AND after every change, so a search that overlapped a
        concurrent reserve/release is never served from the memo afterwards."""
        d = self.__dict__
        ver = d.get("_ver", 0)
        cache = d.get("_fit")
        if cache is not None and cache[0] == ver and n in cache[1]:
            return cache[1][n]
        r = self._find_units(n)
        if cache is None or cache[0] != ver:
            cache = (ver, {})
            d["_fit"] = cache
        cache[1][n] = r
        return r

    def invalidate(self) -> None:
        d = self.__dict__
        d["_ver"] = d.get("_ver", 0) + 1
        d.pop("_fit", None)
        d.pop("_slo", None)     # plugin's resident summary (scoring.DeviceSummary)

    def _find_units(self, n: int) -> Optional[int]:
        if n > len(self.used_units):
            return None
        align = 1
        while align < n:
            align *= 2
        best, best_free_around = None, None
        for s in range(0, len(self.used_units) - n + 1, align):
            if not any(self.used_units[s:s + n]):
                # prefer placements inside the most-used aligned block (less fragmentation)
                blk = max(align * 2, 2)
                b0 = (s // blk) * blk
                free_in_blk = self.used_units[b0:b0 + blk].count(False)
                if best is None or free_in_blk < best_free_around:
                    best, best_free_around = s, free_in_blk
        return best


class DeviceLedger:
    """Per-node device reservations, updated by Reserve/Unreserve and informer events.
    Thread-safe; Score reads a consistent view under the lock."""

    def __init__(self) -> None:
        self._lock = threading.RLock()
        self.nodes: Dict[str, Dict[str, DeviceState]] = {}
        self.pod_index: Dict[str, Tuple[str, List[str]]] = {}     # pod key -> (node, uuids)
        self.generation = 0
        self.node_gen: Dict[str, int] = {}      # per-node change counter (Score memo key)
        from ...framework.changes import ChangeFanout
        self.changes = ChangeFanout()           # scheduling-cycle node-result caches

    def set_devices(self, node: str, devices: Iterable[Device]) -> None:
        with self._lock:
            old = self.nodes.get(node, {})
            new: Dict[str, DeviceState] = {}
            for d in devices:
                st = old.get(d.uuid)
                if st is not None and st.device.units == d.units:
                    st.device = d
                    new[d.uuid] = st
                else:
                    new[d.uuid] = DeviceState(d)
            self.nodes[node] = new
            self.generation += 1
            self.node_gen[node] = self.node_gen.get(node, 0) + 1
            self.changes.touch(node)

    def devices(self, node: str) -> List[DeviceState]:
        with self._lock:
            return list(self.nodes.get(node, {}).values())

    def has_node(self, node: str) -> bool:
        return node in self.nodes

    def reserve(self, node: str, pod_key: str, pod_name: str, slo: float,
                allocs: List[Tuple[str, int, int, float, bool]], work: float = 0.0, iters: float = 0.0) -> bool:
        """allocs: (uuid, first_unit, n_units, hbm_gib, whole).  All-or-nothing.  `work` is
        the pod's predicted GPU time (split evenly over its devices), summed per device for
        the plugin's load-balance term."""
        with self._lock:
            if pod_key in self.pod_index:
                self.release(pod_key)
            states = self.nodes.get(node, {})
            for uuid, u0, n, hbm, whole in allocs:
                st = states.get(uuid)
                if st is None or any(st.used_units[u0:u0 + n]) or u0 + n > len(st.used_units):
                    return False
                if hbm > st.hbm_free + 1e-6:
                    return False
            for uuid, u0, n, hbm, whole in allocs:
                st = states[uuid]
                st.invalidate()
                for u in range(u0, u0 + n):
                    st.used_units[u] = True
                st.hbm_used += hbm
                share = work / max(len(allocs), 1)
                st.pods[pod_key] = PodUse(pod_key, pod_name, slo, n * CUS_PER_XCD, hbm, (u0, n), whole, share, iters)
                st.work += share
                st.invalidate()
            self.pod_index[pod_key] = (node, [a[0] for a in allocs])
            self.generation += 1
            self.node_gen[node] = self.node_gen.get(node, 0) + 1
            self.changes.touch(node)
            return True

    def release(self, pod_key: str) -> bool:
        with self._lock:
            ent = self.pod_index.pop(pod_key, None)
            if ent is None:
                return False
            node, uuids = ent
            for uuid in uuids:
                st = self.nodes.get(node, {}).get(uuid)
                if st is None:
                    continue
                use = st.pods.pop(pod_key, None)
                if use is None:
                    continue
                u0, n = use.units
                st.invalidate()
                for u in range(u0, u0 + n):
                    st.used_units[u] = False
                st.hbm_used = max(0.0, st.hbm_used - use.hbm_gib)
                st.work = max(0.0, st.work - use.work) if st.pods else 0.0
                st.invalidate()
            self.generation += 1
            self.node_gen[node] = self.node_gen.get(node, 0) + 1
            self.changes.touch(node)
            return True

    def invalidate_summaries(self) -> None:
        """Drop every device's cached scoring summary (new prediction tables)."""
        with self._lock:
            for states in self.nodes.values():
                for st in states.values():
                    st.__dict__.pop("_slo", None)
            self.changes.touch_all()

    def gpu_work(self, node: str) -> Dict[int, float]:
        """Predicted GPU time of the pods resident on each physical GPU of a node (its
        partitions / fractional shares summed)."""
        with self._lock:
            out: Dict[int, float] = {}
            for st in self.nodes.get(node, {}).values():
                out[st.device.gpu] = out.get(st.device.gpu, 0.0) + st.work
            return out

    def placement(self, pod_key: str) -> Optional[Tuple[str, List[str]]]:
        with self._lock:
            return self.pod_index.get(pod_key)

    def snapshot_json(self) -> str:
        with self._lock:
            return json.dumps({n: {u: {"free_units": s.free_units, "hbm_used": s.hbm_used, "pods": list(s.pods)}
                                   for u, s in devs.items()} for n, devs in self.nodes.items()})
