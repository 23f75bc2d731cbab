"""Node agent (the reference's "profiler" DaemonSet, re-designed).

Reference behaviour: a bash loop runs `parse_smi_uuids.py` every 2 s
and, when the UUID list changed, pipes NODE/POD/NS/UUIDS into a Go client that filters
MIG UUIDs and `SET <nodeName> <json list>` in Redis
(reference pkg/profiler/profile_gpu.sh:3-13, pkg/profiler/cmd/client/client.go:23-80).

The MI355X agent is one process that, every `poll_s`:
  * enumerates devices/partitions (amd-smi -> HIP -> static) and, on change, publishes
    the reference key `<node>` = JSON UUID list plus the richer `gpusched:devices:<node>`
    descriptors and `gpusched:topology:<node>` xGMI link matrix;
  * samples telemetry and feeds the Prometheus exporter (+ optional TelemetryCache);
  * appends per-pod usage history (`gpusched:hist:<pod>`) for the recommender's resize
    loop, attributing GPU processes to pods through their cgroup;
  * reconciles compute partitioning: when the node label `amd.com/compute-partition`
    asks for a different mode, taint the node (`amd.com/partitioning=NoSchedule`), apply
    through amd-smi, republish, untaint -- asynchronous, never inside Score
    (fixes SURVEY.md §2.9 #3).
The reference's 4-line stdin protocol is kept as `publish_from_stdin`.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from typing import Any, Callable, Dict, List, Optional

from ..api import constants as C
from ..api import objects as O
from ..kube.client import KubeClient
from ..kube.resources import Resources
from ..store import schema
from ..store.resp import Redis
from .devices import DeviceSource
from .health import HealthMonitor

log = logging.getLogger(__name__)


def pod_of_pid(pid: int, proc: str = "/proc") -> Optional[str]:
    """Pod UID of a process from its cgroup path (kubepods...pod<uid>...)."""
    try:
        with open(f"{proc}/{pid}/cgroup") as f:
            txt = f.read()
    except OSError:
        return None
    import re
    m = re.search(r"pod([0-9a-f]{8}[-_][0-9a-f]{4}[-_][0-9a-f]{4}[-_][0-9a-f]{4}[-_][0-9a-f]{12})", txt)
    return m.group(1).replace("_", "-") if m else None


class NodeAgent:
    def __init__(self, node: str, redis: Redis, source: DeviceSource, client: Optional[KubeClient] = None,
                 poll_s: float = C.PROFILER_POLL_S, exporter: Any = None, telemetry: Any = None,
                 apply_partitions: bool = True, pod_resolver: Optional[Callable[[int], Optional[str]]] = None,
                 health: Optional[HealthMonitor] = None, evict_unhealthy: bool = False):
        self.node, self.redis, self.source, self.client = node, redis, source, client
        self.poll_s = poll_s
        self.exporter = exporter
        self.telemetry = telemetry
        self.apply_partitions = apply_partitions
        self.pod_resolver = pod_resolver or pod_of_pid
        self.prev_uuids: Optional[List[str]] = None
        self.publishes = 0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.partition_state = "idle"
        self.health = health or HealthMonitor()
        # Evict the pods of a device that turned unhealthy (their controllers recreate them
        # and the scheduler places them elsewhere -- the elastic-recovery path); off by
        # default, as with Kubernetes device plugins
        self.evict_unhealthy = evict_unhealthy
        self.evicted: List[str] = []
        self.on_inventory_change: List[Callable[[], None]] = []    # e.g. the device plugin's changed()

    # ------------------------------------------------------------------ publish
    def inventory(self) -> List[Dict[str, Any]]:
        """Device descriptors with the current health verdicts (what publish() writes and
        what the kubelet device plugin advertises)."""
        devs = self.source.devices()
        for d in devs:
            d["healthy"] = self.health.healthy(d["uuid"])
        return devs

    def publish(self, force: bool = False) -> bool:
        devs = self.inventory()
        uuids = [d["uuid"] for d in devs]
        if not force and uuids == self.prev_uuids:
            return False
        schema.publish_uuids(self.redis, self.node, uuids)
        schema.publish_devices(self.redis, self.node, devs)
        topo = self.source.topology()
        if topo:
            self.redis.set(schema.topology_key(self.node), json.dumps(topo, separators=(",", ":")))
        self.prev_uuids = uuids
        self.publishes += 1
        for cb in self.on_inventory_change:
            try:
                cb()
            except Exception as e:
                log.warning("inventory-change callback failed: %s", e)
        log.info("published %d devices for %s", len(uuids), self.node)
        return True

    # ------------------------------------------------------------------ telemetry
    def sample(self) -> List[Dict[str, Any]]:
        samples = self.source.samples()
        devs = self.source.devices()
        idx_uuid = {i: d["uuid"] for i, d in enumerate(devs)}
        if self.exporter is not None and samples:
            self.exporter.observe_samples(samples, idx_uuid)
        if self.telemetry is not None:
            from ..telemetry.cache import DeviceSample
            for s in samples:
                u = idx_uuid.get(int(s.get("index", 0)))
                if u:
                    self.telemetry.update(self.node, u, DeviceSample(
                        gfx_activity=max(0.0, float(s.get("gfx_activity", 0))) / 100.0,
                        umc_activity=max(0.0, float(s.get("umc_activity", 0))) / 100.0,
                        vram_used_mb=float(s.get("vram_used_mb", 0)),
                        vram_total_mb=float(s.get("vram_total_mb", C.MI355X_HBM_GIB * 1024)),
                        power_w=float(s.get("power_w", 0)), temp_c=float(s.get("temp_c", 0)),
                        xgmi_tx_bps=float(s.get("xgmi_write_bps", 0)), xgmi_rx_bps=float(s.get("xgmi_read_bps", 0))))
        return samples

    def check_health(self, samples: Optional[List[Dict[str, Any]]] = None) -> bool:
        """Health verdicts from the latest samples; on a transition republish the
        descriptors, update the node annotation (the schedulers' change trigger) and,
        with evict_unhealthy, delete the pods assigned to newly failed devices."""
        if samples is None:
            samples = self.source.samples()
        before = self.health.unhealthy()
        devs = self.source.devices()
        changed = self.health.update(samples, devs)
        if self.exporter is not None:
            self.exporter.observe_health({i: self.health.healthy(d["uuid"]) for i, d in enumerate(devs)},
                                         {i: d["uuid"] for i, d in enumerate(devs)})
        if not changed:
            return False
        bad = self.health.unhealthy()
        self.publish(force=True)
        if self.client is not None:
            try:
                self.client.patch("nodes", self.node, {"metadata": {"annotations": {
                    C.ANNOT_UNHEALTHY: json.dumps(bad, sort_keys=True, separators=(",", ":"))}}}, "merge")
            except Exception as e:
                log.warning("health annotation on %s failed: %s", self.node, e)
            newly = set(bad) - set(before)
            if self.evict_unhealthy and newly:
                self._evict_on(newly)
        log.warning("device health on %s changed: %s", self.node, bad or "all healthy")
        return True

    def _evict_on(self, uuids: set) -> None:
        try:
            pods, _ = self.client.list("pods", field_selector=f"spec.nodeName={self.node}")
        except Exception as e:
            log.warning("listing pods for eviction failed: %s", e)
            return
        for p in pods:
            assigned = set(filter(None, O.annotations(p).get(C.ANNOT_DEVICES, "").split(",")))
            if assigned & uuids and not O.is_terminal(p):
                try:
                    self.client.delete("pods", O.name(p), O.namespace(p))
                    self.evicted.append(O.key(p))
                except Exception as e:
                    log.warning("evicting %s failed: %s", O.key(p), e)

    def record_history(self, uid_to_pod: Optional[Dict[str, str]] = None) -> int:
        """Per-pod usage samples from the per-process list (VRAM, CU occupancy)."""
        n = 0
        uid_to_pod = uid_to_pod or {}
        for i, d in enumerate(self.source.devices()):
            for p in self.source.processes(i):
                uid = self.pod_resolver(int(p.get("pid", 0)))
                pod = uid_to_pod.get(uid or "", uid)
                if not pod:
                    continue
                schema.append_history(self.redis, pod, {
                    "ts": time.time(), "device": d["uuid"], "hbm_gib": p.get("vram_bytes", 0) / 2**30,
                    "cu_busy": min(1.0, p.get("cu_occupancy", 0) / max(d.get("cus", C.MI355X_CUS), 1)),
                    "cu": d.get("cus", C.MI355X_CUS)})
                n += 1
        return n

    # ------------------------------------------------------------------ partitions
    def desired_partition(self) -> Optional[str]:
        if self.client is None:
            return None
        try:
            node = self.client.get("nodes", self.node)
        except Exception:
            return None
        return O.labels(node).get(C.LABEL_COMPUTE_PARTITION)

    def current_partition(self) -> str:
        devs = self.source.devices()
        parts = max((d.get("partitions", 1) for d in devs), default=1)
        return C.PARTITIONS_TO_MODE.get(parts, "SPX")

    def reconcile_partitions(self) -> bool:
        want = self.desired_partition()
        if not want or want.upper() not in C.COMPUTE_PARTITIONS or not self.apply_partitions:
            return False
        want = want.upper()
        if want == self.current_partition():
            return False
        res = Resources(self.client, "default")
        self.partition_state = f"applying {want}"
        res.taint_node(self.node, C.TAINT_PARTITIONING, want, "NoSchedule")
        self.redis.set(schema.partition_key(self.node), json.dumps({"state": "applying", "mode": want}))
        errs = []
        gpus = sorted({d["gpu"] for d in self.source.devices()})
        for g in gpus:
            idx = next(i for i, d in enumerate(self.source.devices()) if d["gpu"] == g)
            e = self.source.set_compute_partition(idx, want)
            if e:
                errs.append(f"gpu{g}: {e}")
        self.publish(force=True)
        res.untaint_node(self.node, C.TAINT_PARTITIONING)
        self.redis.set(schema.partition_key(self.node), json.dumps(
            {"state": "failed" if errs else "applied", "mode": want, "errors": errs}))
        self.partition_state = "idle"
        if errs:
            log.warning("partitioning %s to %s: %s", self.node, want, errs)
        return not errs

    # ------------------------------------------------------------------ loop
    def step(self) -> None:
        try:
            self.reconcile_partitions()
        except Exception as e:
            log.warning("partition reconcile failed: %s", e)
        self.publish()
        samples = self.sample()
        try:
            self.check_health(samples)
        except Exception as e:
            log.warning("health check failed: %s", e)

    def run(self) -> None:
        while not self._stop.is_set():
            try:
                self.step()
            except Exception as e:      # Redis/apiserver blips: keep looping
                log.warning("agent step failed: %s", e)
            self._stop.wait(self.poll_s)

    def start(self) -> "NodeAgent":
        self._thread = threading.Thread(target=self.run, daemon=True, name="node-agent")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)


def publish_from_stdin(lines: List[str], redis: Redis) -> str:
    """The reference's stdin protocol: NODE, POD, NS, "['uuid', ...]"
    (reference pkg/profiler/cmd/client/client.go:24-46, test.sh)."""
    node = lines[0].strip()
    raw = lines[3] if len(lines) > 3 else ""
    for ch in "'[] ":
        raw = raw.replace(ch, "")
    uuids = [u for u in raw.split(",") if u]
    return schema.publish_uuids(redis, node, uuids)
