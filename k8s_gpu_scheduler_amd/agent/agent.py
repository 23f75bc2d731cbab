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
  * reconciles partitioning: when the node label `amd.com/compute-partition` (and/or
    `amd.com/memory-partition`) asks for a different mode, check the mode against the
    read-only amd-smi capability probe (published as the node annotation
    `partition-caps`), check that the GPUs are idle (no process in amd-smi's process list,
    no pod bound to the node) -- tainting `amd.com/partitioning=NoSchedule` meanwhile so
    the node drains, and giving up after `drain_timeout_s` -- then apply through amd-smi
    (memory mode first), republish, untaint.  Asynchronous, never inside Score (fixes
    SURVEY.md §2.9 #2-#4); every outcome is recorded in the node annotation
    `partition-state` and the Redis key `gpusched:partition:<node>`.
The reference's 4-line stdin protocol is kept as `publish_from_stdin`.
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api import constants as C
from ..api import objects as O
from ..kube.client import KubeClient
from ..kube.resources import Resources
from ..store import schema
from ..store.resp import Redis
from .devices import DeviceSource, PartitionCaps, partition_capabilities
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
                 health: Optional[HealthMonitor] = None, evict_unhealthy: bool = False,
                 drain_timeout_s: float = 300.0, evict_hbm_overuse: bool = False, history_every: int = 1,
                 hbm_tolerance_gib: float = 0.5, host_proc: str = "/host/proc", profile_dir: str = "",
                 partition_dry_run: bool = False, fabric: Any = None, set_checks: Any = None,
                 background_probes: bool = False,
                 corun_send: Optional[Callable[[List[Dict[str, Any]]], Any]] = None,
                 busy_poll_s: float = 0.1):
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
        self.drain_timeout_s = drain_timeout_s
        self._drain_since: Optional[float] = None
        self._caps_published: Optional[str] = None
        self._overuse_published: Optional[str] = None
        self._overuse_flagged: set = set()
        self.evict_hbm_overuse = evict_hbm_overuse
        # slack over a pod's HBM cap before it counts as overuse: amd-smi's per-process VRAM
        # includes the HIP runtime's own allocations (~0.3 GiB per process on MI355X), which
        # the pod's amd.com/gpu-memory request does not -- the tolerance must cover them
        self.hbm_tolerance_gib = hbm_tolerance_gib
        self.host_proc = host_proc
        # dry run: a partition request goes through every check (capabilities, idleness) but
        # instead of calling amd-smi the agent records the exact calls it would make
        # (node annotation partition-state "dry-run", `dry_run_calls`)
        self.partition_dry_run = partition_dry_run
        # measured per-pair xGMI copy rates (agent.fabric.FabricProber), published with the
        # topology for the multi-GPU placement
        self.fabric = fabric
        # background_probes: the fabric probe and the RCCL checks of multi-GPU pods' GPU sets
        # (set_checks, agent.probes.SetChecker) run on their own thread with the node tainted
        # (agent.probes.ProbeWorker); otherwise the fabric probe runs inside step()
        self.probes = None
        if background_probes or set_checks is not None:
            from .probes import ProbeWorker
            self.probes = ProbeWorker(self, set_checks)
        self.dry_run_calls: List[Dict[str, Any]] = []
        # per-pod rocprofv3 output the profiling webhook (agent.profile_webhook) routes to a
        # hostPath: finished runs become workload-history samples (pod_profiler.ProfileIngestor)
        self.profiles = None
        self.corun = None
        if profile_dir:
            from ..recommender.admission import RedisHistory
            from .pod_profiler import ProfileIngestor
            # co-run observations from the traces (agent.corun_observer): pods that overlapped
            # on one device, sent to the recommender's online co-run model
            self.corun = None
            if corun_send is not None:
                from .corun_observer import CorunObserver
                self.corun = CorunObserver(corun_send, running_on=self._running_on if client is not None else None,
                                           finished_on=self._finished_on if client is not None else None)
            self.profiles = ProfileIngestor(profile_dir, RedisHistory(redis), node=node, corun=self.corun,
                                            pod_lookup=self._pod_lookup if client is not None else None)
        self.history_every = max(1, history_every)
        self._steps = 0
        # per-pod GPU busy time from amd-smi's per-process engine counters (or a profiled
        # pod's trace), written as the busy-ms annotation when the pod terminates
        # (agent.busy; the completion feedback's millisecond measurement)
        from .busy import BusyTracker
        self.busy = BusyTracker()
        # the busy sampler's own period (its thread, started with the agent): the occupancy
        # integral's resolution; 0 = sample only in step()
        self.busy_poll_s = busy_poll_s
        self._busy_query_s = 0.0          # EMA of one process-list round's own duration
        self._busy_thread: Optional[threading.Thread] = None
        if self.profiles is not None:
            self.profiles.on_busy = self.busy.note_profiled
        # this node's pods, listed once per step and shared by every user of the step (the
        # usage attribution, the busy-ms pass, the co-run observer's lookups)
        self._pod_cache: Optional[List[Dict[str, Any]]] = None
        self._in_step = False
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
        self.publish_topology()
        self.prev_uuids = uuids
        self.publishes += 1
        for cb in self.on_inventory_change:
            try:
                cb()
            except Exception as e:
                log.warning("inventory-change callback failed: %s", e)
        log.info("published %d devices for %s", len(uuids), self.node)
        return True

    def publish_topology(self) -> None:
        """`gpusched:topology:<node>`: the static link matrix plus, once probed, the measured
        per-pair bandwidth (`bw_gbps`)."""
        topo = self.source.topology()
        last = self.fabric.last if self.fabric is not None else None
        if last and last.get("bw_gbps"):
            topo = dict(topo or {"n": len(last["bw_gbps"])})
            topo["bw_gbps"] = last["bw_gbps"]
        sets = self.probes.sets if self.probes is not None else None
        if sets is not None and sets.results:
            topo = dict(topo or {"n": len(self.source.devices())})
            topo["set_checks"] = sets.to_json()
            topo["bad_sets"] = sets.bad_sets()
        if topo:
            self.redis.set(schema.topology_key(self.node), json.dumps(topo, separators=(",", ":")))

    def probe_fabric(self) -> bool:
        """Measure the fabric when due and the GPUs are idle; republish the topology."""
        if self.fabric is None:
            return False
        res = self.fabric.maybe_probe(self.busy_reasons)
        if res is None:
            return False
        from .fabric import degraded_pairs
        bad = degraded_pairs(res.get("bw_gbps") or [])
        if bad:
            log.warning("fabric on %s: degraded GPU pairs %s", self.node, bad)
        self.publish_topology()
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
        if not samples and not getattr(self.source, "has_telemetry", True):
            return False                     # no telemetry source: no verdicts to reach
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

    def _node_pods(self) -> List[Dict[str, Any]]:
        """Every pod bound to this node (any phase): one LIST per agent step, shared by the
        step's users; outside a step a fresh LIST.  Raises on apiserver errors."""
        if self._in_step and self._pod_cache is not None:
            return self._pod_cache
        pods, _ = self.client.list("pods", field_selector=f"spec.nodeName={self.node}")
        if self._in_step:
            self._pod_cache = pods
        if self.profiles is not None and hasattr(self.profiles, "note_pods"):
            self.profiles.note_pods(pods)
        return pods

    def _pods_on_node(self) -> Dict[str, Dict[str, Any]]:
        """uid -> pod object of the non-terminal pods bound to this node ({} without apiserver)."""
        if self.client is None:
            return {}
        try:
            pods = self._node_pods()
        except Exception as e:
            log.debug("listing pods on %s failed: %s", self.node, e)
            return {}
        return {O.uid(p): p for p in pods if not O.is_terminal(p) and O.uid(p)}

    def sample_busy(self) -> None:
        """One busy-time sampling round over the attributed processes (agent.busy).  An interval
        counts at most 2.5 sampling periods, where the period is the poll wait plus the process
        query's own (averaged) duration: amd-smi's process list can take longer than the poll
        wait on a loaded node, and capping at twice the wait alone dropped a quarter of a pod's
        busy time on MI355X (1,480 vs 2,002 ms); a sampler stalled well past its period still
        does not count its stall."""
        try:
            wait = max(self.busy_poll_s, 0.05) if self._busy_thread is not None else self.poll_s
            gap = 2.5 * (wait + self._busy_query_s)
            t0 = time.monotonic()
            self.busy.sample(self.source, self.pod_resolver, len(self.source.devices()), max_gap_s=gap)
            dt = time.monotonic() - t0
            self._busy_query_s = dt if self._busy_query_s == 0.0 else 0.8 * self._busy_query_s + 0.2 * dt
        except Exception as e:
            log.debug("process list for busy time failed: %s", e)

    def _busy_loop(self) -> None:
        while not self._stop.is_set():
            self.sample_busy()
            self._stop.wait(self.busy_poll_s)

    def start_busy_sampler(self) -> None:
        if self.busy_poll_s > 0 and self._busy_thread is None:
            self._busy_thread = threading.Thread(target=self._busy_loop, daemon=True, name="busy-sampler")
            self._busy_thread.start()

    def track_busy(self) -> List[str]:
        """Write busy-ms on this node's pods that have terminated since (agent.busy), after a
        sampling round when no sampler thread runs.  Returns the pods annotated."""
        if self._busy_thread is None:
            self.sample_busy()
        if self.client is None or not self.busy.tracked():
            return []
        done = self.busy.annotate_finished(self.client, self._node_pods())
        self.busy.expire()
        return done

    def pod_usage(self, uid_to_pod: Optional[Dict[str, str]] = None) -> Dict[str, Dict[str, Any]]:
        """Per-pod GPU usage from amd-smi's per-process list: processes are attributed to
        pods through their cgroup (pod_resolver), VRAM summed over a pod's processes and
        devices.  Keyed by "ns/name"; `uid_to_pod` overrides the apiserver lookup."""
        pods = self._pods_on_node() if uid_to_pod is None else {}
        out: Dict[str, Dict[str, Any]] = {}
        for i, d in enumerate(self.source.devices()):
            for p in self.source.processes(i):
                uid = self.pod_resolver(int(p.get("pid", 0)))
                if not uid:
                    continue
                obj = pods.get(uid)
                key = (uid_to_pod or {}).get(uid) or (O.key(obj) if obj is not None else None)
                if not key:
                    continue
                u = out.setdefault(key, {"pod": obj, "hbm_gib": 0.0, "cu_busy": 0.0, "devices": [], "pids": [],
                                         "cus": d.get("cus", C.MI355X_CUS)})
                u["hbm_gib"] += float(p.get("vram_bytes", 0)) / 2**30
                u["cu_busy"] = max(u["cu_busy"], min(1.0, float(p.get("cu_occupancy", 0)) /
                                                     max(d.get("cus", C.MI355X_CUS), 1)))
                if d["uuid"] not in u["devices"]:
                    u["devices"].append(d["uuid"])
                u["pids"].append(int(p.get("pid", 0)))
                if "throughput" in p:           # executors that know their pods' rate report it
                    u["throughput"] = float(p["throughput"])
        return out

    def record_history(self, uid_to_pod: Optional[Dict[str, str]] = None,
                       usage: Optional[Dict[str, Dict[str, Any]]] = None) -> int:
        """Append one usage sample per running pod to its history in Redis -- keyed by the
        pod's WORKLOAD (recommender.admission.workload_key), which is what the resize
        admission reads; `uid_to_pod` (tests / no apiserver) keys by the given name."""
        from ..recommender.admission import workload_key
        usage = self.pod_usage(uid_to_pod) if usage is None else usage
        n = 0
        for key, u in usage.items():
            pod = u.get("pod")
            hist_key = workload_key(pod) if pod is not None else key
            _, cu_req, _ = O.gpu_request(pod) if pod is not None else (0, 0, 0.0)
            sample = {"ts": time.time(), "pod": key, "device": ",".join(u["devices"]), "hbm_gib": u["hbm_gib"],
                      "cu_busy": u["cu_busy"], "cu": int(cu_req or u.get("cus", C.MI355X_CUS)), "source": "agent"}
            if "throughput" in u:
                sample["throughput"] = u["throughput"]
            schema.append_history(self.redis, hist_key, sample)
            n += 1
        return n

    def check_hbm(self, usage: Optional[Dict[str, Dict[str, Any]]] = None, tolerance_gib: Optional[float] = None,
                  evict: Optional[bool] = None) -> Dict[str, Dict[str, float]]:
        """HBM share enforcement by detection (the driver does not cap a process's VRAM the
        way MPS's CUDA_MPS_PINNED_DEVICE_MEM_LIMIT does, reference gpu_plugins.go:896-903):
        a pod whose processes hold more VRAM than its cap -- its amd.com/gpu-memory request
        (= the GPU_SCHED_HBM_LIMIT_GIB the scheduler gave it) -- is flagged in the node
        annotation `hbm-overuse`, the exporter gauge `amd_gpu_pod_hbm_overuse` and a Warning
        event, and with `evict_hbm_overuse` evicted through the Eviction API (PodDisruptionBudgets
        apply; its controller recreates it).  A pod is marked handled only once its event (and,
        when evicting, its eviction) went through, so a failed attempt is retried next step
        while the pod keeps overusing."""
        usage = self.pod_usage() if usage is None else usage
        evict = self.evict_hbm_overuse if evict is None else evict
        tolerance_gib = self.hbm_tolerance_gib if tolerance_gib is None else tolerance_gib
        over: Dict[str, Dict[str, float]] = {}
        for key, u in usage.items():
            pod = u.get("pod")
            cap = O.gpu_request(pod)[2] if pod is not None else float(u.get("cap_gib", 0.0))
            if self.exporter is not None:
                self.exporter.observe_pod_hbm(key, u["hbm_gib"], cap)
            if cap > 0 and u["hbm_gib"] > cap + tolerance_gib:
                over[key] = {"used_gib": round(u["hbm_gib"], 3), "cap_gib": cap}
        raw = json.dumps(over, sort_keys=True, separators=(",", ":"))
        if raw != self._overuse_published and self.client is not None:
            try:
                self.client.patch("nodes", self.node, {"metadata": {"annotations": {C.ANNOT_HBM_OVERUSE: raw}}},
                                  "merge")
                self._overuse_published = raw
            except Exception as e:
                log.warning("hbm-overuse annotation on %s failed: %s", self.node, e)
        handled = self._overuse_flagged & set(over)         # still over, already handled
        for key in set(over) - self._overuse_flagged:
            pod = usage[key].get("pod")
            msg = f"HBM {over[key]['used_gib']:.2f} GiB exceeds the pod's {over[key]['cap_gib']:g} GiB share"
            log.warning("%s: %s", key, msg)
            if pod is None or self.client is None:
                handled.add(key)
                continue
            try:
                self.client.create_event(pod, "GPUMemoryOveruse", msg, "Warning")
                if evict:
                    self.client.evict(O.namespace(pod), O.name(pod))
                    self.evicted.append(key)
                handled.add(key)
            except Exception as e:              # retried at the next step
                log.warning("%s %s failed: %s", "evicting" if evict else "flagging", key, e)
        self._overuse_flagged = handled
        return over

    # ------------------------------------------------------------------ partitions
    def desired_partition(self) -> Optional[str]:
        return self.desired_partitions()[0]

    def desired_partitions(self) -> Tuple[Optional[str], Optional[str]]:
        """(compute mode, memory mode) the node labels ask for (None = unset / unreadable)."""
        if self.client is None:
            return None, None
        try:
            node = self.client.get("nodes", self.node)
        except Exception:
            return None, None
        lab = O.labels(node)
        c = (lab.get(C.LABEL_COMPUTE_PARTITION) or "").upper() or None
        m = (lab.get(C.LABEL_MEMORY_PARTITION) or "").upper() or None
        return c, m

    def current_partition(self) -> str:
        devs = self.source.devices()
        parts = max((d.get("partitions", 1) for d in devs), default=1)
        return C.PARTITIONS_TO_MODE.get(parts, "SPX")

    def _gpu_indices(self) -> Dict[int, int]:
        """physical GPU -> index of its first device (partition) in the source."""
        out: Dict[int, int] = {}
        for i, d in enumerate(self.source.devices()):
            out.setdefault(int(d.get("gpu", i)), i)
        return out

    def partition_caps(self) -> Optional[PartitionCaps]:
        """What every GPU of the node supports (intersection of the per-GPU probes)."""
        caps: Optional[PartitionCaps] = None
        for idx in self._gpu_indices().values():
            c = partition_capabilities(self.source.partition_info(idx) or {})
            if caps is None:
                caps = c
                continue
            caps.probed = caps.probed and c.probed
            caps.compute_modes = [m for m in caps.compute_modes if m in c.compute_modes]
            for m in list(caps.memory_by_compute):
                caps.memory_by_compute[m] = [x for x in caps.memory_by_compute[m] if x in c.memory_by_compute.get(m, [])]
            caps.memory_modes = [m for m in caps.memory_modes if m in c.memory_modes]
        return caps

    def publish_caps(self, force: bool = False) -> None:
        """Node annotation + Redis key with the probed capabilities (read by the controller)."""
        caps = self.partition_caps()
        if caps is None:
            return
        raw = json.dumps(caps.to_json(), sort_keys=True, separators=(",", ":"))
        if raw == self._caps_published and not force:
            return
        self.redis.set(schema.partition_caps_key(self.node), raw)
        if self.client is not None:
            try:
                self.client.patch("nodes", self.node, {"metadata": {"annotations": {C.ANNOT_PARTITION_CAPS: raw}}},
                                  "merge")
            except Exception as e:
                log.warning("partition-caps annotation on %s failed: %s", self.node, e)
                return
        self._caps_published = raw

    def _is_own_process(self, host_pid: int) -> bool:
        """Does a host PID (what amd-smi reports) belong to this agent's container?  Its PID
        namespace hides the host PID from os.getpid(), so the match is by cgroup: the host
        process's /host/proc/<pid>/cgroup equals our own /proc/self/cgroup.  Without the host
        proc mount only a same-namespace PID compare is possible."""
        if host_pid == os.getpid():
            return True
        try:
            with open(os.path.join(self.host_proc, str(host_pid), "cgroup")) as f:
                theirs = f.read()
            with open("/proc/self/cgroup") as f:
                mine = f.read()
        except OSError:
            return False
        return bool(mine.strip()) and theirs == mine

    def busy_reasons(self) -> List[str]:
        """Why the GPUs are not idle: processes in amd-smi's list (other than this agent's
        own) and non-terminal GPU pods bound to the node.  Empty = safe to repartition."""
        out = []
        for i, d in enumerate(self.source.devices()):
            for p in self.source.processes(i):
                if not self._is_own_process(int(p.get("pid", 0))):
                    out.append(f"gpu{d.get('gpu', i)}: pid {p.get('pid')} ({p.get('name', '?')})")
        if self.client is not None:
            try:
                pods, _ = self.client.list("pods", field_selector=f"spec.nodeName={self.node}")
            except Exception as e:
                return out + [f"cannot list pods on the node: {e}"]
            for p in pods:
                if not O.is_terminal(p) and (O.wants_gpu(p) or O.annotations(p).get(C.ANNOT_DEVICES)):
                    out.append(f"pod {O.key(p)}")
        return out

    def _set_partition_state(self, state: str, **kw: Any) -> None:
        doc = {"state": state, "ts": time.time(), **kw}
        raw = json.dumps(doc, sort_keys=True, separators=(",", ":"))
        self.partition_state = state
        self.redis.set(schema.partition_key(self.node), raw)
        if self.client is not None:
            try:
                self.client.patch("nodes", self.node, {"metadata": {"annotations": {C.ANNOT_PARTITION_STATE: raw}}},
                                  "merge")
            except Exception as e:
                log.warning("partition-state annotation on %s failed: %s", self.node, e)

    def _revert_request(self, cur_c: str, cur_m: str) -> None:
        """Set the labels back to what the node runs, so a refused request is not retried."""
        try:
            self.client.patch("nodes", self.node, {"metadata": {"labels": {
                C.LABEL_COMPUTE_PARTITION: cur_c, C.LABEL_MEMORY_PARTITION: cur_m}}}, "merge")
        except Exception as e:
            log.warning("reverting the partition labels of %s failed: %s", self.node, e)

    def reconcile_partitions(self) -> bool:
        """One reconcile pass; True when a change was applied successfully."""
        if not self.apply_partitions or self.client is None:
            return False
        want_c, want_m = self.desired_partitions()
        if want_c is not None and want_c not in C.COMPUTE_PARTITIONS:
            want_c = None
        if want_m is not None and want_m not in C.MEMORY_PARTITIONS:
            want_m = None
        caps = self.partition_caps()
        cur_c = self.current_partition()
        cur_m = caps.current_memory if caps is not None else "NPS1"
        if (want_c is None or want_c == cur_c) and (want_m is None or want_m == cur_m):
            if self._drain_since is not None:       # request withdrawn while draining
                self._drain_since = None
                Resources(self.client, "default").untaint_node(self.node, C.TAINT_PARTITIONING)
                self._set_partition_state("idle", mode=cur_c, memory=cur_m)
            return False
        target_c, target_m = want_c or cur_c, want_m or cur_m
        why = caps.check(target_c, target_m) if caps is not None else "no GPU to partition"
        if why:
            log.warning("partition request %s/%s on %s refused: %s", target_c, target_m, self.node, why)
            self._set_partition_state("refused", mode=target_c, memory=target_m, reason=why)
            self._revert_request(cur_c, cur_m)
            return False
        res = Resources(self.client, "default")
        busy = self.busy_reasons()
        if busy:
            now = time.monotonic()
            if self._drain_since is None:
                self._drain_since = now
                res.taint_node(self.node, C.TAINT_PARTITIONING, target_c, "NoSchedule")   # drain: no new pods
            if now - self._drain_since > self.drain_timeout_s:
                self._drain_since = None
                res.untaint_node(self.node, C.TAINT_PARTITIONING)
                self._set_partition_state("refused", mode=target_c, memory=target_m,
                                          reason="GPUs not idle: " + "; ".join(busy[:8]))
                self._revert_request(cur_c, cur_m)
            else:
                self._set_partition_state("waiting-idle", mode=target_c, memory=target_m, busy=busy[:8])
            return False
        self._drain_since = None
        if self.partition_dry_run:
            calls = []
            for step, mode, cur, fn in (("memory", target_m, cur_m, "amdsmi_set_gpu_memory_partition"),
                                        ("compute", target_c, cur_c, "amdsmi_set_gpu_compute_partition")):
                if mode != cur:
                    for g in sorted(self._gpu_indices()):
                        calls.append({"gpu": g, "device_index": self._gpu_indices()[g], "call": fn, "mode": mode})
            if calls != self.dry_run_calls:
                self.dry_run_calls = calls
                log.info("partition dry run on %s: %s", self.node, calls)
                self._set_partition_state("dry-run", mode=target_c, memory=target_m, calls=calls)
            return False
        res.taint_node(self.node, C.TAINT_PARTITIONING, target_c, "NoSchedule")
        self._set_partition_state("applying", mode=target_c, memory=target_m)
        errs: List[str] = []
        for step, mode, cur, fn in (("memory", target_m, cur_m, self.source.set_memory_partition),
                                    ("compute", target_c, cur_c, self.source.set_compute_partition)):
            if mode == cur:
                continue
            for g in sorted(self._gpu_indices()):
                idx = self._gpu_indices()[g]      # re-read: a change re-enumerates the devices
                e = fn(idx, mode)
                if e:
                    errs.append(f"gpu{g} {step} {mode}: {e}")
            if errs:
                break                   # never apply the compute mode after a failed memory change
        if self.fabric is not None:
            self.fabric.invalidate()            # partitions changed: re-measure when idle
        self.publish(force=True)
        self.publish_caps(force=True)
        res.untaint_node(self.node, C.TAINT_PARTITIONING)
        self._set_partition_state("failed" if errs else "applied", mode=target_c, memory=target_m, errors=errs)
        if errs:
            log.warning("partitioning %s to %s/%s: %s", self.node, target_c, target_m, errs)
        return not errs

    # ------------------------------------------------------------------ loop
    def step(self) -> None:
        self._in_step, self._pod_cache = True, None
        try:
            self._step()
        finally:
            self._in_step, self._pod_cache = False, None

    def _step(self) -> None:
        try:
            self.reconcile_partitions()
        except Exception as e:
            log.warning("partition reconcile failed: %s", e)
        self.publish()
        if self.probes is None:
            try:
                self.probe_fabric()
            except Exception as e:
                log.warning("fabric probe failed: %s", e)
        else:
            try:
                self.probes.note_pods()
            except Exception as e:
                log.warning("noting multi-GPU pods for set checks failed: %s", e)
        try:
            self.publish_caps()
        except Exception as e:
            log.warning("publishing partition capabilities failed: %s", e)
        samples = self.sample()
        try:
            self.check_health(samples)
        except Exception as e:
            log.warning("health check failed: %s", e)
        self._steps += 1
        if self._steps % self.history_every == 0:
            try:
                usage = self.pod_usage()
                if usage:
                    self.record_history(usage=usage)
                self.check_hbm(usage)
            except Exception as e:
                log.warning("per-pod usage / HBM check failed: %s", e)
        if self.profiles is not None:
            try:
                if self.client is not None:
                    self._node_pods()           # this step's pods: the ingestor's known UIDs
                self.profiles.step()
            except Exception as e:
                log.warning("ingesting per-pod profiles failed: %s", e)
            if self.corun is not None:
                try:
                    self.corun.step()
                except Exception as e:
                    log.warning("co-run observations failed: %s", e)
        try:
            self.track_busy()
        except Exception as e:
            log.warning("busy-ms pass failed: %s", e)

    def _pod_lookup(self, ns: str, name: str) -> Optional[Dict[str, Any]]:
        from ..kube.client import NotFound
        try:
            return self.client.get("pods", name, ns)
        except NotFound:
            return None

    def _running_on(self, uuid: str) -> set:
        """Keys of this node's non-terminal pods assigned to device `uuid`."""
        pods = self._node_pods()
        out = set()
        for p in pods:
            if O.is_terminal(p):
                continue
            if uuid in (O.annotations(p).get(C.ANNOT_DEVICES) or "").split(","):
                out.add(O.key(p))
        return out

    def _finished_on(self, uuid: str, span: Tuple[float, float]) -> set:
        """Keys of this node's terminal pods on device `uuid` whose containers ran during
        `span` (epoch s: another pod's container startedAt .. finishedAt)."""
        from ..plugins.gpu.feedback import container_span
        pods = self._node_pods()
        out = set()
        for p in pods:
            if not O.is_terminal(p) or uuid not in (O.annotations(p).get(C.ANNOT_DEVICES) or "").split(","):
                continue
            sp = container_span(p)
            if sp is not None and sp[1] > span[0] and sp[0] < span[1]:
                out.add(O.key(p))
        return out

    def run(self) -> None:
        if self.probes is not None:
            self.probes.start()
        while not self._stop.is_set():
            try:
                self.step()
            except Exception as e:      # Redis/apiserver blips: keep looping
                log.warning("agent step failed: %s", e)
            self._stop.wait(self.poll_s)

    def start(self) -> "NodeAgent":
        self.start_busy_sampler()
        self._thread = threading.Thread(target=self.run, daemon=True, name="node-agent")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self.probes is not None:
            self.probes.stop()
        if self._thread:
            self._thread.join(timeout=5)
        if self._busy_thread is not None:
            self._busy_thread.join(timeout=5)


def publish_from_stdin(lines: List[str], redis: Redis) -> str:
    """The reference's stdin protocol: NODE, POD, NS, "['uuid', ...]"
    (reference pkg/profiler/cmd/client/client.go:24-46, test.sh)."""
    node = lines[0].strip()
    raw = lines[3] if len(lines) > 3 else ""
    for ch in "'[] ":
        raw = raw.replace(ch, "")
    uuids = [u for u in raw.split(",") if u]
    return schema.publish_uuids(redis, node, uuids)
