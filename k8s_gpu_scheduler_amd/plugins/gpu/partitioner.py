"""Scheduler-driven MI355X compute partitioning (the reference's MIG reconfigurer, made safe).

Reference behaviour (reference pkg/plugins/gpu_plugin/gpu_plugins.go:357-453,
478-496): on every Score of an A30 node, pick a MIG layout from the incoming pod's predicted
throughput per layout, relabel the node (`nvidia.com/mig.config`), delete the profiler pod
and busy-poll Redis every 2 s -- unbounded -- until the UUID list changes.  That runs inside
Score under a global mutex, on nodes that are "empty" by a check that compares a node name
to a pod name (§2.9 #2-#4).

Here the decision is a controller next to the GPU plugin, never inside Score:

  1. Pods that need a hard-isolated partition carry `gpu-scheduler.amd.com/isolation:
     partition`.  Their size is their `amd.com/gpu-cu` request, or -- for SLO-only pods --
     the controller sizes them from the recommender's predictions with the reference's
     intent ("most partitions whose predicted throughput still meets the SLO", i.e.
     `reconfigure_choice(fixed=True)` over the MI355X columns 1P/2P/4P/8P) and writes
     `gpu-scheduler.amd.com/partition-cus` on the pod.
  2. The GPU plugin's Filter admits such a pod only on a free partition of exactly its size,
     so without one it stays pending ("no free CPX partition").
  3. Each period the controller sums the pending demand per mode, subtracts the free
     partitions of that size (and partitions already requested on other nodes), and for
     the remaining deficit picks nodes that are IDLE in the ledger (no reserved/assumed
     pod on any device), not tainted, not already being changed, and whose probed
     capabilities (node annotation `partition-caps`, written by the agent) allow the mode;
     it sets `amd.com/compute-partition=<mode>` on them -- asynchronously, never blocking a
     scheduling cycle.  A busy node is never chosen.
  4. The node agent re-checks idleness on the device (amd-smi process list + pods bound to
     the node), taints `amd.com/partitioning=NoSchedule`, applies through amd-smi,
     republishes the UUIDs (64 on a CPX node) and untaints (agent.NodeAgent.reconcile_partitions);
     the scheduler re-reads the inventory on the node update and the pending pods bind.
  5. A request the agent refused or failed (node annotation `partition-state`, or a request
     of ours whose label came back reverted without the mode being applied -- e.g. the node
     was busy with GPU work the ledger cannot see) backs that node off for that mode for
     `backoff_s`, so an unledgered busy node is not tainted, drained and reverted in a loop.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from collections import Counter
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from ...api import constants as C
from ...api import objects as O

log = logging.getLogger(__name__)
Obj = Dict[str, Any]

MODES_BY_PARTS = sorted(C.COMPUTE_PARTITIONS.items(), key=lambda kv: kv[1])       # SPX .. CPX


def mode_for_cus(cus: int) -> str:
    return C.PARTITIONS_TO_MODE.get(max(1, C.MI355X_CUS // max(cus, 1)), "SPX")


def size_from_predictions(conf: Dict[str, float], slo: float, model: str = C.MI355X,
                          modes: Optional[List[str]] = None) -> Optional[int]:
    """CUs of the smallest partition whose predicted throughput still meets the SLO (the
    most partitions per GPU: more pods fit); none meets it -> the best-predicted size;
    no predictions -> None.  The fixed-mode form of the reference's MIG choice
    (gpu_plugins.go:365-399, whose satisfied branch goes negative -- SURVEY §2.9 #4)."""
    cand = []
    for mode, parts in MODES_BY_PARTS:
        if modes is not None and mode not in modes:
            continue
        v = conf.get(f"{parts}P_{model}")
        if v is not None:
            cand.append((parts, float(v)))
    if not cand:
        return None
    ok = [p for p, v in cand if slo > 0 and v >= slo]
    parts = max(ok) if ok else max(cand, key=lambda pv: pv[1])[0]
    return C.MI355X_CUS // parts


@dataclass
class Decision:
    node: str
    mode: str
    demand: int
    reason: str = ""
    ts: float = field(default_factory=time.time)


class PartitionController:
    def __init__(self, plugin: Any, period_s: float = 2.0, max_nodes_per_step: int = 4, backoff_s: float = 600.0):
        self.plugin = plugin
        self.period_s = period_s
        self.max_nodes_per_step = max_nodes_per_step
        self.backoff_s = backoff_s
        self.decisions: List[Decision] = []
        self._requested: Dict[str, Decision] = {}          # node -> our outstanding request
        self._backoff: Dict[Tuple[str, str], float] = {}    # (node, mode) -> until (wall clock)
        # partition sizes (CUs) whose pending demand no node can be re-partitioned for (every
        # node busy, changing, backed off or unable): SLO-sized pods of these sizes may then
        # take any larger free partition instead of waiting (plugin._whole_choice)
        self.stuck: set = set()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # ---------------------------------------------------------------- inputs
    @property
    def client(self):
        return self.plugin.handle.client

    def _pods(self) -> List[Obj]:
        try:
            return self.plugin.handle.informer_factory.pods().lister.list()
        except Exception:
            return self.client.list("pods")[0]

    def _nodes(self) -> List[Obj]:
        try:
            return self.plugin.handle.informer_factory.nodes().lister.list()
        except Exception:
            return self.client.list("nodes")[0]

    def pending_isolated(self) -> List[Obj]:
        """Pending pods of this scheduler that need an isolated partition: annotated
        `isolation: partition`, or SLO-only pods whose SLO no fractional share can meet
        (the GPU plugin's parse_request turns them into partition requests)."""
        ours = getattr(self.plugin.handle, "framework_for", None)
        out = []
        for p in self._pods():
            if O.node_name_of(p) or O.is_terminal(p):
                continue
            if not (ours(p) is not None if ours else O.scheduler_name(p) == C.SCHEDULER_NAME):
                continue
            if O.annotations(p).get(C.ANNOT_ISOLATION) == "partition" or self.plugin.parse_request(p).isolated:
                out.append(p)
        return out

    @staticmethod
    def node_caps(node: Obj):
        from ...agent.devices import PartitionCaps
        raw = O.annotations(node).get(C.ANNOT_PARTITION_CAPS)
        if not raw:
            return None
        try:
            return PartitionCaps.from_json(json.loads(raw))
        except (ValueError, TypeError):
            return None

    def current_mode(self, node: str) -> str:
        devs = self.plugin.ledger.devices(node)
        parts = max((st.device.partitions for st in devs), default=1)
        return C.PARTITIONS_TO_MODE.get(parts, "SPX")

    def node_idle(self, node: str) -> bool:
        return all(not st.pods for st in self.plugin.ledger.devices(node))

    # ---------------------------------------------------------------- backoff
    def _note_outcomes(self, nodes: Dict[str, Obj], now: float) -> None:
        """Back off (node, mode) pairs whose last request was refused or failed."""
        for name, node in nodes.items():
            raw = O.annotations(node).get(C.ANNOT_PARTITION_STATE)
            if not raw:
                continue
            try:
                st = json.loads(raw)
            except ValueError:
                continue
            if st.get("state") in ("refused", "failed") and st.get("mode"):
                until = float(st.get("ts", now)) + self.backoff_s
                key = (name, str(st["mode"]).upper())
                if until > now and until > self._backoff.get(key, 0.0):
                    self._backoff[key] = until
                    log.info("partitioning: %s -> %s %s (%s); backing off %.0fs", name, key[1], st["state"],
                             st.get("reason") or st.get("errors"), until - now)
        for name, d in list(self._requested.items()):
            node = nodes.get(name)
            if node is None:
                del self._requested[name]
                continue
            want = O.labels(node).get(C.LABEL_COMPUTE_PARTITION, "").upper()
            tainted = any(t.get("key") == C.TAINT_PARTITIONING for t in O.node_taints(node))
            if want == d.mode or tainted:
                if self.current_mode(name) == d.mode:
                    del self._requested[name]          # applied
                continue
            del self._requested[name]                  # label reverted, mode not applied: refused
            if self.current_mode(name) != d.mode:
                self._backoff[(name, d.mode)] = max(self._backoff.get((name, d.mode), 0.0), now + self.backoff_s)

    def backed_off(self, node: str, mode: str, now: Optional[float] = None) -> bool:
        return self._backoff.get((node, mode), 0.0) > (time.time() if now is None else now)

    # ---------------------------------------------------------------- decision
    def size_pod(self, pod: Obj) -> Optional[int]:
        """CUs of the partition a pending isolated pod needs (writes the annotation when the
        size came from predictions)."""
        _, cu, _ = O.gpu_request(pod)
        if cu > 0:
            from .plugin import partition_size
            return partition_size(cu)
        req = self.plugin.parse_request(pod)
        if req.isolated and req.part_cus and not O.annotations(pod).get(C.ANNOT_PARTITION_CUS):
            # an SLO-only pod the plugin sized from its predictions: record the size
            try:
                self.client.patch("pods", O.name(pod), {"metadata": {"annotations": {
                    C.ANNOT_PARTITION_CUS: str(req.part_cus)}}}, "merge", O.namespace(pod))
            except Exception as e:
                log.warning("annotating %s with its partition size failed: %s", O.key(pod), e)
            return req.part_cus
        ann = O.annotations(pod).get(C.ANNOT_PARTITION_CUS)
        if ann:
            try:
                return int(float(ann))
            except ValueError:
                pass
        conf, _ = self.plugin._pod_predictions(O.name(pod))
        size = size_from_predictions(conf or {}, O.pod_slo(pod), self.plugin.args.model)
        if size is None:
            return None
        try:
            self.client.patch("pods", O.name(pod), {"metadata": {"annotations": {C.ANNOT_PARTITION_CUS: str(size)}}},
                              "merge", O.namespace(pod))
        except Exception as e:
            log.warning("annotating %s with its partition size failed: %s", O.key(pod), e)
        return size

    def step(self) -> List[Decision]:
        pending = self.pending_isolated()
        if not pending:
            self.stuck = set()
            return []
        demand: Counter = Counter()
        for p in pending:
            size = self.size_pod(p)
            if size:
                demand[size] += 1
        if not demand:
            self.stuck = set()
            return []
        nodes = {O.name(n): n for n in self._nodes()}
        now = time.time()
        self._note_outcomes(nodes, now)
        ledger = self.plugin.ledger
        # supply per size: free partitions now + partitions of nodes already asked to switch
        supply: Counter = Counter()
        busy_or_changing = set()
        for name, node in nodes.items():
            want = O.labels(node).get(C.LABEL_COMPUTE_PARTITION, "").upper()
            cur = self.current_mode(name)
            changing = (want and want != cur) or any(t.get("key") == C.TAINT_PARTITIONING
                                                     for t in O.node_taints(node))
            if changing:
                busy_or_changing.add(name)
                if want in C.COMPUTE_PARTITIONS:
                    gpus = len({st.device.gpu for st in ledger.devices(name)}) or O.node_gpu_count(node)
                    supply[C.MI355X_CUS // C.COMPUTE_PARTITIONS[want]] += gpus * C.COMPUTE_PARTITIONS[want]
                continue
            for st in ledger.devices(name):
                if st.device.healthy and not st.pods:
                    supply[st.device.cus] += 1
        out: List[Decision] = []
        stuck = set()
        # largest deficit first; one node switches to one mode per step
        for size, need in sorted(demand.items(), key=lambda kv: kv[1] - supply[kv[0]], reverse=True):
            deficit = need - supply[size]
            mode = mode_for_cus(size)
            parts = C.COMPUTE_PARTITIONS[mode]
            while deficit > 0 and len(out) < self.max_nodes_per_step:
                cands = []
                for name, node in nodes.items():
                    if name in busy_or_changing or not self.node_idle(name):
                        continue                     # never a node with pods, never twice
                    if self.current_mode(name) == mode or not ledger.devices(name):
                        continue
                    if self.backed_off(name, mode, now):
                        continue                     # refused / failed recently for this mode
                    caps = self.node_caps(node)
                    if caps is not None and caps.check(mode) is not None:
                        continue
                    # prefer nodes whose current partitions nobody pending wants
                    cur_size = C.MI355X_CUS // C.COMPUTE_PARTITIONS[self.current_mode(name)]
                    cands.append((demand.get(cur_size, 0) > 0, name))
                if not cands:
                    stuck.add(size)
                    break
                cands.sort()
                name = cands[0][1]
                gpus = len({st.device.gpu for st in ledger.devices(name)})
                try:
                    self.client.patch("nodes", name, {"metadata": {"labels": {C.LABEL_COMPUTE_PARTITION: mode}}},
                                      "merge")
                except Exception as e:
                    log.warning("requesting %s on %s failed: %s", mode, name, e)
                    busy_or_changing.add(name)
                    continue
                d = Decision(name, mode, need, f"{need} pending pod(s) need {size}-CU partitions, "
                                                 f"{supply[size]} available")
                log.info("partitioning: %s -> %s (%s)", name, mode, d.reason)
                out.append(d)
                self._requested[name] = d
                busy_or_changing.add(name)
                supply[size] += gpus * parts
                deficit -= gpus * parts
        self.stuck = stuck
        self.decisions.extend(out)
        return out

    # ---------------------------------------------------------------- loop
    def run(self) -> None:
        while not self._stop.is_set():
            try:
                self.step()
            except Exception as e:
                log.warning("partition controller step failed: %s", e)
            self._stop.wait(self.period_s)

    def start(self) -> "PartitionController":
        if self._thread is None:
            self._thread = threading.Thread(target=self.run, daemon=True, name="partition-controller")
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
