"""DefaultPreemption (PostFilter) -- GPU-aware.

The reference runs inside upstream kube-scheduler, so its binary had kube-scheduler's default
PostFilter, DefaultPreemption (enabled by the v1beta1 defaults its config inherits,
reference deploy/scheduler.yaml:1-23).  Re-created here with the same shape:

1. a pod that no node can take, with `preemptionPolicy` != Never, looks for nodes where
   evicting pods of LOWER priority would make it fit;
2. per node, every lower-priority pod is removed in a what-if NodeInfo and the filters are
   re-run (the GPU plugin answers from a copy of the device ledger with the victims' CU units
   and HBM released); victims are then "reprieved" highest priority first while the pod still
   fits, leaving a minimal set;
3. the node is chosen by (lowest highest-victim priority, fewest victims, lowest sum of
   victim priorities, latest start of the highest-priority victim, name) -- upstream's order;
4. the pod gets `status.nominatedNodeName`, the victims are deleted (the deletes requeue the
   preemptor through the AssignedPodDelete event), and the cycle ends Unschedulable.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional, Tuple

from ..api import objects as O
from .cache import NodeInfo
from .interface import Code, CycleState, PostFilterPlugin, Status

log = logging.getLogger(__name__)
Obj = Dict[str, Any]


class WhatIfNodeInfo(NodeInfo):
    """A NodeInfo clone with some pods removed; `removed` names them for plugins whose state
    lives outside NodeInfo (the GPU plugin's ledger)."""
    __slots__ = ("removed",)

    @classmethod
    def without(cls, ni: NodeInfo, victims: List[Obj]) -> "WhatIfNodeInfo":
        w = cls()
        w.node, w._name = ni.node, ni._name
        w.pods, w.requested, w.allocatable = dict(ni.pods), dict(ni.requested), dict(ni.allocatable)
        w.non_zero = list(ni.non_zero)
        w.generation = ni.generation
        w.removed = set()
        for v in victims:
            w.remove_pod(v)
            w.removed.add(O.key(v))
        return w


def _start_time(pod: Obj) -> str:
    st = pod.get("status") or {}
    return st.get("startTime") or O.meta(pod).get("creationTimestamp") or ""


class DefaultPreemption(PostFilterPlugin):
    NAME = "DefaultPreemption"

    def __init__(self, args: Optional[Dict[str, Any]] = None, handle: Any = None):
        self.handle = handle
        self.args = args or {}

    def _fits(self, fw: Any, state: CycleState, pod: Obj, ni: NodeInfo) -> bool:
        return fw.run_filter(state, pod, ni).ok

    def select_victims(self, fw: Any, state: CycleState, pod: Obj, ni: NodeInfo) -> Optional[List[Obj]]:
        prio = O.priority(pod)
        lower = [p for p in ni.pods.values() if O.priority(p) < prio]
        if not lower:
            return None
        if not self._fits(fw, state, pod, WhatIfNodeInfo.without(ni, lower)):
            return None
        # reprieve: try to keep victims, most important first (higher priority, older)
        lower.sort(key=lambda p: (-O.priority(p), _start_time(p)))
        victims = list(lower)
        for p in lower:
            trial = [v for v in victims if v is not p]
            if self._fits(fw, state, pod, WhatIfNodeInfo.without(ni, trial)):
                victims = trial
        return victims

    def post_filter(self, state: CycleState, pod: Obj, filtered: Dict[str, Status]) -> Tuple[Optional[str], Status]:
        if (pod.get("spec") or {}).get("preemptionPolicy") == "Never":
            return None, Status(Code.UNSCHEDULABLE_AND_UNRESOLVABLE, ["preemption disabled by the pod"], self.NAME)
        fw = self.handle.framework_for(pod)
        snap = self.handle.snapshot()
        best: Optional[Tuple[Tuple, str, List[Obj]]] = None
        for name, st in filtered.items():
            if st.code == Code.UNSCHEDULABLE_AND_UNRESOLVABLE:
                continue
            ni = snap.get(name)
            if ni is None:
                continue
            victims = self.select_victims(fw, state, pod, ni)
            if not victims:
                continue
            prios = [O.priority(v) for v in victims]
            top = max(prios)
            newest_top = max(_start_time(v) for v in victims if O.priority(v) == top)
            key = (top, len(victims), sum(prios), tuple(-ord(c) for c in newest_top), name)
            if best is None or key < best[0]:
                best = (key, name, victims)
        if best is None:
            return None, Status.unschedulable("preemption: no node where evicting lower-priority pods helps",
                                              self.NAME)
        _, node, victims = best
        client = self.handle.client
        try:
            client.patch("pods", O.name(pod), {"status": {"nominatedNodeName": node}}, "merge", O.namespace(pod))
        except Exception as e:
            log.warning("preemption: nominating %s on %s failed: %s", O.key(pod), node, e)
        for v in victims:
            try:
                client.delete("pods", O.name(v), O.namespace(v), grace_period_seconds=0)
                self.handle.event(v, "Preempted", f"Preempted by {O.key(pod)} on node {node}", "Normal")
            except Exception as e:
                log.warning("preemption: deleting victim %s failed: %s", O.key(v), e)
        log.info("preemption: %s nominated on %s, %d victim(s)", O.key(pod), node, len(victims))
        return node, Status(Code.UNSCHEDULABLE, [f"preempting {len(victims)} pod(s) on {node}"], self.NAME)
